#!/bin/bash
# dev: where the fused DCT kernel's time goes.  FP issue rates (micro), then the
# bench's DCT launch time (kernel timestamps) under HIC_DCT_DBG knobs:
#   16 no DCT, 32 no RLE tile record, 64 no pixel loads, 128 no coefficient stores
# usage (GPU box): bash tools/dbg_dct.sh <tag> [knob ...]
set -e -o pipefail
tag=${1:-dbg}
shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
if [ -z "$NO_MICRO" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w tools/micro/fp64_rate.hip -o /tmp/fp_rate
  timeout -k 10 60 /tmp/fp_rate | tee $out/fp_rate.txt
fi
for v in 0 "$@"; do
  if [ "$v" = 0 ]; then unset HIC_DCT_DBG; else export HIC_DCT_DBG=$v; fi
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 40 > $out/bench_$v.json 2>&1
  echo "DBG=$v $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' $out/bench_$v.json | tr '\n' ' ')"
done
