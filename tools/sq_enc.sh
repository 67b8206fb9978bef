#!/bin/bash
# dev: SQ instruction / stall counters of the fused encoder per DCT variant
# usage (GPU box): bash tools/sq_enc.sh <tag> "label:knob=v" ...
set -e -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for spec in "$@"; do
  lab=${spec%%:*}
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    -d $out/$lab -o run --output-format csv -- python3 tools/enc_ab.py "$spec" > $out/$lab.log 2>&1
  f=$(find $out/$lab -name '*counter_collection.csv' | head -1)
  echo "== $spec"; python3 tools/pmc_kernel.py "$f" k_encode420
done
