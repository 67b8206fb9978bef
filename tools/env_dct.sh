#!/bin/bash
# dev: the bench's DCT launch time (kernel timestamps) under environment variants
# usage (GPU box): bash tools/env_dct.sh <tag> "VAR=x VAR2=y" ...   ("base" = no vars)
set -e -o pipefail
tag=${1:-env}
shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
i=0
for v in "$@"; do
  i=$((i+1))
  vars=""
  [ "$v" != base ] && vars="$v"
  ( [ -n "$vars" ] && export $vars
    timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 40 > $out/bench_$i.json 2>&1 )
  echo "$v: $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' $out/bench_$i.json | tr '\n' ' ')"
done
