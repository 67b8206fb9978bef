#!/bin/bash
# dev: A/B of environment variants of the bench's DCT launch, interleaved over
# repetitions (box-to-box noise cancels).  usage: tools/ab_env.sh <tag> <reps> base "VAR=x" ...
set -e -o pipefail
tag=${1:-ab}; reps=${2:-3}
shift 2 || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq 1 $reps); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    vars=""
    [ "$v" != base ] && vars="$v"
    ( [ -n "$vars" ] && export $vars
      timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 40 > $out/b_${r}_$i.json 2>&1 )
    echo "$r [$v] $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' $out/b_${r}_$i.json | tr '\n' ' ')"
  done
done
