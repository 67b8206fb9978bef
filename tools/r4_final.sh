#!/bin/bash
# dev: a round-4 checkpoint on the GPU box -- the GPU suite, smoke, the default
# bench line (gpurun -- bash tools/r4_final.sh <tag>)
set -o pipefail
tag=${1:-a}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/final_$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -3 $out/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
cat $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2>&1 || { tail -20 $out/bench_default.json; exit 1; }
grep '^{' $out/bench_default.json | tail -1 | cut -c1-1500
