#!/bin/bash
# dev: round-5 check on the GPU box (gpurun -- bash tools/r5_check.sh <tag> [tests-filter]):
# the GPU suite (or a -k filter), smoke, the default bench line (extras included)
set -o pipefail
tag=${1:-a}
filt=${2:-}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/check_$tag
mkdir -p $out
if [ -n "$filt" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$filt" \
    > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
fi
tail -3 $out/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
cat $out/smoke.log
[ "${3:-}" = "nobench" ] && exit 0
timeout -k 10 500 python -u bench.py > $out/bench_default.json 2>&1 || { tail -20 $out/bench_default.json; exit 1; }
grep '^{' $out/bench_default.json | tail -1 | cut -c1-400
