#!/bin/bash
# dev: the round-4 final pass on the GPU box (gpurun -- bash tools/r4_final.sh <tag>):
# the GPU suite, smoke, the default bench line (extras included), then the
# profiles: kernel trace of the 8K bench on one stream and with the default 4,
# calibrated FETCH_SIZE / WRITE_SIZE passes and one SQ pass (tools/prof_r2.sh)
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
timeout -k 10 500 python -u bench.py > $out/bench_default.json 2>&1 || { tail -20 $out/bench_default.json; exit 1; }
grep '^{' $out/bench_default.json | tail -1 | cut -c1-600
[ "${2:-}" = "noprof" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace4 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $out/trace4.json.log 2>&1 || { tail -5 $out/trace4.json.log; exit 1; }
timeout -k 10 900 bash tools/prof_r2.sh r4_$tag > $out/prof_r2.log 2>&1 || { tail -5 $out/prof_r2.log; exit 1; }
python3 tools/prof_r2_summary.py gpurun_out/prof_r4_$tag $out/prof_summary.json && echo profiled
