#!/bin/bash
# dev: the round-5 final pass on the GPU box (gpurun -- bash tools/r5_final.sh <tag> [noprof]):
# the GPU suite, smoke, the default bench line (extras included); then the profiles:
# a kernel trace of the default bench command (every extra's launches in order:
# tools/trace_launches.py), the one-stream 8K bench trace + calibrated
# FETCH_SIZE / WRITE_SIZE + SQ pass (tools/prof_r2.sh), and SQ passes of the
# 16-plane 8K luma launch per dct path (tools/r5_sq.sh)
set -o pipefail
tag=${1:-a}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/final_$tag
mkdir -p $out
if [ "${2:-}" != "profonly" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -3 $out/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
grep -v amdgpu.ids $out/smoke.log
timeout -k 10 500 python -u bench.py > $out/bench_default.json 2>&1 || { tail -20 $out/bench_default.json; exit 1; }
grep '^{' $out/bench_default.json | tail -1 | cut -c1-400
fi
[ "${2:-}" = "noprof" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ "${2:-}" = "profonly" ] || timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace_default -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline > $out/trace_default.json.log 2>&1 || { tail -5 $out/trace_default.json.log; exit 1; }
[ "${2:-}" = "profonly" ] || { python3 tools/trace_launches.py $out/trace_default/run_kernel_trace.csv k_dct \
  > $out/trace_default_dct_launches.txt; head -c 3000 $out/trace_default_dct_launches.txt; }
[ "${2:-}" = "trace" ] && exit 0
timeout -k 10 900 bash tools/prof_r2.sh r5_$tag > $out/prof_r2.log 2>&1 || { tail -5 $out/prof_r2.log; exit 1; }
python3 tools/prof_r2_summary.py gpurun_out/prof_r5_$tag $out/prof_summary.json && echo profiled
timeout -k 10 600 bash tools/r5_sq.sh $tag "1" > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 1; }
cat $out/sq.log
