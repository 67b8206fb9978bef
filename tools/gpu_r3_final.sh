#!/bin/bash
# dev: round-3 GPU pass: the GPU test suite, the default bench line, the default
# bench command (no extras) under a kernel trace (its isolated phase is what the
# line's roofline times: tools/trace_phases.py), then the round's profiles
# (tools/prof_r2.sh: one-stream kernel trace + calibrated PMC + SQ).
#   gpurun -- bash tools/gpu_r3_final.sh <tag>
set -e -o pipefail
tag=${1:-r03}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gputest.log 2>&1
timeout -k 10 500 python bench.py > gpurun_out/${tag}_bench.log 2>&1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
  -d "$GRAFT_REPO_ROOT/gpurun_out/${tag}_default_trace" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-extras --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_default_trace.log" 2>&1)
bash tools/prof_r2.sh $tag
echo done
