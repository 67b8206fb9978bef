#!/bin/bash
# dev: round-3 GPU pass: the GPU test suite, the default bench line, then the
# round's profiles (tools/prof_r2.sh: kernel trace + calibrated PMC + SQ).
#   gpurun -- bash tools/gpu_r3_final.sh <tag>
set -e -o pipefail
tag=${1:-r03}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gputest.log 2>&1
timeout -k 10 500 python bench.py > gpurun_out/${tag}_bench.log 2>&1
bash tools/prof_r2.sh $tag
echo done
