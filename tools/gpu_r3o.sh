#!/bin/bash
# dev: RLE emit tile order (rev = last tiles first, the encoder's latest stores)
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
mkdir -p gpurun_out/r3o
HICCUP_HIP_LIB=$L/libhiccup_hip_devrev.so timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3o/gputest_codec_rev.log 2>&1
tail -1 gpurun_out/r3o/gputest_codec_rev.log
SKIP_TESTS=1 bash tools/gpu_ab_libs.sh r3o fwd rev
