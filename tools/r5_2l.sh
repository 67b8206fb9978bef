#!/bin/bash
# dev: the two-lanes-per-block kernel (dct_path 4) on the GPU box: its parity tests,
# then the plane-kernel A/B against the one-lane float64 kernel, grid sizes swept
set -o pipefail
tag=${1:-a}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/2l_$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${2:-full_size or structured or records_free or sixteen or three_planes}" > $out/gputest.log 2>&1 \
  || { tail -40 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
timeout -k 10 500 python -u tools/dct_ab.py -r 2 "f64:dct_path=1" "2l:dct_path=4" "2l16:dct_path=4,dct_waves_per_cu=16" \
  "2l0:dct_path=4,dct_waves_per_cu=0" > $out/dct_ab.log 2>&1 || { tail -20 $out/dct_ab.log; exit 1; }
grep -v amdgpu.ids $out/dct_ab.log
