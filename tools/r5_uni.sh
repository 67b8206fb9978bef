#!/bin/bash
# dev: the one-table batch dispatch: batch parity tests, then the plane A/B against
# the library before it (hiccup_amd/lib/libhiccup_hip_devold.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/uni_${1:-a}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "batch or records or full_size" > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/dct_ab.py "new:dct_path=1" > $out/new_$r.log 2>&1 || { tail -20 $out/new_$r.log; exit 1; }
  grep -v amdgpu.ids $out/new_$r.log
  HICCUP_HIP_LIB=$PWD/hiccup_amd/lib/libhiccup_hip_devold.so timeout -k 10 200 python -u tools/dct_ab.py "old:dct_path=1" \
    > $out/old_$r.log 2>&1 || { tail -20 $out/old_$r.log; exit 1; }
  grep -v amdgpu.ids $out/old_$r.log
done
