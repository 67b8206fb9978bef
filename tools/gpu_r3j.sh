#!/bin/bash
# dev: plane DCT register budget A/B (dev libs: base = 3 waves + prefetch, w4 = 4
# waves without prefetch + split odd phase, w4pf = 4 waves + prefetch, w3npf = 3
# waves without prefetch), float64 path, the bench's plane workloads.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3j
mkdir -p $o
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
HICCUP_HIP_LIB=$L/libhiccup_hip_devw4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest_transform_w4.log 2>&1
tail -1 $o/gputest_transform_w4.log
for rep in 1 2; do
  for v in base w4 w4pf w3npf; do
    HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so timeout -k 10 200 python tools/dct_pk_ab.py 1 > $o/dct_$v.log 2>&1
    echo "$v $(head -1 $o/dct_$v.log)"
  done
done
echo done
