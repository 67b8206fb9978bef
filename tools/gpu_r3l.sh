#!/bin/bash
# dev: plane DCT at 4 waves per SIMD with its cold paths out of line (w4cc), the
# same at 3 waves (w3cc), against the product (base); float64 path.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3l
mkdir -p $o
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
HICCUP_HIP_LIB=$L/libhiccup_hip_devw4cc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest_transform_w4cc.log 2>&1
tail -1 $o/gputest_transform_w4cc.log
for rep in 1 2; do
  for v in base w4cc w3cc; do
    HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so timeout -k 10 200 python tools/dct_pk_ab.py 1 > $o/dct.log 2>&1
    echo "$v $(grep path $o/dct.log | head -1)" | tee -a $o/ab.txt
  done
done
echo done
