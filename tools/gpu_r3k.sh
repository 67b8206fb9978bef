#!/bin/bash
# dev: plane DCT prefetch / grid A/B (dev libs pf1 = round-2 prefetch, pf0 = the new
# default, pkpf0 = packed path without its prefetch), transform GPU tests first.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3k
mkdir -p $o
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_transform.py tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/gputest.log 2>&1
tail -1 $o/gputest.log
for rep in 1 2; do
  for v in "pf1:1:" "pf0:1:" "pf0:1:dct_waves_per_cu=0" "pf0:1:dct_waves_per_cu=16" "pf0:4:" "pkpf0:4:"; do
    IFS=: read lib path kn <<< "$v"
    AB_KNOBS=$kn HICCUP_HIP_LIB=$L/libhiccup_hip_dev$lib.so timeout -k 10 200 python tools/dct_pk_ab.py $path > $o/dct.log 2>&1
    echo "$v $(grep path $o/dct.log | head -1)"
  done
done
echo done
