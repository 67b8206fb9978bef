#!/bin/bash
# dev: plane DCT, the tree's library against hiccup_amd/lib/libhiccup_hip_dev$1.so, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
v=${1:-pf2}
out=gpurun_out/r4/dct_$v
mkdir -p $out
for r in 1 2 3; do
  for lib in libhiccup_hip.so libhiccup_hip_dev$v.so; do
    HICCUP_HIP_LIB=$GRAFT_REPO_ROOT/hiccup_amd/lib/$lib timeout -k 10 200 python -u tools/dct_ab.py >> $out/ab.log 2>&1 || { tail -5 $out/ab.log; exit 1; }
  done
done
grep "us" $out/ab.log
