#!/bin/bash
# dev: A/B of the packed plane kernel against dev builds that skip work (results
# invalid): gpurun -- bash tools/r5_dev.sh <tag>
set -o pipefail
tag=${1:-a}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/dev_$tag
mkdir -p $out
timeout -k 10 300 python -u tools/dct_ab.py "f64:dct_path=1" "pk16:dct_path=3" > $out/ab.log 2>&1 || { tail -20 $out/ab.log; exit 1; }
cat $out/ab.log
for v in ${DEVS:-1 16}; do
  HICCUP_HIP_LIB=$PWD/hiccup_amd/lib/libhiccup_hip_devpk$v.so timeout -k 10 200 python -u tools/dct_ab.py "dev$v:dct_path=3" \
    > $out/ab_dev$v.log 2>&1 || { tail -20 $out/ab_dev$v.log; exit 1; }
  cat $out/ab_dev$v.log
  HICCUP_HIP_LIB=$PWD/hiccup_amd/lib/libhiccup_hip_devpk$v.so timeout -k 10 200 python -u tools/enc_ab.py "dev$v:encode_pk=1" \
    > $out/enc_dev$v.log 2>&1 || { tail -20 $out/enc_dev$v.log; exit 1; }
  cat $out/enc_dev$v.log
done
timeout -k 10 200 python -u tools/enc_ab.py f64:encode_pk=0 pk:encode_pk=1 > $out/enc.log 2>&1 || { tail -20 $out/enc.log; exit 1; }
cat $out/enc.log
