# dev A/B of the forward DCT launch across dev library builds
set -u
for L in dev dev2; do
  echo "== $L" >> gpurun_out/ab.log
  HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_$L.so timeout -k 10 300 python -u tools/dct_ab.py "$@" >> gpurun_out/ab.log 2>&1; echo rc=$?
done
