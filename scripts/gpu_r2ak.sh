# fused encoder workgroup size: 4 waves (one per SIMD) vs 1 or 2 waves per workgroup
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devwpb1.so run 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused and random" > gpurun_out/ak_pytest.log 2>&1
for i in 1 2; do
for v in "" wpb1 wpb2; do
  if [ -n "$v" ]; then L=hiccup_amd/lib/libhiccup_hip_dev$v.so; else L=hiccup_amd/lib/libhiccup_hip.so; fi
  HICCUP_HIP_LIB=$L run 200 python -u tools/enc_ab.py "wpb${v:-4}:" >> gpurun_out/ak_ab.log 2>&1
done
done
