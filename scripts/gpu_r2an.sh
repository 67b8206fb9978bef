# dequant + IDCT: persistent LDS-DMA prefetching zig-zag kernel vs the previous build
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/ -k "idct or inv_dct or decode or roundtrip or jpeg" > gpurun_out/an_pytest.log 2>&1
for i in 1 2; do
  HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devoldidct.so run 120 python -u tools/idct_ab.py old >> gpurun_out/an_ab.log 2>&1
  run 120 python -u tools/idct_ab.py new >> gpurun_out/an_ab.log 2>&1
done
