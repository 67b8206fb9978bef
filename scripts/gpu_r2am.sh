# decode colour kernel: packed pyrUp + v_dot2 colour (new) vs the previous build
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 300 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "decode_colour or shard or jpeg_compression or 16k_roundtrip" > gpurun_out/am_pytest.log 2>&1
for i in 1 2; do
  HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devoldcol.so run 120 python -u tools/colour_dec_ab.py old >> gpurun_out/am_ab.log 2>&1
  run 120 python -u tools/colour_dec_ab.py new >> gpurun_out/am_ab.log 2>&1
done
