# encode-side colour walk kernel: dot4 colour + packed pyrDown (new) vs the previous build
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/ -k "colour or color or shard or unfused or jpeg_compression or pyr" > gpurun_out/aq_pytest.log 2>&1
for i in 1 2; do
  HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devoldcol.so run 120 python -u tools/colour_enc_ab.py old >> gpurun_out/aq_ab.log 2>&1
  run 120 python -u tools/colour_enc_ab.py new >> gpurun_out/aq_ab.log 2>&1
done
