# colour split around the first Y DCT: A/B against the unsplit order and lookahead 4 / 8; fused parity
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused or pipeline_encoder or shards" > gpurun_out/s_pytest.log 2>&1
for v in "" s19 la4 la8 nodct "" s19; do
  if [ -n "$v" ]; then L=hiccup_amd/lib/libhiccup_hip_dev$v.so; else L=hiccup_amd/lib/libhiccup_hip.so; fi
  HICCUP_HIP_LIB=$L run 200 python -u tools/enc_ab.py "w2:" "w2b:" >> gpurun_out/s_ab.log 2>&1
done
