# A/B of nontemporal block stores in the RLE decode (HIC_RLD_NT=1) on the 16K round trip
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
HIC_RLD_NT=1 run 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_codec.py -k "16k or rle_decode or pipeline_encoder" > gpurun_out/rnt_pytest.log 2>&1
for r in a b c; do
  run 200 python -u -c "import torch, bench; torch.cuda.set_device(0); print(bench.extra_16k_roundtrip(8))" > gpurun_out/rnt0_$r.log 2>&1
  HIC_RLD_NT=1 run 200 python -u -c "import torch, bench; torch.cuda.set_device(0); print(bench.extra_16k_roundtrip(8))" > gpurun_out/rnt1_$r.log 2>&1
done
