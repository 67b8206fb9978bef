#!/bin/bash
# dev: fused encoder, 3 waves per SIMD with the colour rows first (encode_waves=3)
# vs the default 2-wave kernel: launch A/B, fused-vs-chain tests of the variants.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3h
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused_encoder" > $o/gputest_fused.log 2>&1
tail -1 $o/gputest_fused.log
timeout -k 10 200 python tools/enc_ab.py "w2:" "w3:encode_waves=3" "w2:" "w3:encode_waves=3" "w3pk:encode_waves=3,encode_dct=2" > $o/enc_ab.log 2>&1
cat $o/enc_ab.log
for v in "" "--knob encode_waves=3" "" "--knob encode_waves=3"; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline $v > $o/bench.log 2>&1
  echo "$v $(tail -1 $o/bench.log | cut -c90-200)"
done
echo done
