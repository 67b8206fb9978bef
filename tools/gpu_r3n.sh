#!/bin/bash
# dev: 3-wave fused kernel with the lane recomputed (no lane spills): fused tests,
# 3 alternating bench pairs (encode_waves 3 vs 2), then the profile pass (trace +
# calibrated PMC + SQ) of the default.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3n
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused_encoder" > $o/gputest_fused.log 2>&1
tail -1 $o/gputest_fused.log
timeout -k 10 200 python tools/enc_ab.py "w3:" "w2:encode_waves=2" "w3:" "w2:encode_waves=2" > $o/enc_ab.log 2>&1
cat $o/enc_ab.log
for rep in 1 2 3; do
  for v in 3 2; do
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --knob encode_waves=$v > $o/bench.log 2>&1
    echo "w$v $rep $(tail -1 $o/bench.log | cut -c90-200)" | tee -a $o/ab.txt
  done
done
bash tools/prof_r2.sh r3n
echo done
