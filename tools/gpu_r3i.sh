#!/bin/bash
# dev: 3-wave fused encoder (colour rows first, packed Y rows pinned) vs the 2-wave
# default; dev libs la3 / la6 = the 3-wave variant's row lookahead.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3i
mkdir -p $o
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
HICCUP_HIP_LIB=$L/libhiccup_hip_devla6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused_encoder" > $o/gputest_fused_la6.log 2>&1
tail -1 $o/gputest_fused_la6.log
for v in la3 la6; do
  HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so timeout -k 10 200 python tools/enc_ab.py "w2:" "w3:encode_waves=3" "w2:" "w3:encode_waves=3" > $o/enc_ab_$v.log 2>&1
  cat $o/enc_ab_$v.log
done
for rep in 1 2; do
  for v in "la6:" "la6:--knob encode_waves=3" "la3:--knob encode_waves=3"; do
    lib=${v%%:*}; k=${v#*:}
    HICCUP_HIP_LIB=$L/libhiccup_hip_dev$lib.so timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline $k > $o/bench.log 2>&1
    echo "$v $(tail -1 $o/bench.log | cut -c90-200)"
  done
done
echo done
