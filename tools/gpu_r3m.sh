#!/bin/bash
# dev: fused encoder 2 vs 3 waves per SIMD on the default bench (product library,
# knob encode_waves), 5 alternating pairs.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3m
mkdir -p $o
for rep in 1 2 3 4 5; do
  for v in 2 3; do
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --knob encode_waves=$v > $o/bench.log 2>&1
    echo "w$v $rep $(tail -1 $o/bench.log | cut -c90-200)" | tee -a $o/ab.txt
  done
done
echo done
