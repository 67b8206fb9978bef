#!/bin/bash
# dev: with the 3-wave kernel and 4 streams: nontemporal coefficient stores (knob
# encode_nt=1) vs cached; the 4K RGB extra on 2 vs 4 streams.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3q
mkdir -p $o
for rep in 1 2 3; do
  for v in "" "--knob encode_nt=1"; do
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline $v > $o/bench.log 2>&1
    echo "[$v] $rep $(tail -1 $o/bench.log | cut -c90-200)" | tee -a $o/ab.txt
  done
done
for rep in 1 2; do
  for n in 2 4; do
    timeout -k 10 200 python -c "
import bench, json, torch
torch.cuda.set_device(0)
print(json.dumps(bench.extra_4k_rgb_encode(n_streams=$n)))" > $o/x4k.log 2>&1
    echo "4k streams $n $rep $(tail -1 $o/x4k.log | cut -c1-220)" | tee -a $o/ab.txt
  done
done
echo done
