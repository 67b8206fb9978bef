#!/bin/bash
# dev: images in flight with the 3-wave fused kernel: --streams 2 (default) vs 4 vs 1
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3p
mkdir -p $o
for rep in 1 2 3; do
  for v in 2 4 1; do
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --streams $v > $o/bench.log 2>&1
    echo "s$v $rep $(tail -1 $o/bench.log | cut -c90-200)" | tee -a $o/ab.txt
  done
done
echo done
