#!/bin/bash
# dev: plane DCT paths (packed with the workgroup-merged final flush vs float64),
# the packed plane-DCT tests, bench with producer / consumer streams vs alternating.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3d
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1
tail -1 $o/gputest.log
timeout -k 10 200 python tools/dct_pk_ab.py 4 1 > $o/dct_ab.log 2>&1
cat $o/dct_ab.log
for v in "" "--split" "" "--split"; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline $v > $o/bench_$v.log 2>&1
  echo "$v $(tail -1 $o/bench_$v.log | cut -c90-200)"
done
echo done
