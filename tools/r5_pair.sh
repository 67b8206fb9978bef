#!/bin/bash
# dev: decode tests, then the 16K decode with Cr + Cb in one launch (pair) against
# one launch each, alternating (same library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/pair_${1:-a}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "indexed or 16k or decode or roundtrip" > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
for r in 1 2 3; do
  for p in 1 0; do
    d=$out/pair${p}_$r
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 tools/prof_dec.py 16384 6 0 0 $p > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    echo "pair=$p r$r: $(grep -o 'median [0-9.]* ms' $d.log)"
    python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rld' in r['Name']:  # noqa
        print('    ', r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
  done
done
