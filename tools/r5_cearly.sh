#!/bin/bash
# dev: decode tests, then the 16K decode (fused RGB form) with the chroma rows
# loaded before the IDCT (product) against after it (libhiccup_hip_devclate.so),
# alternating
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 300 --timeout-method thread -k "indexed or 16k or decode or roundtrip" > gpurun_out/cearly_tests.log 2>&1 || { tail -30 gpurun_out/cearly_tests.log; exit 1; }
tail -1 gpurun_out/cearly_tests.log
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/cearly_${1:-a}
mkdir -p $out
for r in 1 2 3; do
  for l in new clate; do
    so=$PWD/hiccup_amd/lib/libhiccup_hip.so
    [ $l = clate ] && so=$PWD/hiccup_amd/lib/libhiccup_hip_devclate.so
    d=$out/${l}_$r
    HICCUP_HIP_LIB=$so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 tools/prof_dec.py 16384 6 0 0 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    echo "$l r$r: $(grep -o 'median [0-9.]* ms' $d.log)"
    python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rld' in r['Name']:  # noqa
        print('    ', r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
  done
done
