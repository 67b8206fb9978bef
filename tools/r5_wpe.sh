#!/bin/bash
# dev: the 16K decode (fused RGB form) with the decode kernels at 4 waves per SIMD
# (product, 128 VGPRs, ~10 spilled) against 3 (hiccup_amd/lib/libhiccup_hip_devwpe3.so,
# 138 VGPRs, no spills), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/wpe_${1:-a}
mkdir -p $out
for r in 1 2 3; do
  for l in new wpe3; do
    so=$PWD/hiccup_amd/lib/libhiccup_hip.so
    [ $l = wpe3 ] && so=$PWD/hiccup_amd/lib/libhiccup_hip_devwpe3.so
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
