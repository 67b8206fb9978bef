#!/bin/bash
# dev: the branch-free indexed gather (rle_core.h gather_tile): decode parity tests,
# then the 16K decode per library (old = the library before it; g8 / g4 = group
# sizes) under a kernel trace, fused and keep_blocks.
# usage: gpurun -- bash tools/r5_gath.sh <tag> "old new g8 g4"
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/gath_${1:-a}
libs=${2:-"old new g8 g4"}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "indexed or 16k or stitch or decode or roundtrip" > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
for r in 1 2; do
  for l in $libs; do
    so=$PWD/hiccup_amd/lib/libhiccup_hip.so
    [ $l != new ] && so=$PWD/hiccup_amd/lib/libhiccup_hip_dev$l.so
    modes="0:1 1:1"  # keep_blocks:planes
    [ $l = new ] && modes="0:0 0:1 1:1"
    for m in $modes; do
      keep=${m%:*}; pl=${m#*:}
      d=$out/${l}_k${keep}p${pl}_$r
      HICCUP_HIP_LIB=$so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
        python3 tools/prof_dec.py 16384 6 $keep $pl > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
      echo "$l r$r: $(grep median $d.log)"
      python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rld' in r['Name'] or 'dequant' in r['Name'] or 'ycrcb' in r['Name']:  # noqa
        print('    ', r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
    done
  done
done
