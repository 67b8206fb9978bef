#!/bin/bash
# dev: scan partition size A/B (HIC_SCAN_PK 1 = round-2 1024-record partitions,
# 8 = 8192-record partitions) on the default bench, alternating, + kernel traces.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3e
mkdir -p $o
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
for rep in 1 2 3; do
  for v in pk1 pk8; do
    HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > $o/bench_${v}_$rep.log 2>&1
    echo "$v $rep $(tail -1 $o/bench_${v}_$rep.log | cut -c90-200)"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in pk1 pk8; do
  HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof_$v -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-cpu-baseline > $GRAFT_REPO_ROOT/$o/prof_$v.log 2>&1
done
cd "$GRAFT_REPO_ROOT"
for v in pk1 pk8; do
python3 - "$o/prof_$v" <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(sys.argv[1][-3:], r['Name'][:50].ljust(50), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
done
echo done
