#!/bin/bash
# dev: A/B of dev library variants on the default bench (alternating, 3 reps) +
# one kernel trace each.  usage: gpu_ab_libs.sh <tag> <variant>... (libhiccup_hip_dev<variant>.so)
# GPU tests of the product library first.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
o=gpurun_out/$tag
mkdir -p $o
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1
  tail -1 $o/gputest.log
fi
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
for rep in 1 2 3; do
  for v in "$@"; do
    HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > $o/bench_${v}_$rep.log 2>&1
    echo "$v $rep $(tail -1 $o/bench_${v}_$rep.log | cut -c90-200)"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$o/prof_$v -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-cpu-baseline > $GRAFT_REPO_ROOT/$o/prof_$v.log 2>&1
done
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
python3 - "$o/prof_$v" "$v" <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_rle' in r['Name'] or 'k_encode' in r['Name']:
        print(sys.argv[2], r['Name'][:50].ljust(50), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
done
echo done
