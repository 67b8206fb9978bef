#!/bin/bash
# dev: one GPU iteration = GPU tests + bench (+ env variants) + kernel stats
set -e -o pipefail
tag=${1:-iter}
shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $out/pytest.log 2>&1
tail -3 $out/pytest.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $out/bench.json 2>&1
tail -1 $out/bench.json
for v in "$@"; do
  env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline > $out/bench_$v.json 2>&1
  echo "$v: $(tail -1 $out/bench_$v.json | cut -c1-140)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_prof.log 2>&1
python3 - "$out" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + '/prof/run_kernel_stats.csv')):
    print(r['Name'][:70].ljust(70), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
