#!/bin/bash
# dev: per-kernel A/B of env variants: GPU tests once (with the first variant),
# then for each variant a bench line and a kernel-trace profile.
# usage: tools/ab_prof.sh <tag> base HIC_X=1 "HIC_X=1 HIC_Y=2" ...
set -e -o pipefail
tag=${1:-ab}
shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $out/pytest.log 2>&1
  tail -2 $out/pytest.log
fi
i=0
for v in "$@"; do
  i=$((i+1))
  vars=""
  [ "$v" != base ] && vars="$v"
  ( [ -n "$vars" ] && export $vars
    timeout -k 10 300 python3 bench.py --no-cpu-baseline > $out/bench_$i.json 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$i -o run --output-format csv -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_prof_$i.log 2>&1 )
  echo "== $v: $(tail -1 $out/bench_$i.json | grep -o '"value": [0-9.e+]*, "unit": "[^"]*"\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
  python3 - "$out/prof_$i" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1] + '/run_kernel_stats.csv')):
    print('  ', r['Name'][:64].ljust(64), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
done
