#!/bin/bash
# dev: one-pass encode vs the chain (fused transform + scan + emit), the bench's
# default 8K line alternating arms on one box; then a kernel trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/op_ab
mkdir -p $out
for r in 1 2 3; do
  for arm in onepass chain; do
    flag=""; [ $arm = onepass ] && flag="--onepass"
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras $flag > $out/b_${arm}_$r.json 2>&1 || { tail -5 $out/b_${arm}_$r.json; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$out/b_${arm}_$r.json') if l.startswith('{')][-1]); print('$arm', $r, d['value'], d['ms_per_step'], d.get('ms_per_step_p10'), d.get('ms_per_step_p50'), d['roofline']['avg_launch_us'], d['roofline']['kernel'][:40])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for arm in onepass chain; do
  flag=""; [ $arm = onepass ] && flag="--onepass"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/tr_$arm -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --streams 1 $flag > $out/tr_$arm.log 2>&1 || { tail -5 $out/tr_$arm.log; exit 1; }
  python3 - <<PY
import csv
rows = list(csv.DictReader(open("$out/tr_$arm/run_kernel_stats.csv")))
for r in rows:
    if "hic::" in r["Name"]:
        print("$arm", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
