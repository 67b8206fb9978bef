#!/bin/bash
# dev: fused-encoder unit order (knob encode_order 0 row-major / 1 vertical stacks):
# (args: output tag, then the orders; 2 / 3: the same XCD-major)
# bench default line alternating, then FETCH_SIZE / WRITE_SIZE passes of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=${1:-order_ab}; shift
ORDERS=${*:-0 1}
out=gpurun_out/r4/$tag
mkdir -p $out
for r in $(seq ${REPS:-3}); do
  for o in $ORDERS; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras --knob encode_order=$o > $out/b_${o}_$r.json 2>&1 || { tail -5 $out/b_${o}_$r.json; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$out/b_${o}_$r.json') if l.startswith('{')][-1]); print('order $o', $r, d['value'], d['ms_per_step'], d.get('ms_per_step_p50'), d['roofline']['avg_launch_us'])"
  done
done
[ -n "$NOPMC" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for o in $ORDERS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pmc_${o}_$c -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras --streams 1 --knob encode_order=$o > $out/pmc_${o}_$c.log 2>&1 || { tail -5 $out/pmc_${o}_$c.log; exit 1; }
    python3 - <<PY
import csv, statistics
rows = [r for r in csv.DictReader(open("$out/pmc_${o}_$c/run_counter_collection.csv")) if "k_encode420" in r["Kernel_Name"]]
vals = [float(r["Counter_Value"]) for r in rows]
print("order $o $c", len(vals), statistics.median(vals) if vals else None)
PY
  done
done
