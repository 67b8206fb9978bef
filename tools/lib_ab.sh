#!/bin/bash
# dev: the default bench line, this tree's library against hiccup_amd/lib/libhiccup_hip_devold.so
# (the same tree with one file at its previous commit), alternating, then a one-stream trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
v2=${1:-old}
out=gpurun_out/r4/lib_ab_$v2
mkdir -p $out
for r in $(seq ${REPS:-3}); do
  for v in new old; do
    lib=""; [ $v = old ] && lib="HICCUP_HIP_LIB=$GRAFT_REPO_ROOT/hiccup_amd/lib/libhiccup_hip_dev$v2.so"
    env $lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras > $out/b_${v}_$r.json 2>&1 || { tail -5 $out/b_${v}_$r.json; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$out/b_${v}_$r.json') if l.startswith('{')][-1]); print('$v', $r, d['value'], d['ms_per_step'], d['ms_per_step_p50'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in new old; do
  lib=""; [ $v = old ] && lib="$GRAFT_REPO_ROOT/hiccup_amd/lib/libhiccup_hip_dev$v2.so"
  HICCUP_HIP_LIB=${lib:-$GRAFT_REPO_ROOT/hiccup_amd/lib/libhiccup_hip.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/tr_$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --streams 1 > $out/tr_$v.log 2>&1 || { tail -5 $out/tr_$v.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$out/tr_$v/run_kernel_stats.csv")):
    if "k_rle" in r["Name"] or "k_encode" in r["Name"]:
        print("$v", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
