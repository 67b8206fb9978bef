#!/bin/bash
# dev: decode A/B, libraries alternating (new = the tree's, old = hiccup_amd/lib/libhiccup_hip_devold.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/dec_ab_${1:-x}
mkdir -p $out
for r in 1 2; do
  for v in new old; do
    lib=""; [ $v = old ] && lib="HICCUP_HIP_LIB=$GRAFT_REPO_ROOT/hiccup_amd/lib/libhiccup_hip_devold.so"
    env $lib timeout -k 10 200 python -u tools/dec_ab.py > $out/${v}_$r.log 2>&1 || { tail -5 $out/${v}_$r.log; exit 1; }
    grep '^{' $out/${v}_$r.log
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/tr_new -o run --output-format csv -- python3 tools/dec_ab.py 16384 > $out/tr_new.log 2>&1 || { tail -5 $out/tr_new.log; exit 1; }
python3 - <<PY
import csv
for r in csv.DictReader(open("$out/tr_new/run_kernel_stats.csv")):
    if "hic::" in r["Name"]:
        print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
