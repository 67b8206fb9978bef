#!/bin/bash
# dev: one-stream kernel traces of 16K and 8K encodes, the tree's library vs libhiccup_hip_devold.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/scan_ab
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 16384 8192; do
  for v in new old; do
    lib=$GRAFT_REPO_ROOT/hiccup_amd/lib/libhiccup_hip.so; [ $v = old ] && lib=$GRAFT_REPO_ROOT/hiccup_amd/lib/libhiccup_hip_devold.so
    HICCUP_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/tr_${v}_$n -o run --output-format csv -- python3 tools/enc16k.py $n > $out/tr_${v}_$n.log 2>&1 || { tail -5 $out/tr_${v}_$n.log; exit 1; }
    python3 - <<PY
import csv
for r in csv.DictReader(open("$out/tr_${v}_$n/run_kernel_stats.csv")):
    if "k_rle" in r["Name"] or "k_encode" in r["Name"]:
        print("$v $n", r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
  done
done
