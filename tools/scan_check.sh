#!/bin/bash
# dev: codec tests, then the 16K round trip and its kernel trace (the scan's share)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/scan
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec.py > $out/codec.log 2>&1 || { tail -30 $out/codec.log; exit 1; }
tail -1 $out/codec.log
timeout -k 10 200 python -u -c "import bench, json; print(json.dumps(bench.extra_16k_roundtrip()))" > $out/rt.log 2>&1 || { tail -5 $out/rt.log; exit 1; }
tail -1 $out/rt.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/tr -o run --output-format csv -- python3 tools/dec_ab.py 16384 > $out/tr.log 2>&1 || { tail -5 $out/tr.log; exit 1; }
python3 - <<PY
import csv
for r in csv.DictReader(open("$out/tr/run_kernel_stats.csv")):
    if "hic::" in r["Name"] and float(r["AverageNs"]) > 20000:
        print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
