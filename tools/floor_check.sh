#!/bin/bash
# dev: the in-run memory floors (bench.measure_floors) and one default bench line without extras
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/floor
mkdir -p $out
timeout -k 10 200 python -u -c "
import bench, json
f = bench.measure_floors()
print(json.dumps(f['encode420_pattern']), json.dumps(f['luma_pattern']['1x']))
" > $out/floor.log 2>&1 || { tail -5 $out/floor.log; exit 1; }
tail -1 $out/floor.log
timeout -k 10 300 python -u bench.py --no-extras > $out/bench.json 2>&1 || { tail -5 $out/bench.json; exit 1; }
grep '^{' $out/bench.json | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['roofline']))"
