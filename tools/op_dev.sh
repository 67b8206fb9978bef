#!/bin/bash
# dev: one-pass kernel timing with parts compiled out (dev libraries: results invalid)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/op_dev
mkdir -p $out
for r in 1 2; do
  for v in prod noemit; do
    lib=""; [ $v != prod ] && lib="HICCUP_HIP_LIB=$GRAFT_REPO_ROOT/hiccup_amd/lib/libhiccup_hip_dev$v.so"
    for st in 1 4; do
      env $lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras --onepass --streams $st > $out/b_${v}_${st}_$r.json 2>&1 || { tail -5 $out/b_${v}_${st}_$r.json; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open('$out/b_${v}_${st}_$r.json') if l.startswith('{')][-1]); print('$v', 'streams $st', $r, d['ms_per_step'], d['roofline']['avg_launch_us'])"
    done
  done
done
