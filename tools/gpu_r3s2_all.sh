#!/bin/bash
# dev: one call (the pool is congested): the final pass (tools/gpu_r3s2_final.sh:
# GPU tests, smoke, bench, N = 2 rehearsal, traces, PMC), then the plane DCT
# prefetch / grid A/B of the dev libs.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r3s2_final.sh r03s2
o=gpurun_out/r3k
mkdir -p $o
L=$GRAFT_REPO_ROOT/hiccup_amd/lib
for rep in 1 2; do
  for v in "pf1:1:" "pf0:1:" "pf0:1:dct_waves_per_cu=0" "pf0:1:dct_waves_per_cu=16" "pf0:4:" "pkpf0:4:"; do
    IFS=: read lib path kn <<< "$v"
    AB_KNOBS=$kn HICCUP_HIP_LIB=$L/libhiccup_hip_dev$lib.so timeout -k 10 200 python tools/dct_pk_ab.py $path > $o/dct.log 2>&1
    echo "$v $(grep path $o/dct.log | head -1)" | tee -a $o/ab.txt
  done
done
echo alldone
