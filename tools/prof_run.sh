#!/bin/bash
# dev: counters for both DCT variants
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in pair single; do
  HIC_DCT_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$v -o run --output-format csv -- python3 tools/prof_dct.py 16 > /dev/null 2>&1
  HIC_DCT_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pm_$v -o run --output-format csv -- python3 tools/prof_dct.py 4 > /dev/null 2>&1
done
echo done
