#!/bin/bash
# dev: kernel trace + SQ counter passes (one rocprofv3 --pmc run each) over the 8K
# luma pass on dct_path $2; summary by tools/counters_table.py
set -e -o pipefail
tag=${1:-lsq}
path=${2:-5}
np=${3:-1}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/prof_luma.py 16 $path $np > $out/trace.log 2>&1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d $out/p$i -o run --output-format csv -- python3 tools/prof_luma.py 8 $path $np \
    > $out/p$i.log 2>&1
done
python3 tools/counters_table.py $out
