#!/bin/bash
# dev: SQ counter passes (one rocprofv3 --pmc run each, kernel trace only) over
# the 8K luma DCT driver; summarise with tools/counters_table.py <dir>.
set -e -o pipefail
tag=${1:-dsq}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set -d $out/p$i -o run --output-format csv -- python3 tools/prof_dct.py 8 \
    > $out/p$i.log 2>&1
done
python3 tools/counters_table.py $out
