#!/bin/bash
# dev: the 16K decode (fused indexed decode-IDCT, and keep_blocks = indexed decode
# + IDCT) under a kernel trace, then two SQ counter passes of the fused form.
# usage: gpurun -- bash tools/r5_dec.sh <tag>
set -o pipefail
tag=${1:-a}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/dec_$tag
mkdir -p $out
for keep in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/trace$keep -o run --output-format csv -- \
    python3 tools/prof_dec.py 16384 4 $keep > $out/trace$keep.log 2>&1 || { tail -5 $out/trace$keep.log; exit 1; }
  tail -1 $out/trace$keep.log
  python3 - $out/trace$keep/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print('  ', r['Name'][:64].ljust(64), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
done
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_IFETCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $out/p$i -o run --output-format csv -- python3 tools/prof_dec.py 16384 2 0 \
    > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; exit 1; }
done
python3 tools/counters_table.py $out
