#!/bin/bash
# dev: kernel trace + two SQ counter passes of the 16-plane 8K luma launch,
# records-free (north_star's pass), per dct_path given; counters_table summary.
# usage: gpurun -- bash tools/r5_sq.sh <tag> "1 3"
set -o pipefail
tag=${1:-a}
paths=${2:-"1 3"}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for p in $paths; do
  out=gpurun_out/r5/sq_$tag/path$p${SQ_SUFFIX:-}
  mkdir -p $out
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- \
    python3 tools/prof_luma.py 16 $p 16 0 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_IFETCH GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d $out/p$i -o run --output-format csv -- python3 tools/prof_luma.py 4 $p 16 0 \
      > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; exit 1; }
  done
  echo "== path $p"
  python3 tools/counters_table.py $out
  python3 - $out/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print('  ', r['Name'][:64].ljust(64), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
done
