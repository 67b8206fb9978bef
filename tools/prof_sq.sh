#!/bin/bash
# dev: SQ issue/stall counters for every kernel of a short bench run
# usage (GPU box): bash tools/prof_sq.sh <tag> [ENV=VAL ...]
set -e -o pipefail
tag=${1:-sq}
shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
[ $# -gt 0 ] && export "$@"
cmd=${CMD:-"python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline"}
timeout -s KILL ${PTO:-90} rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU \
  -d $out/p1 -o run --output-format csv -- $cmd > $out/p1.log 2>&1
timeout -s KILL ${PTO:-90} rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAVES \
  -d $out/p2 -o run --output-format csv -- $cmd > $out/p2.log 2>&1
timeout -s KILL ${PTO:-90} rocprofv3 --pmc FETCH_SIZE -d $out/p3 -o run --output-format csv -- $cmd > $out/p3.log 2>&1
timeout -s KILL ${PTO:-90} rocprofv3 --pmc WRITE_SIZE -d $out/p4 -o run --output-format csv -- $cmd > $out/p4.log 2>&1
python3 tools/counters_table.py $out
