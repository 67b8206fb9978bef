#!/bin/bash
# dev: SQ + TCC counters for every kernel of a short bench run, plus bandwidth ceilings
set -e -o pipefail
tag=${1:-cnt}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag
mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -o $out/bw tools/micro/bw.hip 2>/dev/null
timeout -k 10 120 $out/bw > $out/bw.log 2>&1
cat $out/bw.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $out/sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/write.log 2>&1
timeout -k 10 120 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES -d $out/sq2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/sq2.log 2>&1
echo done
