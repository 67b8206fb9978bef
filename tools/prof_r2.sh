#!/bin/bash
# dev: round-2 profiles.  On the GPU box:  gpurun -- bash tools/prof_r2.sh <tag>
# 0) calibration kernels (tools/micro/cal_patterns.hip: each encode kernel's load
#    pattern with known bytes)
# 1) rocprofv3 --kernel-trace --stats of the 8K bench on one stream (every launch
#    alone: per-kernel durations)
# 2) separate --pmc passes FETCH_SIZE, WRITE_SIZE (bench and calibration) and one
#    SQ pass (wave-cycle breakdown)
set -e -o pipefail
tag=${1:-r02}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -o $out/cal_patterns tools/micro/cal_patterns.hip
timeout -k 10 120 $out/cal_patterns > $out/cal_patterns.log 2>&1
B="python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-extras --streams 1 ${PROF_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $B > $out/trace.json.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d $out/pmc_$c -o run --output-format csv -- $B > $out/pmc_$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/cal_$c -o run --output-format csv -- $out/cal_patterns > $out/cal_$c.log 2>&1
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $out/pmc_sq -o run --output-format csv -- $B > $out/pmc_sq.log 2>&1
echo done
