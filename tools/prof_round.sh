#!/bin/bash
# dev: the round's committed profiles.  Run on the GPU box:
#   gpurun -- bash tools/prof_round.sh <tag>
# 0) the plain bench command (JSON line incl. extra_configs and cpu_baseline)
# 1) rocprofv3 --kernel-trace --stats of the bench command without its extra
#    configs (they launch the same kernels on other sizes), i.e. exactly the 8K
#    encode whose roofline the JSON line reports: once on one stream (every DCT
#    launch runs alone, as in the bench's roofline pass) and once with the
#    default two overlapped streams
# 2) separate --pmc passes FETCH_SIZE and WRITE_SIZE over the 8K luma DCT driver
#    and over the access-pattern calibration kernel (tools/micro/cal_traffic.hip)
set -e -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -o $out/cal_traffic tools/micro/cal_traffic.hip
timeout -k 10 120 $out/cal_traffic > $out/cal_traffic.log 2>&1
timeout -k 10 300 python3 bench.py > $out/bench_plain.json.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/bench -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --streams 1 > $out/bench.json.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/bench_s2 -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $out/bench_s2.json.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c -d $out/pmc_$c -o run --output-format csv -- python3 tools/prof_dct.py 8 \
    > $out/pmc_$c.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $c -d $out/cal_$c -o run --output-format csv -- $out/cal_traffic \
    > $out/cal_$c.log 2>&1
done
echo done
