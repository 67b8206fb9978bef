# k_dct_planes on its own: SQ wave-cycle breakdown (bench --unfused, one stream) + the new 8K luma extra
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-extras --streams 1 --unfused"
run 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/ab_sq -o run --output-format csv -- $B > gpurun_out/ab_sq.log 2>&1
run 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1
