# emit: dense pass, unrolled copy-out with uniform tile offsets: full GPU suite, emit kernel stats, bench
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/z_pytest.log 2>&1
B="python -u bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-extras"
run 200 $B > gpurun_out/z_b1.log 2>&1
run 200 $B > gpurun_out/z_b2.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/z_prof -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-extras --streams 1 > gpurun_out/z_prof.log 2>&1
