# emit change: codec GPU tests + bench
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 500 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_codec.py > gpurun_out/h_pytest.log 2>&1
run 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/h_bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/h_trace -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-extras --streams 1 > gpurun_out/h_trace.log 2>&1
