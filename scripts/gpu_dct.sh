# DCT path check: transform GPU tests + bench (no extras) + kernel trace
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_transform.py > gpurun_out/d_pytest.log 2>&1
run 300 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/d_bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/d_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --streams 1 > gpurun_out/d_prof.log 2>&1
