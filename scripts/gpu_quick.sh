# quick GPU check: gpu tests + one bench line (no extras)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/q_pytest.log 2>&1
run 300 python -u bench.py --steps 20 --warmup 5 --no-extras > gpurun_out/q_bench.log 2>&1
