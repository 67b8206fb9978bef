# round-2 checkpoint: full GPU suite, smoke, default bench (the driver's command)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/ai_pytest.log 2>&1
run 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/ai_smoke.log 2>&1
run 400 python -u bench.py > gpurun_out/ai_bench.log 2>&1
