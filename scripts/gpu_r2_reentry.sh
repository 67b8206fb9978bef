# re-entry check of the current tree: GPU tests, smoke, default bench, self-launched 2-rank rehearsal on one GPU
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out/reentry
run 500 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/reentry/pytest.log 2>&1
run 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/reentry/smoke.log 2>&1
run 300 python -u bench.py > gpurun_out/reentry/bench.log 2>&1
run 300 python -u bench.py --gpus 2 --steps 8 --warmup 2 --dist-backend gloo --same-device > gpurun_out/reentry/bench_n2.log 2>&1
