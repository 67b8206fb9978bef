# full GPU suite + smoke + N=1 bench + N=2 same-device rehearsal (gloo) with the no-gather context line
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/o_pytest.log 2>&1
run 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/o_smoke.log 2>&1
run 300 python -u bench.py > gpurun_out/o_bench1.log 2>&1
run 300 python -u bench.py --gpus 2 --steps 8 --warmup 2 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/o_bench2.log 2>&1
