# multi-rank rehearsal on one GPU: gloo ranks sharing cuda:0 (self-launched), strong 8K + gather, 4K, weak
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 python -u bench.py --gpus 2 --steps 6 --warmup 2 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/m_strong2.log 2>&1
run 300 python -u bench.py --gpus 2 --steps 6 --warmup 2 --dist-backend gloo --same-device --no-cpu-baseline --workload 4k > gpurun_out/m_4k2.log 2>&1
run 300 python -u bench.py --gpus 3 --steps 4 --warmup 2 --dist-backend gloo --same-device --no-cpu-baseline --mode weak > gpurun_out/m_weak3.log 2>&1
run 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/m_pytest.log 2>&1
