# sharded decode: GPU tests (one-process shards + 2/3-process gloo ranks), 2-rank bench rehearsal with the 16K trip
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "shards or roundtrip" > gpurun_out/b_pytest.log 2>&1
run 400 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/b_dist.log 2>&1
run 300 python -u bench.py --gpus 2 --steps 6 --warmup 2 --dist-backend gloo --same-device > gpurun_out/b_m2.log 2>&1
