# batched group encodes + grouped rotating gathers: one-GPU multi-process tests, gloo bench rehearsals, N=1 bench
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 300 python -u -m pytest -x -v -m gpu --timeout 250 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/at_pytest.log 2>&1
run 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 8 --warmup 3 --dist-backend gloo --same-device --no-extras > gpurun_out/at_dist2.log 2>&1
run 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 3 --steps 7 --warmup 2 --dist-backend gloo --same-device --no-extras > gpurun_out/at_dist3.log 2>&1
run 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/at_n1.log 2>&1
