# GPU tests, smoke, a 2-rank gloo rehearsal of the bench on one GPU, then the round profiles
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/chk_pytest.log 2>&1
run 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/chk_smoke.log 2>&1
run 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 8 --warmup 2 --dist-backend gloo --same-device > gpurun_out/chk_dist2.log 2>&1
run 600 bash tools/prof_round.sh ${1:-v9}
