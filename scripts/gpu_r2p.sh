# dot4 colour stage: fused parity, launch timing, bench
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused or pipeline_encoder or shards" > gpurun_out/p_pytest.log 2>&1
run 200 python -u tools/enc_ab.py "w2:" "w2b:" > gpurun_out/p_ab.log 2>&1
run 300 python -u bench.py --no-cpu-baseline > gpurun_out/p_bench1.log 2>&1
