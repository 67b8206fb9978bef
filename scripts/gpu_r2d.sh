# fused encoder: parity tests, then bench fused vs unfused, kernel A/B
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused or pipeline_encoder or shards" > gpurun_out/d_pytest.log 2>&1
run 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/d_bench_fused.log 2>&1
run 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --unfused > gpurun_out/d_bench_unfused.log 2>&1
run 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --streams 1 > gpurun_out/d_bench_fused_s1.log 2>&1
