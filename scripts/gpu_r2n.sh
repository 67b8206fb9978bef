# fused variants parity (restored f32 code) + streams A/B
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused" > gpurun_out/n_pytest.log 2>&1
B="python -u bench.py --steps 40 --warmup 5 --no-extras --no-cpu-baseline"
for i in 1 2; do
run 200 $B --streams 2 > gpurun_out/n_s2_$i.log 2>&1
run 200 $B --streams 4 > gpurun_out/n_s4_$i.log 2>&1
done
