# fused encoder A/B: 3 vs 2 waves per SIMD, unfused; kernel trace of the fused bench
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline"
run 200 $B > gpurun_out/e_w3.log 2>&1
run 200 $B --knob encode_waves=2 > gpurun_out/e_w2.log 2>&1
run 200 $B --unfused > gpurun_out/e_unf.log 2>&1
run 200 $B --knob encode_waves=2 --streams 1 > gpurun_out/e_w2s1.log 2>&1
