# fused kernel float32 DCT variant: parity (all variants), timing A/B
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused or pipeline_encoder" > gpurun_out/l_pytest.log 2>&1
run 200 python -u tools/enc_ab.py "f64w2:encode_dct=0,encode_waves=2" "f32w2:encode_dct=1,encode_waves=2" "f32w3:encode_dct=1,encode_waves=3" "f64w3:encode_dct=0,encode_waves=3" "f64w2:encode_dct=0,encode_waves=2" "f32w2:encode_dct=1,encode_waves=2" > gpurun_out/l_ab.log 2>&1
run 200 python -u bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline --knob encode_dct=1 > gpurun_out/l_b32.log 2>&1
run 200 python -u bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/l_b64.log 2>&1
