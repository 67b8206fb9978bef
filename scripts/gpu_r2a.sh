# round 2 first check: GPU tests, DCT path A/B (production library), bench line, 2-rank rehearsal
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 500 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/a_pytest.log 2>&1
run 200 python -u tools/dct_ab.py "f64aan:dct_path=1" "f32aan:dct_path=3" "exact:dct_path=0" "f64aan:dct_path=1" "f32aan:dct_path=3" > gpurun_out/a_ab.log 2>&1
run 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/a_bench.log 2>&1
run 300 python -u bench.py --gpus 2 --steps 6 --warmup 2 --dist-backend gloo --same-device --no-cpu-baseline > gpurun_out/a_m2.log 2>&1
