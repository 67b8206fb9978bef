# A/B of the DCT coefficient-store variant: GPU tests with it on, bench with it off and on
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/diag_all.log 2>&1
HIC_DCT_WT=0 run 200 python -u bench.py > gpurun_out/bench_wt0.json 2>&1
run 200 python -u bench.py > gpurun_out/bench_wt1.json 2>&1
HIC_DCT_WT=0 run 200 python -u bench.py > gpurun_out/bench_wt0b.json 2>&1
run 200 python -u bench.py > gpurun_out/bench_wt1b.json 2>&1
