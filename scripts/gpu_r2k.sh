# round-2 profiles + the plain bench line (extras + CPU baseline)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u bench.py > gpurun_out/k_bench_plain.log 2>&1
run 900 bash tools/prof_r2.sh r02b
