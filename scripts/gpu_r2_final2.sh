# round-2 end check of the final tree: GPU tests, smoke, default bench (N=1), 2-rank
# same-device rehearsals (8K strong with gather, 4K), then the round profiles
# (tools/prof_r2.sh: kernel trace, calibrated PMC traffic of every encode kernel, SQ)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
o=gpurun_out/final2; mkdir -p $o
run 500 python -u -m pytest -x -q -m gpu --timeout 150 --timeout-method thread tests > $o/pytest_gpu.log 2>&1
run 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
run 300 python -u bench.py > $o/bench_plain.json.log 2>&1
run 300 python -u bench.py --gpus 2 --steps 8 --warmup 2 --dist-backend gloo --same-device > $o/bench_n2_8k.log 2>&1
run 300 python -u bench.py --gpus 2 --steps 8 --warmup 2 --dist-backend gloo --same-device --workload 4k --no-extras > $o/bench_n2_4k.log 2>&1
run 200 rocprofv3 --kernel-trace --stats -d $o/default_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras > $o/default_bench.json.log 2>&1
run 700 bash tools/prof_r2.sh final2
echo done
