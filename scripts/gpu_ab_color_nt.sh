# A/B of nontemporal plane stores in the colour kernel (HIC_COLOR_NT=1)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
HIC_COLOR_NT=1 run 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_codec.py -k "pipeline_encoder or colour" > gpurun_out/cnt_pytest.log 2>&1
for r in a b; do
  run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 --streams 1 > gpurun_out/cnt0_s1_$r.json 2>&1
  HIC_COLOR_NT=1 run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 --streams 1 > gpurun_out/cnt1_s1_$r.json 2>&1
  run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/cnt0_s2_$r.json 2>&1
  HIC_COLOR_NT=1 run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/cnt1_s2_$r.json 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIC_COLOR_NT=1 run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cnt1prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --streams 1 > /dev/null 2>&1
