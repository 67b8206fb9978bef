# A/B of nontemporal symbol stores in the RLE emit: GPU tests with them on, then the bench off/on twice
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/nt_pytest.log 2>&1
for r in a b; do
  HIC_RLE_NT=0 run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 --streams 1 > gpurun_out/nt0_s1_$r.json 2>&1
  run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 --streams 1 > gpurun_out/nt1_s1_$r.json 2>&1
  HIC_RLE_NT=0 run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/nt0_s2_$r.json 2>&1
  run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 > gpurun_out/nt1_s2_$r.json 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HIC_RLE_NT=0 run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/nt0prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --streams 1 > /dev/null 2>&1
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/nt1prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --streams 1 > /dev/null 2>&1
