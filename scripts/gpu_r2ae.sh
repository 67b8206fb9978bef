# emit grid A/B (persistent 12 / 8 waves per CU vs one wave per tile) + plane DCT default check + GPU suite
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/ae_pytest.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
for v in cur ew0 ew8; do
  if [ $v = cur ]; then L=hiccup_amd/lib/libhiccup_hip.so; else L=hiccup_amd/lib/libhiccup_hip_dev$v.so; fi
  HICCUP_HIP_LIB=$L run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ae_${v}_$i -o run --output-format csv -- python3 bench.py --steps 24 --warmup 4 --no-cpu-baseline --no-extras --streams 1 > gpurun_out/ae_${v}_$i.log 2>&1
done
done
run 300 python -u tools/dct_ab.py "default:" > gpurun_out/ae_dct.log 2>&1
