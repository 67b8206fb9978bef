# emit with coalesced tile loads + LDS transpose: full GPU suite, bench A/B against the per-lane block loads
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/v_pytest.log 2>&1
B="python -u bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-extras"
for i in 1 2; do
for v in "" emitold; do
  if [ -n "$v" ]; then L=hiccup_amd/lib/libhiccup_hip_dev$v.so; else L=hiccup_amd/lib/libhiccup_hip.so; fi
  HICCUP_HIP_LIB=$L run 200 $B > gpurun_out/v_b_${v}_$i.log 2>&1
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "" emitold; do
  if [ -n "$v" ]; then L=hiccup_amd/lib/libhiccup_hip_dev$v.so; else L=hiccup_amd/lib/libhiccup_hip.so; fi
  HICCUP_HIP_LIB=$L run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v_prof_$v -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-extras --streams 1 > gpurun_out/v_prof_$v.log 2>&1
done
