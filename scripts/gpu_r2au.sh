# fused encoder workgroup -> units: column groups (new default) vs row-major; parity, kernel time, bench, FETCH_SIZE
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused or shard or 16k" > gpurun_out/au_pytest.log 2>&1
OLD=hiccup_amd/lib/libhiccup_hip_devrowmaj.so
B="python -u bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-extras"
for i in 1 2; do
  HICCUP_HIP_LIB=$OLD run 200 python -u tools/enc_ab.py "rowmajor:" >> gpurun_out/au_ab.log 2>&1
  run 200 python -u tools/enc_ab.py "cols:" >> gpurun_out/au_ab.log 2>&1
  HICCUP_HIP_LIB=$OLD run 200 $B > gpurun_out/au_bench_row_$i.log 2>&1
  run 200 $B > gpurun_out/au_bench_cols_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
HICCUP_HIP_LIB=$OLD run 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/au_pmc_row -o run --output-format csv -- python3 tools/enc_ab.py "rowmajor:" > gpurun_out/au_pmc_row.log 2>&1
run 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/au_pmc_cols -o run --output-format csv -- python3 tools/enc_ab.py "cols:" > gpurun_out/au_pmc_cols.log 2>&1
