# fused kernel: vertical unit grouping per workgroup -- parity + timing + PMC fetch
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "fused or pipeline_encoder or shards" > gpurun_out/m_pytest.log 2>&1
run 200 python -u tools/enc_ab.py "f64w2:" "f64w2:" > gpurun_out/m_ab.log 2>&1
run 200 python -u bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/m_b1.log 2>&1
run 200 python -u bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/m_b2.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/m_pmc -o run --output-format csv -- python3 tools/enc_ab.py "f64w2:" > gpurun_out/m_pmc.log 2>&1
