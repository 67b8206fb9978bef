# A/B: fused encoder with XCD-banded workgroups (knob encode_xcd=1) vs dispatch order;
# parity of both variants first, then launch times, bench lines and read traffic
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
o=gpurun_out/xcd; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py -k "fused_encoder_matches" > $o/pytest.log 2>&1
run 200 python -u tools/enc_ab.py base: xcd:encode_xcd=1 base: xcd:encode_xcd=1 base: xcd:encode_xcd=1 > $o/enc_ab.log 2>&1
for i in 1 2; do
  run 200 python -u bench.py --no-extras --no-cpu-baseline > $o/bench_base_$i.log 2>&1
  run 200 python -u bench.py --no-extras --no-cpu-baseline --knob encode_xcd=1 > $o/bench_xcd_$i.log 2>&1
done
for c in FETCH_SIZE; do
  run 120 rocprofv3 --pmc $c -d $o/pmc_base_$c -o run --output-format csv -- python3 tools/enc_ab.py base: > $o/pmc_base_$c.log 2>&1
  run 120 rocprofv3 --pmc $c -d $o/pmc_xcd_$c -o run --output-format csv -- python3 tools/enc_ab.py xcd:encode_xcd=1 > $o/pmc_xcd_$c.log 2>&1
done
echo done
