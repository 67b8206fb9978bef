# multi-workgroup tile-offset scan in the hot-path decode: parity (long dense
# stream past one scan chunk, 16K round trip) then the default bench under rocprof
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 400 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_codec.py -k "rle_decode_blocks_hot_path or 16k_roundtrip" > gpurun_out/al_pytest.log 2>&1
cd /tmp && export TMPDIR=/tmp
run 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/al_prof -o al -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/al_bench.log 2>&1
