# GPU Huffman: device-vs-host, golden payloads, encoder .hic; then the full GPU suite
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 300 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "huffman or hic_image or golden or lenna or compression" > gpurun_out/j_pytest.log 2>&1
run 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/j_all.log 2>&1
