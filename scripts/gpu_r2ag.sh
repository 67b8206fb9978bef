# codec.jpeg_encode's Huffman back end at 8K (tools/hic_timing.py)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py -k "huffman or hic_image or jpeg_encode" > gpurun_out/ag_pytest.log 2>&1 && timeout -k 10 300 python -u tools/hic_timing.py --profile > gpurun_out/ag.log 2>&1; echo rc=$?
