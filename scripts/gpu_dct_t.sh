# transform GPU tests + dev A/B of the DCT launch
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_transform.py > gpurun_out/d_pytest.log 2>&1
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_dev.so run 300 python -u tools/dct_ab.py "$@" > gpurun_out/ab.log 2>&1
