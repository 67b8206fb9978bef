# dev A/B of the forward DCT launch (dev library: results invalid under dev bits)
set -u
export HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_dev.so
timeout -k 10 300 python -u tools/dct_ab.py "$@" > gpurun_out/ab.log 2>&1; echo rc=$?
