# k_dct_planes register budget / grid A/B (tools/dct_ab.py)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 300 python -u tools/dct_ab.py "wpe3-g12:" "wpe3-g8:dct_waves_per_cu=8" "wpe3-g16:dct_waves_per_cu=16" "wpe3-g0:dct_waves_per_cu=0" > gpurun_out/ad.log 2>&1
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devdw2.so run 300 python -u tools/dct_ab.py "wpe2-g8:dct_waves_per_cu=8" "wpe2-g0:dct_waves_per_cu=0" >> gpurun_out/ad.log 2>&1
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devdw4.so run 300 python -u tools/dct_ab.py "wpe4-g16:dct_waves_per_cu=16" "wpe4-g0:dct_waves_per_cu=0" >> gpurun_out/ad.log 2>&1
run 300 python -u tools/dct_ab.py "wpe3-g12:" >> gpurun_out/ad.log 2>&1
