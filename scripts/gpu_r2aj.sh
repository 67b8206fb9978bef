# plane DCT grid per workload: one wave per set vs persistent 8 / 12 waves per CU (4K luma, 8K luma, 8K planes)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 400 python -u tools/dct_ab.py "g0:" "g8:dct_waves_per_cu=8" "g12:dct_waves_per_cu=12" "g0b:" "g8b:dct_waves_per_cu=8" > gpurun_out/aj.log 2>&1
