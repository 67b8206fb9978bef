# two vertically adjacent units per wave (HIC_ENC_VG=2) vs one: fused parity + GPU suite, launch timing, bench
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/ah_pytest.log 2>&1
for i in 1 2; do
run 200 python -u tools/enc_ab.py "vg2:" >> gpurun_out/ah_ab.log 2>&1
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devvg1.so run 200 python -u tools/enc_ab.py "vg1:" >> gpurun_out/ah_ab.log 2>&1
done
B="python -u bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-extras"
run 200 $B > gpurun_out/ah_b_vg2.log 2>&1
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_devvg1.so run 200 $B > gpurun_out/ah_b_vg1.log 2>&1
