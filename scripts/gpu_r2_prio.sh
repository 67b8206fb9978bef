# A/B: wave priority of the fused encoder's colour vs DCT phases (dev builds
# libhiccup_hip_devpc.so: colour phases at priority 2; _devpd: DCT phases at 2)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
o=gpurun_out/prio; mkdir -p $o
L=hiccup_amd/lib
for r in 1 2 3; do
  for v in base pc pd; do
    if [ $v = base ]; then lib=$L/libhiccup_hip.so; else lib=$L/libhiccup_hip_dev$v.so; fi
    HICCUP_HIP_LIB=$lib run 120 python -u tools/enc_ab.py $v: >> $o/enc_ab.log 2>&1
  done
done
for r in 1 2; do
  for v in base pc pd; do
    if [ $v = base ]; then lib=$L/libhiccup_hip.so; else lib=$L/libhiccup_hip_dev$v.so; fi
    HICCUP_HIP_LIB=$lib run 200 python -u bench.py --no-extras --no-cpu-baseline > $o/bench_${v}_$r.log 2>&1
  done
done
echo done
