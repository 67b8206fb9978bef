# A/B: LLVM AMDGPU scheduler strategy for the whole library (dev builds: default,
# iterative-ilp, max-ilp), fused encoder launch time and the bench line
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
o=gpurun_out/sched; mkdir -p $o
L=hiccup_amd/lib
for r in 1 2 3; do
  for v in base iilp milp; do
    HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so run 120 python -u tools/enc_ab.py $v: >> $o/enc_ab.log 2>&1
  done
done
for v in base iilp milp; do
  HICCUP_HIP_LIB=$L/libhiccup_hip_dev$v.so run 200 python -u bench.py --no-extras --no-cpu-baseline > $o/bench_$v.log 2>&1
done
echo done
