# nontemporal RGB loads in the fused encoder: does the emit's coefficient re-read hit the Infinity Cache?
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
B="python -u bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-extras"
for i in 1 2; do
for v in "" ldnt ldsc0nt; do
  if [ -n "$v" ]; then L=hiccup_amd/lib/libhiccup_hip_dev$v.so; else L=hiccup_amd/lib/libhiccup_hip.so; fi
  HICCUP_HIP_LIB=$L run 200 $B > gpurun_out/u_b_${v}_$i.log 2>&1
done
done
