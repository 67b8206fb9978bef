# dot4 colour: where the fused kernel's time goes (no-DCT / no-colour dev builds) and the load lookahead
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
for v in "" nodct nocol la4 la9; do
  if [ -n "$v" ]; then L=hiccup_amd/lib/libhiccup_hip_dev$v.so; else L=hiccup_amd/lib/libhiccup_hip.so; fi
  HICCUP_HIP_LIB=$L run 200 python -u tools/enc_ab.py "w2:" "w2b:" > gpurun_out/r_ab_$v.log 2>&1
done
