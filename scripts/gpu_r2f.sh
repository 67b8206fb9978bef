# fused encoder dev A/B over variant libraries (dev bits give invalid results)
set -u
for L in la6 la10 la18 nodct nocol; do
  HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_dev$L.so timeout -k 10 200 python -u tools/enc_ab.py "w3:encode_waves=3" "w2:encode_waves=2" >> gpurun_out/f_ab.log 2>&1 || { echo "fail $L"; exit 1; }
done
echo done
