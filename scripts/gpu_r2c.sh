# dev A/B of the forward DCT paths (dev library: dev bits give invalid results)
set -u
export HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_dev.so
timeout -k 10 300 python -u tools/dct_ab.py "f64:dct_path=1" "f32:dct_path=3" "f32-notier2:dct_path=3,dev=1" \
  "f32-nostore:dct_path=3,dev=4" "f32-noload:dct_path=3,dev=8" "f32-nodct:dct_path=3,dev=16" \
  "f32-compute:dct_path=3,dev=12" "f32-compute-notier2:dct_path=3,dev=13" "f32-mem:dct_path=3,dev=17" \
  "f32-w12:dct_path=3,dct_waves_per_cu=12" "f32-w8:dct_path=3,dct_waves_per_cu=8" "f32-w20:dct_path=3,dct_waves_per_cu=20" \
  "f64-w8:dct_path=1,dct_waves_per_cu=8" "f64-w16:dct_path=1,dct_waves_per_cu=16" "f64:dct_path=1" > gpurun_out/c_ab.log 2>&1; echo rc=$?
