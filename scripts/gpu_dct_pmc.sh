# SQ counters of the forward DCT launch under a dev variant (dev library)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_dev.so
i=0
for v in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/pmc_$i -o run --output-format csv -- python3 tools/dct_ab.py "$v" > gpurun_out/pmc_$i.log 2>&1
  echo "variant $i ($v) rc=$?"
  i=$((i+1))
done
