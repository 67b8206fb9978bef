# PMC SQ counters of the fused encoder (w2) and its dev variants
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
for L in "" devnodct devnocol; do
  lib=hiccup_amd/lib/libhiccup_hip${L:+_$L}.so
  HICCUP_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/g_pmc_${L:-full} -o run --output-format csv -- python3 tools/enc_ab.py "w2:encode_waves=2" > gpurun_out/g_${L:-full}.log 2>&1 || { echo "fail $L"; exit 1; }
done
echo done
