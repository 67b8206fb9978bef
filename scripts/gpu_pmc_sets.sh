# two SQ counter passes over one DCT dev variant: lib=$1 variant=$2
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_$1.so
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU -d gpurun_out/pa -o run --output-format csv -- python3 tools/dct_ab.py "$2" > gpurun_out/pa.log 2>&1; echo rc=$?
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_LEVEL_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_IFETCH_LEVEL SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU -d gpurun_out/pb -o run --output-format csv -- python3 tools/dct_ab.py "$2" > gpurun_out/pb.log 2>&1; echo rc=$?
