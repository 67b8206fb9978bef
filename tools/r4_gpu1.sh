#!/bin/bash
# round 4 GPU batch: parity of the MFMA paths, then the A/Bs (dev tool)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_transform.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4/t_transform.log 2>&1 || { tail -30 gpurun_out/r4/t_transform.log; exit 1; }
tail -2 gpurun_out/r4/t_transform.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread \
  -k "fused_encoder" > gpurun_out/r4/t_fused.log 2>&1 || { tail -30 gpurun_out/r4/t_fused.log; exit 1; }
tail -2 gpurun_out/r4/t_fused.log
timeout -k 10 400 python -u tools/mfma_var_ab.py 2 > gpurun_out/r4/ab_var.log 2>&1 || { tail -5 gpurun_out/r4/ab_var.log; exit 1; }
cat gpurun_out/r4/ab_var.log | grep rep
timeout -k 10 300 python -u tools/enc_mfma_ab.py 3 > gpurun_out/r4/ab_enc.log 2>&1 || { tail -5 gpurun_out/r4/ab_enc.log; exit 1; }
cat gpurun_out/r4/ab_enc.log | grep rep
