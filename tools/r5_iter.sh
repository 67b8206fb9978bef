#!/bin/bash
# dev: one iteration on the GPU box (gpurun -- bash tools/r5_iter.sh <tag> [filter]):
# GPU tests (a -k filter), then the plane-kernel and fused-encoder A/Bs (float64 vs
# packed), twice alternating
set -o pipefail
tag=${1:-a}
filt=${2:-"PK or pk or fused or tie or structured or full_size or records"}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/it_$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$filt" \
  > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
timeout -k 10 400 python -u tools/dct_ab.py -r 2 "f64:dct_path=1" "pk:dct_path=3" > $out/dct_ab.log 2>&1 \
  || { tail -20 $out/dct_ab.log; exit 1; }
grep -v amdgpu.ids $out/dct_ab.log
timeout -k 10 200 python -u tools/enc_ab.py f64:encode_pk=0 pk:encode_pk=1 f64b:encode_pk=0 pkb:encode_pk=1 \
  > $out/enc_ab.log 2>&1 || { tail -20 $out/enc_ab.log; exit 1; }
grep -v amdgpu.ids $out/enc_ab.log
