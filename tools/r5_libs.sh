#!/bin/bash
# dev: the plane-kernel / fused A/B (tools/dct_ab.py, tools/enc_ab.py) with each
# in-tree library variant named (hiccup_amd/lib/libhiccup_hip_dev<v>.so; "prod" =
# the product library).  usage: gpurun -- bash tools/r5_libs.sh <tag> "prod v1 v2" ["spec" ...]
set -o pipefail
tag=${1:-a}
libs=${2:-prod}
shift 2
specs=("$@")
[ ${#specs[@]} -eq 0 ] && specs=("pk:dct_path=3")
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/libs_$tag
mkdir -p $out
for r in 1 2; do
  for v in $libs; do
    lib=$PWD/hiccup_amd/lib/libhiccup_hip_dev$v.so
    [ "$v" = prod ] && lib=$PWD/hiccup_amd/lib/libhiccup_hip.so
    HICCUP_HIP_LIB=$lib timeout -k 10 200 python -u tools/dct_ab.py "${specs[@]/#/$v.}" > $out/ab_${v}_$r.log 2>&1 \
      || { tail -20 $out/ab_${v}_$r.log; exit 1; }
    grep -v amdgpu.ids $out/ab_${v}_$r.log
    HICCUP_HIP_LIB=$lib timeout -k 10 200 python -u tools/enc_ab.py "$v.pk:encode_pk=1" > $out/enc_${v}_$r.log 2>&1 \
      || { tail -20 $out/enc_${v}_$r.log; exit 1; }
    grep -v amdgpu.ids $out/enc_${v}_$r.log
  done
done
