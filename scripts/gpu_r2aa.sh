# same-box A/B of the emit kernel: current tree vs the previous commit (dev build "prev")
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
for v in cur prev; do
  if [ $v = prev ]; then L=hiccup_amd/lib/libhiccup_hip_devprev.so; else L=hiccup_amd/lib/libhiccup_hip.so; fi
  HICCUP_HIP_LIB=$L run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/aa_${v}_$i -o run --output-format csv -- python3 bench.py --steps 24 --warmup 4 --no-cpu-baseline --no-extras --streams 1 > gpurun_out/aa_${v}_$i.log 2>&1
done
done
