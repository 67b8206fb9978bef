# producer / consumer CU split (bench --cu-split F) vs the 2-stream default
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
B="python -u bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-extras"
run 200 $B > gpurun_out/af_base.log 2>&1
for f in 0.5 0.55 0.6 0.65; do
  run 200 $B --cu-split $f > gpurun_out/af_$f.log 2>&1
done
run 200 $B > gpurun_out/af_base2.log 2>&1
