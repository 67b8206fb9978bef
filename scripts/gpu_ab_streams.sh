# A/B: consecutive 8K images on 2 vs 4 HIP streams (3 alternations)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in a b c; do
  for n in 2 4; do
    run 200 python -u bench.py --no-extras --no-cpu-baseline --steps 40 --streams $n > gpurun_out/ab2_s${n}_$r.json 2>&1
  done
done
