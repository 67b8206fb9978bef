# encode_lds_pad: one encode workgroup per CU so the other stream's emit runs beside it
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
B="python -u bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-extras"
for i in 1 2; do
  run 200 $B > gpurun_out/w_pad0_$i.log 2>&1
  run 200 $B --knob encode_lds_pad=40 > gpurun_out/w_pad40_$i.log 2>&1
  run 200 $B --knob encode_lds_pad=40 --streams 4 > gpurun_out/w_pad40s4_$i.log 2>&1
done
run 200 python -u tools/enc_ab.py "p0:" "p40:encode_lds_pad=40" > gpurun_out/w_ab.log 2>&1
