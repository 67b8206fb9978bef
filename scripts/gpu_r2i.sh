# A/B: nontemporal vs cached coefficient stores in the fused kernel; 1 and 2 streams
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
B="python -u bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline"
for i in 1 2; do
run 200 $B > gpurun_out/i_nt_$i.log 2>&1
run 200 $B --knob encode_nt=0 > gpurun_out/i_c_$i.log 2>&1
run 200 $B --streams 1 > gpurun_out/i_nt_s1_$i.log 2>&1
run 200 $B --knob encode_nt=0 --streams 1 > gpurun_out/i_c_s1_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/i_trace -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-extras --streams 1 --knob encode_nt=0 > gpurun_out/i_trace.log 2>&1
