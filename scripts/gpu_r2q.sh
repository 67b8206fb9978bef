# 3 vs 2 waves after the dot4 colour stage; profile v2 (trace + PMC + SQ)
set -u
run() { timeout -k 10 "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
mkdir -p gpurun_out
run 200 python -u tools/enc_ab.py "w2:" "w3:encode_waves=3" "w2b:" "w3b:encode_waves=3" > gpurun_out/q_ab.log 2>&1
run 900 bash tools/prof_r2.sh r02v2 > gpurun_out/q_prof.log 2>&1
