#!/bin/bash
# dev: re-entry GPU pass (round 3, session 2): GPU tests, smoke, bench line, then
# the fused encoder's DCT variant x register budget A/B and the plane DCT paths.
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3c
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1
tail -2 $o/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 400 python bench.py > $o/bench.log 2>&1
tail -1 $o/bench.log | cut -c1-400
timeout -k 10 200 python tools/enc_ab.py "f64w2:" "pkw2:encode_dct=2" "pkw3:encode_dct=2,encode_waves=3" "f64w3:encode_waves=3" "f64w2b:" "pkw3b:encode_dct=2,encode_waves=3" > $o/enc_ab.log 2>&1
cat $o/enc_ab.log
echo done
