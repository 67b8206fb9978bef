#!/bin/bash
# dev: the GPU suite, smoke and the host-copy timings after the pinned staging change
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/pin
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 200 python -u tools/prof_d2h.py > $out/d2h.log 2>&1 || { tail -5 $out/d2h.log; exit 1; }
tail -4 $out/d2h.log
timeout -k 10 200 python -u tools/api_times.py > $out/api.log 2>&1 || { tail -5 $out/api.log; exit 1; }
tail -3 $out/api.log
