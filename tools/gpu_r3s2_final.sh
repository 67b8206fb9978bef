#!/bin/bash
# dev: round-3 (second session) final GPU pass: GPU tests, smoke, the default
# bench line, an N = 2 same-device gloo rehearsal of the stream gather, the default
# bench command under a kernel trace, then tools/prof_r2.sh (one-stream kernel
# trace + calibrated PMC + SQ).   gpurun -- bash tools/gpu_r3s2_final.sh <tag>
set -e -o pipefail
tag=${1:-r03s2}
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1
tail -1 $o/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 400 python bench.py > $o/bench_default.json 2>&1
tail -1 $o/bench_default.json | cut -c1-300
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --same-device --no-extras --no-cpu-baseline --steps 8 --warmup 2 > $o/bench_n2_samedev_gloo.json 2>&1
tail -1 $o/bench_n2_samedev_gloo.json | cut -c1-300
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d "$GRAFT_REPO_ROOT/$o/default_trace" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-extras --no-cpu-baseline > "$GRAFT_REPO_ROOT/$o/default_trace.log" 2>&1)
bash tools/prof_r2.sh $tag
echo done
