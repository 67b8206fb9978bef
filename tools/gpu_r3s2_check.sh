#!/bin/bash
# dev: final-state check: GPU tests, smoke, default bench line, the default bench
# command under a kernel trace.
set -e -o pipefail
tag=${1:-r03s2c}
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$tag
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gputest.log 2>&1
tail -1 $o/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 400 python bench.py > $o/bench_default.json 2>&1
tail -1 $o/bench_default.json | cut -c1-200
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d "$GRAFT_REPO_ROOT/$o/default_trace" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-extras --no-cpu-baseline > "$GRAFT_REPO_ROOT/$o/default_trace.log" 2>&1)
echo done
