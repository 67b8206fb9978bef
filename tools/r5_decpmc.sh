#!/bin/bash
# dev: FETCH_SIZE and WRITE_SIZE (one rocprofv3 --pmc pass each) of the 16K decode
# kernels (tools/prof_dec.py, fused RGB form, 2 decodes); per-kernel means
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/decpmc_${1:-a}
mkdir -p $out
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/p$i -o run --output-format csv -- python3 tools/prof_dec.py 16384 2 0 \
    > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; exit 1; }
done
python3 tools/counters_table.py $out
