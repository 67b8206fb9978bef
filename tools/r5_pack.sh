#!/bin/bash
# dev: decode tests, then the 16K decode (fused RGB form, and the planes form) for
# the product library against hiccup_amd/lib/libhiccup_hip_devprev.so, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/pack_${1:-a}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_transform.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "indexed or 16k or stitch or decode or roundtrip or idct or layouts" > $out/gputest.log 2>&1 \
  || { tail -30 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
for r in 1 2 3; do
  for l in new prev; do
    so=$PWD/hiccup_amd/lib/libhiccup_hip.so
    [ $l = prev ] && so=$PWD/hiccup_amd/lib/libhiccup_hip_devprev.so
    d=$out/${l}_$r
    HICCUP_HIP_LIB=$so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 tools/prof_dec.py 16384 6 0 0 2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    echo "$l r$r: $(grep median $d.log | cut -c1-60)"
    python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rld' in r['Name']:  # noqa
        print('    ', r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3, 2))
PY
  done
done
# Cb beside Cr on a side stream (chroma_streams 2, the default) vs both on one stream
for r in 1 2; do
  for cs in 2 1; do
    d=$out/cs${cs}_$r
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 tools/prof_dec.py 16384 6 0 0 $cs > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    echo "cs=$cs r$r: $(grep median $d.log | cut -c1-90)"
  done
done
