#!/bin/bash
# dev: round-5 packed-DCT check (gpurun -- bash tools/r5_pk.sh <tag> [filter]): GPU tests
# (a -k filter or all), smoke, the plane-kernel A/B (float64 vs packed, prefetch), bench
set -o pipefail
tag=${1:-a}
filt=${2:-}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5/pk_$tag
mkdir -p $out
if [ -n "$filt" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$filt" \
    > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; exit 1; }
fi
tail -2 $out/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u tools/dct_ab.py -r 2 "f64:dct_path=1" "pk:dct_path=3,dct_pk_pf=0" "pk_pf:dct_path=3,dct_pk_pf=1" \
  > $out/dct_ab.log 2>&1 || { tail -20 $out/dct_ab.log; exit 1; }
cat $out/dct_ab.log
timeout -k 10 200 python -u tools/enc_ab.py f64:encode_pk=0 pk:encode_pk=1 f64b:encode_pk=0 pkb:encode_pk=1 \
  > $out/enc_ab.log 2>&1 || { tail -20 $out/enc_ab.log; exit 1; }
cat $out/enc_ab.log
for v in 0 1 0 1; do
  timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --knob encode_pk=$v > $out/bench_pk$v.json 2>&1 \
    || { tail -20 $out/bench_pk$v.json; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$out/bench_pk$v.json') if l.startswith('{')][-1]);print('encode_pk=$v', d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['ms_per_step_regions'])"
done
[ "${3:-}" = "nobench" ] && exit 0
timeout -k 10 500 python -u bench.py > $out/bench_default.json 2>&1 || { tail -20 $out/bench_default.json; exit 1; }
grep '^{' $out/bench_default.json | tail -1 | cut -c1-300
