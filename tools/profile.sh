#!/bin/bash
# The round's profiling driver (dev tool; run on the GPU box):
#   gpurun -- bash tools/profile.sh <step> <tag>
# Every step writes under gpurun_out/r6/<tag>/; the summaries worth keeping are
# copied into profiles/r06/ and cited from DESIGN.md.
#   final : pytest -m gpu, smoke(), the default bench line (extras, CPU baseline)
#   trace : rocprofv3 --kernel-trace --stats of the default bench command (every
#           extra's launches in order) + the DCT launches and the 16K trip listed
#           (tools/trace_launches.py)
#   pmc   : the 8K bench on one stream (every launch alone): kernel trace, separate
#           FETCH_SIZE / WRITE_SIZE passes corrected by the calibration kernels of
#           the same access patterns (tools/micro/cal_patterns.hip), one SQ pass;
#           tools/prof_summary.py -> prof_summary.json (per-kernel HBM bytes)
#   luma  : north_star's pass (the 16-plane 8K luma DCT + quantize launch,
#           records-free, tools/prof_luma.py): kernel trace + two SQ / GRBM counter
#           passes (GRBM_GUI_ACTIVE and SQ_BUSY_CYCLES: the shader clock per
#           dispatch); tools/counters_table.py
#   dec   : the 16K round trip's kernels (tools/prof_roundtrip.py) traced
set -o pipefail
step=${1:?step}
tag=${2:-a}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6/$tag
mkdir -p $out
prof() { (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && "$@"); }
case $step in
final)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
  tail -3 $out/gputest.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
  grep -v amdgpu.ids $out/smoke.log
  timeout -k 10 500 python -u bench.py > $out/bench_default.json 2>&1 || { tail -20 $out/bench_default.json; exit 1; }
  grep '^{' $out/bench_default.json | tail -1 | cut -c1-600
  ;;
trace)
  prof timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/trace_default -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $out/trace_default.json.log 2>&1 || { tail -5 $out/trace_default.json.log; exit 1; }
  python3 tools/trace_launches.py $out/trace_default/run_kernel_trace.csv k_dct > $out/trace_default_dct_launches.txt
  python3 tools/trace_launches.py $out/trace_default/run_kernel_trace.csv k_encode420 k_rle k_rld > \
    $out/trace_default_encode_launches.txt
  head -c 2000 $out/trace_default_dct_launches.txt
  ;;
pmc)
  hipcc --offload-arch=gfx950 -O3 -o $out/cal_patterns tools/micro/cal_patterns.hip
  timeout -k 10 120 $out/cal_patterns > $out/cal_patterns.log 2>&1 || exit 1
  B="python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-extras --streams 1 ${PROF_ARGS:-}"
  prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $B \
    > $out/trace.json.log 2>&1 || { tail -5 $out/trace.json.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    prof timeout -s KILL 180 rocprofv3 --pmc $c -d $out/pmc_$c -o run --output-format csv -- $B > $out/pmc_$c.log 2>&1 \
      || { tail -5 $out/pmc_$c.log; exit 1; }
    prof timeout -s KILL 120 rocprofv3 --pmc $c -d $out/cal_$c -o run --output-format csv -- $out/cal_patterns \
      > $out/cal_$c.log 2>&1 || { tail -5 $out/cal_$c.log; exit 1; }
  done
  prof timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $out/pmc_sq -o run --output-format csv -- $B \
    > $out/pmc_sq.log 2>&1 || { tail -5 $out/pmc_sq.log; exit 1; }
  python3 tools/prof_summary.py $out $out/prof_summary.json > /dev/null && echo "prof_summary.json written"
  ;;
luma)
  prof timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/luma_trace -o run --output-format csv -- \
    python3 tools/prof_luma.py 16 1 16 0 > $out/luma_trace.log 2>&1 || { tail -5 $out/luma_trace.log; exit 1; }
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_CYCLES"; do
    i=$((i+1))
    prof timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $out/luma_p$i -o run --output-format csv -- \
      python3 tools/prof_luma.py 16 1 16 0 > $out/luma_p$i.log 2>&1 || { tail -5 $out/luma_p$i.log; exit 1; }
  done
  python3 tools/counters_table.py $out > $out/luma_counters.txt 2>&1; cat $out/luma_counters.txt
  python3 tools/luma_clock.py $out/luma_p1 16 > $out/luma_clock.txt 2>&1; cat $out/luma_clock.txt
  ;;
dec)
  prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/dec_trace -o run --output-format csv -- \
    python3 tools/prof_roundtrip.py > $out/dec_trace.log 2>&1 || { tail -5 $out/dec_trace.log; exit 1; }
  python3 tools/trace_launches.py $out/dec_trace/run_kernel_trace.csv k_ > $out/dec_launches.txt
  head -c 3000 $out/dec_launches.txt
  ;;
decsq)
  # SQ counters of the round trip's kernels (two passes), RT_N = 8192 keeps them short
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    RT_N=${RT_N:-8192} prof timeout -s KILL 120 rocprofv3 --pmc $set -d $out/decsq_p$i -o run --output-format csv -- \
      python3 tools/prof_roundtrip.py > $out/decsq_p$i.log 2>&1 || { tail -5 $out/decsq_p$i.log; exit 1; }
  done
  python3 tools/counters_table.py $out > $out/decsq.txt 2>&1; cat $out/decsq.txt
  ;;
*)
  echo "unknown step $step"; exit 2 ;;
esac
