# the default bench command under rocprofv3 --kernel-trace --stats (trace phases vs the bench line's events)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/x_prof -o run --output-format csv -- python3 bench.py > gpurun_out/x_bench.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
