#!/bin/bash
# dev: 2-rank rehearsal of the N > 1 bench on the one-GPU box (gloo, same device):
# the gathered streams are verified bit-exact against a one-GPU encode in the line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4/n2
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --same-device --dist-backend gloo --steps 8 --warmup 2 \
  > $out/bench_n2.json 2>&1 || { tail -20 $out/bench_n2.json; exit 1; }
grep '^{' $out/bench_n2.json | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('gather_verify'))"
