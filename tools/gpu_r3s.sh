#!/bin/bash
# dev: the 4K RGB extra (north_star's 4K point) on 2 vs 4 streams, 4 alternating pairs
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r3s
mkdir -p $o
timeout -k 10 600 python -c "
import bench, json, torch
torch.cuda.set_device(0)
for rep in range(4):
    for n in (2, 4):
        r = bench.extra_4k_rgb_encode(n_streams=n)
        print(n, rep, r['ms_per_image'], r['mpix_s'], flush=True)
" > $o/ab.txt 2>&1
cat $o/ab.txt
