"""A/B timer (dev tool): hic_dequant_idct_u8 on a 16384 x 16384 luma plane of
zig-zag int16 coefficients (4.19M blocks: 537 MB read, 268 MB written), HIP
events around 20 launches after 3 warmups.
usage: HICCUP_HIP_LIB=... python tools/idct_ab.py label"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from hiccup_amd import _lib, device  # noqa: E402

H = W = 16384
nblk = (H // 8) * (W // 8)
g = torch.Generator(device="cuda").manual_seed(2)
coef = torch.randint(-40, 41, (nblk, 64), dtype=torch.int16, device="cuda", generator=g)
out = torch.empty((H, W), dtype=torch.uint8, device="cuda")


def launch():
    _lib.call("hic_dequant_idct_u8", device.ptr(coef), 2, H, W, 0, device.ptr(out), W, device.stream_ptr())


for _ in range(3):
    launch()
torch.cuda.synchronize()
best = 1e9
for rep in range(3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        launch()
    e.record()
    e.synchronize()
    best = min(best, s.elapsed_time(e) * 1e3 / 20)
nbytes = nblk * 128 + H * W
print("%s dequant+IDCT 16K luma: %.1f us per launch, %.0f GB/s (%.3f of 8 TB/s), checksum %d" % (
    sys.argv[1] if len(sys.argv) > 1 else "", best, nbytes / best * 1e-3, nbytes / best * 1e-3 / 8000,
    int(out[::97, ::89].to(torch.int64).sum())))
