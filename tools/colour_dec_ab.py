"""A/B timer (dev tool): hic_ycrcb420_to_rgb on a 16384 x 16384 image (Y 268 MB,
Cr / Cb 67 MB each, RGB 805 MB written), HIP events around 20 launches after 3
warmups; prints us per launch and GB/s of algorithmic traffic.
usage: HICCUP_HIP_LIB=... python tools/colour_dec_ab.py label"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from hiccup_amd import _lib, device  # noqa: E402

H = W = 16384
h, w = H // 2, W // 2
g = torch.Generator(device="cuda").manual_seed(1)
y = torch.randint(0, 256, (H, W), dtype=torch.uint8, device="cuda", generator=g)
cr = torch.randint(0, 256, (h, w), dtype=torch.uint8, device="cuda", generator=g)
cb = torch.randint(0, 256, (h, w), dtype=torch.uint8, device="cuda", generator=g)
out = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")


def launch():
    _lib.call("hic_ycrcb420_to_rgb", device.ptr(y), y.stride(0), device.ptr(cr), device.ptr(cb), h, w,
              device.ptr(out), device.stream_ptr())


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
nbytes = H * W + 2 * h * w + 3 * H * W
print("%s decode colour 16K: %.1f us per launch, %.0f GB/s (%.3f of 8 TB/s), checksum %d" % (
    sys.argv[1] if len(sys.argv) > 1 else "", best, nbytes / best * 1e-3, nbytes / best * 1e-3 / 8000,
    int(out[::97, ::89].to(torch.int64).sum())))
