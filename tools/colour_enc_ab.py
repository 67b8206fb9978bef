"""A/B timer (dev tool): hic_rgb_to_ycrcb420 (the two-kernel path's colour +
4:2:0 pyrDown) on 7680 x 4320 and 3840 x 2160 RGB; HIP events around 20 launches
after 3 warmups; algorithmic bytes = 3 B read + 1.5 B written per pixel.
usage: HICCUP_HIP_LIB=... python tools/colour_enc_ab.py label"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from hiccup_amd import _lib, device  # noqa: E402

for H, W in ((4320, 7680), (2160, 3840)):
    g = torch.Generator(device="cuda").manual_seed(3)
    rgb = torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda", generator=g)
    y = torch.empty((H, W), dtype=torch.uint8, device="cuda")
    cr = torch.empty((H // 2, W // 2), dtype=torch.uint8, device="cuda")
    cb = torch.empty_like(cr)

    def launch():
        _lib.call("hic_rgb_to_ycrcb420", device.ptr(rgb), H, W, device.ptr(y), device.ptr(cr), device.ptr(cb),
                  device.stream_ptr())

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
    nbytes = H * W * 3 + H * W + 2 * (H // 2) * (W // 2)
    print("%s colour+pyrDown %dx%d: %.1f us per launch, %.0f GB/s (%.3f of 8 TB/s), checksum %d" % (
        sys.argv[1] if len(sys.argv) > 1 else "", W, H, best, nbytes / best * 1e-3, nbytes / best * 1e-3 / 8000,
        int(y[::7, ::5].to(torch.int64).sum() + cr[::3, ::7].to(torch.int64).sum() + cb[::5, ::3].to(torch.int64).sum())),
        flush=True)
