"""Quick kernel-rate probe (dev tool): times each kernel over rotating buffers."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from hiccup_amd import _lib, device, transform

def timeit(fn, n, rot):
    for i in range(3): fn(i % rot)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n): fn(i % rot)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us

H, W = 4320, 7680
rot = 12
g = torch.Generator(device='cuda'); g.manual_seed(0)
planes = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device='cuda', generator=g) for _ in range(rot)]
nblk = (H // 8) * (W // 8)
for layout, name, bpp in ((2, 'zigzag_i16', 3), (1, 'raster_i16', 3), (0, 'raster_i32', 5)):
    outs = [device.empty((nblk, 64), torch.int16 if layout else torch.int32) for _ in range(rot)]
    for tab in (0, 1):
        us = timeit(lambda i: transform.dct_channel_device(planes[i], tab, layout, out=outs[i]), 40, rot)
        print("dct %s tab%d: %.1f us  %.1f Gpix/s  %.0f GB/s" % (name, tab, us, H*W/us/1e3, H*W*bpp/us/1e3))
    recs = [device.empty((H, W), torch.uint8) for _ in range(rot)]
    us = timeit(lambda i: transform.inv_dct_channel_device(outs[i], H, W, 0, layout, out=recs[i]), 40, rot)
    print("idct %s: %.1f us  %.1f Gpix/s  %.0f GB/s" % (name, us, H*W/us/1e3, H*W*bpp/us/1e3))
    del outs, recs
# colour
rgbs = [torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device='cuda', generator=g) for _ in range(4)]
ys = [device.empty((H, W), torch.uint8) for _ in range(4)]
crs = [device.empty((H//2, W//2), torch.uint8) for _ in range(4)]
cbs = [device.empty((H//2, W//2), torch.uint8) for _ in range(4)]
def col(i):
    _lib.call("hic_rgb_to_ycrcb420", device.ptr(rgbs[i]), H, W, device.ptr(ys[i]), device.ptr(crs[i]), device.ptr(cbs[i]), device.stream_ptr())
us = timeit(col, 20, 4)
print("rgb->ycrcb420: %.1f us  %.0f GB/s (4.5 B/px)" % (us, H*W*4.5/us/1e3))
# memcpy reference
a = torch.empty(1<<28, dtype=torch.uint8, device='cuda'); b = torch.empty_like(a)
us = timeit(lambda i: b.copy_(a), 20, 1)
print("d2d copy 256MB: %.1f us  %.0f GB/s" % (us, 2*(1<<28)/us/1e3))
