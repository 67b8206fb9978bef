"""dev: A/B the forward/inverse kernel variants in one process (interleaved rounds)."""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hiccup_amd import _lib, device, transform
H, W = 4320, 7680
rot = 12
g = torch.Generator(device='cuda'); g.manual_seed(0)
planes = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device='cuda', generator=g) for _ in range(rot)]
nblk = (H // 8) * (W // 8)
outs = {L: [device.empty((nblk, 64), torch.int16 if L else torch.int32) for _ in range(rot)] for L in (0, 1, 2)}
recs = [device.empty((H, W), torch.uint8) for _ in range(rot)]
def t(fn, n=30):
    for i in range(3): fn(i % rot)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n): fn(i % rot)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3
res = {}
for rnd in range(3):
    for L in (2, 1, 0):
        for tab in (0, 1):
            us = t(lambda i: transform.dct_channel_device(planes[i], tab, L, out=outs[L][i]))
            res.setdefault(('dct', L, tab), []).append(us)
    us = t(lambda i: transform.inv_dct_channel_device(outs[2][i], H, W, 0, 2, out=recs[i]))
    res.setdefault(('idct', 2, 0), []).append(us)
for k, v in res.items():
    print(os.environ.get('HIC_DCT_VARIANT', 'default'), k, 'min %.1f us  med %.1f  -> %.0f GB/s (3B/px)' % (min(v), sorted(v)[1], H*W*3/min(v)/1e3))
