"""dev: per-block cost of the forward kernel with HBM-cold (rotating) vs cache-hot buffers."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hiccup_amd import _lib, device, transform
def run(H, W, rot, n=40):
    g = torch.Generator(device='cuda'); g.manual_seed(0)
    planes = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device='cuda', generator=g) for _ in range(rot)]
    nblk = (H // 8) * (W // 8)
    outs = [device.empty((nblk, 64), torch.int16) for _ in range(rot)]
    f = lambda i: transform.dct_channel_device(planes[i % rot], 0, 2, out=outs[i % rot])
    for i in range(3): f(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n): f(i)
    e.record(); torch.cuda.synchronize()
    us = s.elapsed_time(e) / n * 1e3
    print("%s %dx%d rot=%d: %.1f us  %.1f ps/block" % (os.environ.get('HIC_DCT_PATH', 'aan'), H, W, rot, us, us * 1e6 / nblk))
run(4320, 7680, 12)
run(4320, 7680, 1)
run(2048, 4096, 1)
run(1024, 2048, 1)
