"""Profile driver (dev tool): N launches of each DCT kernel variant on 8K Y."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hiccup_amd import _lib, device, transform
H, W = 4320, 7680
rot = 12
g = torch.Generator(device='cuda'); g.manual_seed(0)
planes = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device='cuda', generator=g) for _ in range(rot)]
nblk = (H // 8) * (W // 8)
outs = [device.empty((nblk, 64), torch.int16) for _ in range(rot)]
recs = [device.empty((H, W), torch.uint8) for _ in range(rot)]
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 24):
    transform.dct_channel_device(planes[i % rot], 0, _lib.LAYOUT_ZIGZAG_I16, out=outs[i % rot])
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 24):
    transform.inv_dct_channel_device(outs[i % rot], H, W, 0, _lib.LAYOUT_ZIGZAG_I16, out=recs[i % rot])
torch.cuda.synchronize()
