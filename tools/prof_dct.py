"""Profile driver (dev tool): N launches of the 8K luminance forward kernel exactly
as the pipeline / bench launch it (hic_dct_quant_rle_u8: DCT + quantize + zig-zag
+ RLE tile records), then N inverse launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hiccup_amd import _lib, device, transform  # noqa: E402

H, W = 4320, 7680
rot = 12
n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
g = torch.Generator(device='cuda')
g.manual_seed(0)
planes = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device='cuda', generator=g) for _ in range(rot)]
nblk = (H // 8) * (W // 8)
outs = [device.empty((nblk, 64), torch.int16) for _ in range(rot)]
ws = device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64))
recs = [device.empty((H, W), torch.uint8) for _ in range(rot)]
for i in range(n):
    _lib.call("hic_dct_quant_rle_u8", device.ptr(planes[i % rot]), H, W, W, 0, 15, device.ptr(outs[i % rot]),
              device.ptr(ws), device.stream_ptr(), None, None)
for i in range(n):
    transform.inv_dct_channel_device(outs[i % rot], H, W, 0, _lib.LAYOUT_ZIGZAG_I16, out=recs[i % rot])
torch.cuda.synchronize()
