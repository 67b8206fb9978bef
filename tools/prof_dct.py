"""Profile driver (dev tool): N launches of the 8K forward DCT pass exactly as the
pipeline / bench launch it (hic_dct_quant_rle_u8_batch over Y 4320x7680 + Cr, Cb
2160x3840: DCT + quantize + zig-zag + RLE tile records, one launch), then N
inverse launches of the luminance plane."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hiccup_amd import _lib, device, transform  # noqa: E402

H, W = 4320, 7680
SHAPES = [(H, W, 0), (H // 2, W // 2, 1), (H // 2, W // 2, 1)]
rot = 8
n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
g = torch.Generator(device='cuda')
g.manual_seed(0)
sets = []
for _ in range(rot):
    planes, outs, wss = [], [], []
    for h, w, _t in SHAPES:
        nblk = (h // 8) * (w // 8)
        planes.append(torch.randint(0, 256, (h, w), dtype=torch.uint8, device='cuda', generator=g))
        outs.append(device.empty((nblk, 64), torch.int16))
        wss.append(device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64)))
    jobs = (_lib.DctPlaneJob * 3)()
    for i, (h, w, t) in enumerate(SHAPES):
        jobs[i] = _lib.DctPlaneJob(planes[i].data_ptr(), h, w, w, t, outs[i].data_ptr(), wss[i].data_ptr())
    sets.append((planes, outs, wss, jobs))
recs = [device.empty((H, W), torch.uint8) for _ in range(rot)]
for i in range(n):
    _lib.call("hic_dct_quant_rle_u8_batch", 3, sets[i % rot][3], 15, device.stream_ptr(), None, None)
for i in range(n):
    transform.inv_dct_channel_device(sets[i % rot][1][0], H, W, 0, _lib.LAYOUT_ZIGZAG_I16, out=recs[i % rot])
torch.cuda.synchronize()
