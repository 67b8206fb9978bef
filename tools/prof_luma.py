"""Profile driver (dev tool): N launches of the 8K luminance forward pass
(hic_dct_quant_rle_u8_batch, one plane, or `nplanes` planes per launch) on the
dct_path given as argv[2] (1 float64 AAN, 3 packed float32), 8 rotating sets;
argv[4] = 0: records-free (no RLE workspaces, north_star's pass), else with the
tile records."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hiccup_amd import _lib, device  # noqa: E402

H, W = 4320, 7680
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
path = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nplanes = int(sys.argv[3]) if len(sys.argv) > 3 else 1
records = int(sys.argv[4]) if len(sys.argv) > 4 else 1
_lib.set_knob("dct_path", path)
rot = max(2, 8 // nplanes)
g = torch.Generator(device='cuda')
g.manual_seed(0)
sets = []
nblk = (H // 8) * (W // 8)
for _ in range(rot):
    planes = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device='cuda', generator=g) for _ in range(nplanes)]
    outs = [device.empty((nblk, 64), torch.int16) for _ in range(nplanes)]
    wss = [device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64)) for _ in range(nplanes)]
    jobs = (_lib.DctPlaneJob * nplanes)()
    for i in range(nplanes):
        jobs[i] = _lib.DctPlaneJob(planes[i].data_ptr(), H, W, W, 0, outs[i].data_ptr(),
                                   wss[i].data_ptr() if records else 0)
    sets.append((planes, outs, wss, jobs))
for i in range(n):
    _lib.call("hic_dct_quant_rle_u8_batch", nplanes, sets[i % rot][3], 15, device.stream_ptr(), None, None)
torch.cuda.synchronize()
