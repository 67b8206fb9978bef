"""dev: where does the colour kernel disagree with the restatement?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hiccup_amd import compression, device
import oracle.oracle_c as orcc
for H, W in ((1080, 1920), (64, 512), (18, 512)):
    rng = np.random.default_rng(8)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    y, cr, cb = compression.ycrcb420_device(device.to_device(rgb))
    ry, rcr, rcb = orcc.rgb_to_ycrcb(rgb)
    for name, got, exp in (("y", device.to_host(y), ry), ("cr", device.to_host(cr), orcc.pyr_down(rcr)),
                           ("cb", device.to_host(cb), orcc.pyr_down(rcb))):
        bad = np.argwhere(got != exp)
        print(H, W, name, len(bad))
        if len(bad):
            print("  rows", np.unique(bad[:, 0] % 8, return_counts=True))
            print("  cols%128", np.unique(bad[:, 1] % 128, return_counts=True))
            print("  first", bad[:10].tolist())
