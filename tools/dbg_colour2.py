"""dev: dump colour outputs for offline analysis."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hiccup_amd import compression, device
H, W = 18, 512
rng = np.random.default_rng(8)
rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
y, cr, cb = compression.ycrcb420_device(device.to_device(rgb))
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/dbg_colour.npz", rgb=rgb, y=device.to_host(y), cr=device.to_host(cr), cb=device.to_host(cb))
