"""dev: in-kernel clock + wave timeline of the fused DCT launch (HIC_DCT_DBG must
include 256).  Runs the 8K encode back to back for ~2 s (COLD=1: rotating inputs
and encoders as bench.py, so HBM is cold), then reads the per-wave s_memtime /
s_memrealtime stamps of the last launch (MI355X_MICROARCH.md DVFS item 6) and
compares the waves' span with the launch's own begin / end timestamps."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from hiccup_amd import device, pipeline
assert int(os.environ.get("HIC_DCT_DBG", "0")) & 256
cold = os.environ.get("COLD") == "1"
nenc, nin = (4, 12) if cold else (1, 1)
encs = [pipeline.Encoder(4320, 7680) for _ in range(nenc)]
g = torch.Generator(device="cuda"); g.manual_seed(3)
xs = [torch.randint(0, 256, (4320, 7680, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nin)]
ev = device.KernelEvents()
t0 = time.time(); n = 0
while time.time() - t0 < 2.0:
    for _ in range(48):
        encs[n % nenc].transform(xs[n % nin]); n += 1
    torch.cuda.synchronize()
last = encs[(n - 1) % nenc]
last.transform(xs[n % nin], dct_events=ev)
torch.cuda.synchronize()
st = last.coef["lum"].view(torch.int64).reshape(-1)[: 4 * 3072].cpu().numpy().reshape(-1, 4).astype(np.float64)
st = st[st[:, 3] > st[:, 1]]
clk = (st[:, 2] - st[:, 0]) / (st[:, 3] - st[:, 1]) * 100.0
r0 = st[:, 1].min()
starts, ends = (st[:, 1] - r0) / 100.0, (st[:, 3] - r0) / 100.0
print("DBG=%s cold=%d waves=%d clock MHz median %.0f; start us p50 %.1f max %.1f; end us p10 %.1f p50 %.1f max %.1f; "
      "launch (events) %.1f us" % (os.environ["HIC_DCT_DBG"], cold, len(clk), np.median(clk), np.median(starts),
                                   starts.max(), np.percentile(ends, 10), np.median(ends), ends.max(),
                                   ev.elapsed_ms() * 1e3))
