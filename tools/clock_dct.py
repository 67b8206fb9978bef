"""dev: in-kernel clock of the fused DCT launch (HIC_DCT_DBG must include 256).
Runs the 8K encode back to back for ~2 s, then reads the per-wave s_memtime /
s_memrealtime stamps of the last launch (MI355X_MICROARCH.md DVFS item 6)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from hiccup_amd import pipeline
assert int(os.environ.get("HIC_DCT_DBG", "0")) & 256
enc = pipeline.Encoder(4320, 7680)
g = torch.Generator(device="cuda"); g.manual_seed(3)
x = torch.randint(0, 256, (4320, 7680, 3), dtype=torch.uint8, device="cuda", generator=g)
t0 = time.time(); n = 0
while time.time() - t0 < 2.0:
    for _ in range(50):
        enc.transform(x)
    torch.cuda.synchronize(); n += 50
st = enc.coef["lum"].view(torch.int64).reshape(-1)[: 4 * 3072].cpu().numpy().reshape(-1, 4).astype(np.float64)
st = st[st[:, 3] > st[:, 1]]
clk = (st[:, 2] - st[:, 0]) / (st[:, 3] - st[:, 1]) * 100.0
dur = (st[:, 3] - st[:, 1]) / 100.0
r0 = st[:, 1].min()
starts, ends = (st[:, 1] - r0) / 100.0, (st[:, 3] - r0) / 100.0
print("  start us: p50 %.1f p90 %.1f max %.1f; end us: p10 %.1f p50 %.1f max %.1f" % (
    np.median(starts), np.percentile(starts, 90), starts.max(), np.percentile(ends, 10), np.median(ends), ends.max()))
hist = np.histogram(starts, bins=10)
print("  start histogram:", list(hist[0]), "edges", [round(e, 1) for e in hist[1]])
print("DBG=%s launches=%d waves=%d clock MHz median %.0f p10 %.0f p90 %.0f; wave us median %.1f max %.1f" % (
    os.environ["HIC_DCT_DBG"], n, len(clk), np.median(clk), np.percentile(clk, 10), np.percentile(clk, 90),
    np.median(dur), dur.max()))
