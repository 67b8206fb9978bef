"""dev: where the drop-in API's wall time goes at 8K: each of
compression.jpeg_compression, codec.jpeg_encode, codec.jpeg_decode and
compression.jpeg_decompression from host arrays, one untimed call then one under
cProfile (top functions by cumulative time), and the PCIe floor of the bytes each
call moves (host <-> device rates measured here with pinned buffers).
usage: python3 tools/api_profile.py [H W]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hiccup_amd import codec, compression, settings  # noqa: E402

H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4320, 7680)
settings.DEBUG = False
rgb = np.random.default_rng(1).integers(0, 256, (H, W, 3), dtype=np.uint8)


def rate(nbytes=256 << 20):
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = {}
    for name, f in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(4):
            f()
        torch.cuda.synchronize()
        out[name] = 4 * nbytes / (time.perf_counter() - t) / 1e9
    return out


r = rate()
print("pinned rates GB/s:", {k: round(v, 1) for k, v in r.items()})
calls = [("jpeg_compression", lambda: compression.jpeg_compression(rgb))]
ci = compression.jpeg_compression(rgb)
calls.append(("jpeg_encode", lambda: codec.jpeg_encode(ci)))
hic = codec.jpeg_encode(ci)
calls.append(("jpeg_decode", lambda: codec.jpeg_decode(hic)))
ci2 = codec.jpeg_decode(hic)
calls.append(("jpeg_decompression", lambda: compression.jpeg_decompression(ci2)))
px = H * W
bits = sum(len(p.packed_bits()[0]) for p in hic.payloads[9:18])
moved = {"jpeg_compression": (3 * px, 4 * px * 3 // 2), "jpeg_encode": (4 * px * 3 // 2, bits),
         "jpeg_decode": (bits, 8 * px * 3 // 2), "jpeg_decompression": (8 * px * 3 // 2, 3 * px)}
for name, f in calls:
    f()
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        f()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t)
    wall = float(np.median(walls))
    up, down = moved[name]
    floor = up / r["h2d"] / 1e6 + down / r["d2h"] / 1e6
    print("== %s: %.1f ms wall (median of 5; %s); PCIe floor %.1f ms (%.0f MB up, %.0f MB down), ratio %.2f"
          % (name, wall * 1e3, " ".join("%.1f" % (w * 1e3) for w in walls), floor, up / 1e6, down / 1e6,
             wall * 1e3 / floor))
    pr = cProfile.Profile()
    pr.enable()
    f()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(22)
    print("\n".join(l for l in s.getvalue().splitlines() if l.strip())[:4000])
