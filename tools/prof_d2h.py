"""dev: int32 device raster -> float64 host array (codec._decode_channel's last step):
D2H of int32 + numpy astype (current), GPU cast + D2H of float64, and D2H of int32 +
astype split over host threads."""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiccup_amd import device  # noqa: E402

r = torch.randint(-1000, 1000, (4320, 7680), dtype=torch.int32, device="cuda")
pool = ThreadPoolExecutor(8)


def cur():
    return device.to_host(r).astype(np.float64)


def gpu_cast():
    return r.to(torch.float64).cpu().numpy()


def threaded():
    h = device.to_host(r)
    out = np.empty(h.shape, np.float64)
    n = h.shape[0]
    parts = [(i * n // 8, (i + 1) * n // 8) for i in range(8)]
    list(pool.map(lambda ab: out.__setitem__(slice(ab[0], ab[1]), h[ab[0]:ab[1]]), parts))
    return out


def pinned():
    return device.to_host_f64(r)


ref = cur()
for f in (cur, gpu_cast, threaded, pinned, cur, gpu_cast, threaded, pinned):
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        o = f()
        ts.append(time.perf_counter() - t)
    assert np.array_equal(o, ref)
    print(f.__name__, round(float(np.median(ts)) * 1e3, 2), "ms", flush=True)
