"""dev: the reference-API entry points at 8K from host arrays (compression.jpeg_compression /
jpeg_decompression, codec.jpeg_encode / jpeg_decode): wall time per call, median of 3."""
import os
import pickle
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hiccup_amd import codec, compression, hicimage, settings  # noqa: E402

settings.DEBUG = False
rgb = np.random.default_rng(1).integers(0, 256, (4320, 7680, 3), dtype=np.uint8)


def med(f, n=3):
    ts = []
    for _ in range(n + 1):
        t = time.perf_counter()
        r = f()
        ts.append(time.perf_counter() - t)
    return r, round(float(np.median(ts[1:])) * 1e3, 1)


ci, t_comp = med(lambda: compression.jpeg_compression(rgb))
hic, t_enc = med(lambda: codec.jpeg_encode(ci))
blob = pickle.dumps(hic.byte_stream())
img = hicimage.HicImage.from_bytes(hicimage._loads(blob))
ci2, t_dec = med(lambda: codec.jpeg_decode(img))
rec, t_decomp = med(lambda: compression.jpeg_decompression(ci2))
same = all(np.array_equal(a, b) for a, b in zip(ci.as_dict.values(), ci2.as_dict.values()))
print({"compress_ms": t_comp, "jpeg_encode_ms": t_enc, "jpeg_decode_ms": t_dec, "decompress_ms": t_decomp,
       "planes_roundtrip_equal": same, "rgb_shape": list(rec.shape)}, flush=True)
