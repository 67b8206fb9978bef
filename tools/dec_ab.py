"""Decode A/B (dev tool): the 16K decode from the encoder-side index (Decoder.decode
with index=: per plane hic_rle_decode_idct_u8_indexed, then the colour kernel),
timed alone after one encode, and the 16K round trip; run once per library
(HICCUP_HIP_LIB), arms alternating in separate processes by tools/dec_ab.sh."""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from hiccup_amd import pipeline  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = torch.randint(0, 256, (n, n, 3), dtype=torch.uint8, device="cuda", generator=g)
    enc, dec = pipeline.Encoder(n, n, index=True), pipeline.Decoder(n, n)
    enc.encode(x)
    torch.cuda.synchronize()
    dec.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out = dec.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dec.check_status()
    h = int(out[::97, ::89].float().sum().item())
    del enc, dec, x, out
    torch.cuda.empty_cache()
    rt = bench.extra_16k_roundtrip() if n == 16384 and "--no-roundtrip" not in sys.argv else None
    print(json.dumps({"lib": os.path.basename(os.environ.get("HICCUP_HIP_LIB", "libhiccup_hip.so")),
                      "decode_ms_median": round(float(np.median(ts)) * 1e3, 3), "checksum": h,
                      "roundtrip_ms": rt["ms_per_roundtrip"] if rt else None}), flush=True)


if __name__ == "__main__":
    main()
