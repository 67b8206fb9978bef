"""A/B of the fused encoder's transform on one GPU (dev tool): float64 AAN
(encode_dct 0) against integer MFMA (encode_dct 1) -- one-stream launch time of
k_encode420 (its own events) and the 4-stream 8K step, alternating."""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from hiccup_amd import _lib, device, pipeline  # noqa: E402

H, W = 4320, 7680


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nin = 12
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    xs = [torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nin)]
    encs = [pipeline.Encoder(H, W) for _ in range(4)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(3)]
    for r in range(reps):
        for dm in (1, 0):
            with _lib.knobs(encode_dct=dm):
                evs = [device.KernelEvents() for _ in range(16)]
                for j in range(24):
                    encs[j % 4].encode(xs[j % nin], dct_events=evs[j - 8] if j >= 8 else None)
                torch.cuda.synchronize()
                us = float(np.median([e.elapsed_ms() for e in evs])) * 1e3
                for j in range(8):
                    with torch.cuda.stream(streams[j % 4]):
                        encs[j % 4].encode(xs[j % nin])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for j in range(40):
                    with torch.cuda.stream(streams[j % 4]):
                        encs[j % 4].encode(xs[(j + 3) % nin])
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 40 * 1e3
                for e in encs:
                    for ci, c in enumerate(e.counts.cpu().tolist()):
                        pipeline.check_count(int(c), pipeline.CHANNELS[ci])
            print(json.dumps({"rep": r, "encode_dct": dm, "fused_launch_us": round(us, 2),
                              "ms_per_image_4streams": round(ms, 4), "gpix_s": round(H * W / ms / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
