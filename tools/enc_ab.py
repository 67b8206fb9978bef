"""dev: time the fused encoder launch (hic_encode420_u8) on the 8K workload with
rotating inputs (>= 1.2 GB), by the launch's own HIP events.
usage: HICCUP_HIP_LIB=... python tools/enc_ab.py "label:knob=v,..." ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hiccup_amd import _lib, device, pipeline  # noqa: E402

H, W = 4320, 7680


def main():
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    nin = 13
    xs = [torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nin)]
    encs = [pipeline.Encoder(H, W, fused=True) for _ in range(4)]
    algo = H * W * 3 + sum(h * w for h, w in encs[0].shapes.values()) * 2
    lib = os.environ.get("HICCUP_HIP_LIB", "default")
    for spec in sys.argv[1:] or ["default:"]:
        label, _, kv = spec.partition(":")
        kw = {k: int(v) for k, v in (p.split("=") for p in kv.split(",") if p)}
        with _lib.knobs(**kw):
            evs = [device.KernelEvents() for _ in range(24)]
            for i in range(8):
                encs[i % 4].transform(xs[i % nin])
            for i, e in enumerate(evs):
                encs[i % 4].transform(xs[(8 + i) % nin], dct_events=e)
            torch.cuda.synchronize()
            us = np.array([e.elapsed_ms() * 1e3 for e in evs])
        med = float(np.median(us))
        print("%-40s %-20s median %7.2f us  min %7.2f  (%.3f of 8 TB/s)" % (lib.split("/")[-1], label, med, us.min(),
                                                                            algo / med / 8e6), flush=True)


if __name__ == "__main__":
    main()
