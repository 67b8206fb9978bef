"""A/B timing of the 8K three-plane forward DCT launch (dev tool): the pass bench.py
reports as its roofline kernel (hic_dct_quant_rle_u8_batch over Y 4320x7680 + Cr, Cb
2160x3840), timed by the launch's own HIP events over rotating inputs (>= 1 GB).
usage: python tools/dct_ab.py "label:knob=v,knob=v" ...   (dev knobs need
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_dev.so)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hiccup_amd import _lib, device  # noqa: E402

H, W = 4320, 7680
SHAPES = [(H, W, 0), (H // 2, W // 2, 1), (H // 2, W // 2, 1)]
ROT = 8


def make_sets():
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    sets = []
    for _ in range(ROT):
        planes, outs, wss = [], [], []
        for h, w, _t in SHAPES:
            nblk = (h // 8) * (w // 8)
            planes.append(torch.randint(0, 256, (h, w), dtype=torch.uint8, device="cuda", generator=g))
            outs.append(device.empty((nblk, 64), torch.int16))
            wss.append(device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64)))
        jobs = (_lib.DctPlaneJob * 3)()
        for i, (h, w, t) in enumerate(SHAPES):
            jobs[i] = _lib.DctPlaneJob(planes[i].data_ptr(), h, w, w, t, outs[i].data_ptr(), wss[i].data_ptr())
        sets.append((planes, outs, wss, jobs))
    return sets


def time_variant(sets, n=24, warm=8, planes=3):
    evs = [device.KernelEvents() for _ in range(n)]
    for i in range(warm):
        _lib.call("hic_dct_quant_rle_u8_batch", planes, sets[i % ROT][3], 15, device.stream_ptr(), None, None)
    for i in range(n):
        e = evs[i]
        _lib.call("hic_dct_quant_rle_u8_batch", planes, sets[(warm + i) % ROT][3], 15, device.stream_ptr(), e.start,
                  e.stop)
    torch.cuda.synchronize()
    return np.array([e.elapsed_ms() * 1e3 for e in evs])


def main():
    torch.cuda.set_device(0)
    sets = make_sets()
    algo = sum(h * w for h, w, _ in SHAPES) * 3
    for spec in sys.argv[1:] or ["default:"]:
        label, _, kv = spec.partition(":")
        kw = {k: int(v) for k, v in (p.split("=") for p in kv.split(",") if p)}
        planes = kw.pop("planes", 3)
        with _lib.knobs(**kw):
            us = time_variant(sets, planes=planes)
        med = float(np.median(us))
        a = algo if planes == 3 else H * W * 3
        print("%-28s median %7.2f us  min %7.2f  (%.3f of 8 TB/s)" % (label, med, us.min(), a / med / 8e6),
              flush=True)


if __name__ == "__main__":
    main()
