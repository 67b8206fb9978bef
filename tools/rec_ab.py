"""8K luma plane pass with and without the fused RLE tile records, per forward path,
beside the memory-only probe of the same byte pattern (dev tool, not product)."""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from hiccup_amd import _lib, device  # noqa: E402

H, W = 4320, 7680
ROT = 1.2e9


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    steps = 24
    px = H * W
    rot = int(np.ceil(ROT / (3 * px)))
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    planes = [torch.randint(0, 256, (H, W), dtype=torch.uint8, device="cuda", generator=g) for _ in range(rot)]
    outs = [device.empty((px // 64, 64), torch.int16) for _ in range(rot)]
    wss = [device.workspace(_lib.load().hic_rle_workspace_bytes(px // 64, 64)) for _ in range(rot)]
    evs = [device.KernelEvents() for _ in range(steps)]

    def timed(launch):
        for i in range(steps + 3):
            ev = evs[i - 3] if i >= 3 else None
            launch(i, ev.start if ev else None, ev.stop if ev else None)
        torch.cuda.synchronize()
        return round(float(np.median([e.elapsed_ms() for e in evs])) * 1e3, 2)

    arms = {
        "records": lambda i, a, b: _lib.call("hic_dct_quant_rle_u8", device.ptr(planes[i % rot]), H, W, W, 0, 15,
                                             device.ptr(outs[i % rot]), device.ptr(wss[i % rot]),
                                             device.stream_ptr(), a, b),
        "no_records": lambda i, a, b: _lib.call("hic_dct_quant_u8_timed", device.ptr(planes[i % rot]), H, W, W, 0,
                                                _lib.LAYOUT_ZIGZAG_I16, device.ptr(outs[i % rot]),
                                                device.stream_ptr(), a, b),
    }
    for r in range(reps):
        row = {"rep": r}
        for wpc in (12, 16):
            row["probe_wpc%d" % wpc] = timed(lambda i, a, b: _lib.call(
                "hic_probe_plane", device.ptr(planes[i % rot]), H, W, device.ptr(outs[i % rot]), wpc,
                device.stream_ptr(), a, b))
        for path, var in ((1, 0), (5, 0), (5, 3)):
            with _lib.knobs(dct_path=path, dct_mfma=var):
                for k, f in arms.items():
                    row["p%d_v%d_%s" % (path, var, k)] = timed(f)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
