"""Exhaustive check (all 2^24 RGB triples) that the fused encoder's colour
arithmetic (encode.hip ycc8: two v_dot4_u32_u8 on the high / low bytes of the 4x
luma weights, chroma on 4x-scaled weights clamped to [0, 2^24 - 1] and read from
byte 2) equals the oracle's OpenCV RGB2YCrCb restatement (oracle.rgb_to_ycrcb).
Run: python tools/check/colour_dot4.py (about 5 s); also run by
tests/test_cpu_host.py::test_fused_colour_arithmetic_exhaustive."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def dot4_ycc(r, g, b):
    w4 = (4 * 4899, 4 * 9617, 4 * 1868)
    lo = [w & 255 for w in w4]
    hi = [w >> 8 for w in w4]
    L = r * lo[0] + g * lo[1] + b * lo[2] + 32768
    H = r * hi[0] + g * hi[1] + b * hi[2] + (L >> 8)
    assert int(H.max()) < 1 << 16
    y = (H >> 8) & 255
    cc4 = 4 * ((128 << 14) + (1 << 13))
    cr = np.clip((r - y) * (4 * 11682) + cc4, 0, 0xFFFFFF) >> 16
    cb = np.clip((b - y) * (4 * 9241) + cc4, 0, 0xFFFFFF) >> 16
    return y, cr, cb


def check():
    from oracle import oracle
    v = np.arange(1 << 24, dtype=np.int64)
    r, g, b = v >> 16, (v >> 8) & 255, v & 255
    y, cr, cb = dot4_ycc(r, g, b)
    img = np.stack([r, g, b], axis=-1).astype(np.uint8).reshape(4096, 4096, 3)
    ry, rcr, rcb = (p.reshape(-1).astype(np.int64) for p in oracle.rgb_to_ycrcb(img))
    assert np.array_equal(ry, y) and np.array_equal(rcr, cr) and np.array_equal(rcb, cb)
    return True


if __name__ == "__main__":
    print("dot4 colour arithmetic == oracle on all 2^24 inputs:", check())
