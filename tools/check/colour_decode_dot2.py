"""Exhaustive check that the decode colour kernel's arithmetic (color.hip
k_ycrcb420_rgb_walk) equals the oracle's pyrUp rounding and OpenCV YCrCb2RGB
restatement (oracle.pyr_up / oracle.ycrcb_to_rgb):
  1. the packed pyrUp sum: every horizontal value carries a bias of -1020 mod 2^16,
     so the vertical sum (weights 8 x 8) is v - 8160 mod 2^16; read as int16 and
     shifted right by 6 it equals ((v + 32) >> 6) - 128 for every reachable sum
     v in [0, 64 * 255];
  2. the colour stage: for all 2^24 (y, cr, cb), each channel is
     sat8((y << 14 | 8192) + dot2((cr - 128, cb - 128), (kCR2x, kCB2x))) >> 14).
Run: python tools/check/colour_decode_dot2.py (a few seconds); also run by
tests/test_cpu_host.py::test_decode_colour_arithmetic_exhaustive."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))

KCR2R, KCR2G, KCB2G, KCB2B = 22987, -11698, -5636, 29049


def packed_round(v):
    """v: pyrUp weighted sums (x64); the kernel's int16 result."""
    biased = (v + 8 * (-1020)) & 0xFFFF
    s16 = np.where(biased >= 1 << 15, biased - (1 << 16), biased)
    return s16 >> 6


def dot2_rgb(y, crs, cbs):
    acc = (y << 14) | 8192
    r = acc + crs * KCR2R
    g = acc + crs * KCR2G + cbs * KCB2G
    b = acc + cbs * KCB2B
    return [np.clip(c >> 14, 0, 255) for c in (r, g, b)]


def check():
    from oracle import oracle
    v = np.arange(64 * 255 + 1, dtype=np.int64)
    assert np.array_equal(packed_round(v), ((v + 32) >> 6) - 128)
    x = np.arange(1 << 24, dtype=np.int64)
    y, cr, cb = x >> 16, (x >> 8) & 255, x & 255
    got = dot2_rgb(y, cr - 128, cb - 128)
    exp = oracle.ycrcb_to_rgb(*(p.astype(np.uint8).reshape(4096, 4096) for p in (y, cr, cb))).reshape(-1, 3)
    return all(np.array_equal(got[c], exp[:, c].astype(np.int64)) for c in range(3))


if __name__ == "__main__":
    print("decode colour arithmetic == oracle (pyrUp rounding, all 2^24 YCrCb):", check())
