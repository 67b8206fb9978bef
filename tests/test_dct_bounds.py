"""The exactness proof of the fast forward DCT paths, pinned (CPU).

tools/check/dct_bounds.py derives rigorous forward-error bounds for every fast
path: E64 for the float64 AAN path the product runs, and E1 /
E2 for the packed-float32 path measured in round 5 and removed (commit ae5c500
compiled its windows from tools/check/dct_windows.h, kept as the proof's output).
These tests re-run the derivation and fail when the committed header and the proof
drift apart (a one-ulp edit of any constant), or when a path's bound no longer sits
inside its margin.
"""
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools", "check"))
import dct_bounds  # noqa: E402

HEADER = os.path.join(REPO, "tools", "check", "dct_windows.h")


def test_windows_header_matches_proof(tmp_path):
    out = tmp_path / "dct_windows.h"
    dct_bounds.emit(str(out))
    assert out.read_text() == open(HEADER).read(), \
        "dct_windows.h differs from tools/check/dct_bounds.py --emit: regenerate it (and re-check the proof)"


def _header_floats(name):
    text = open(HEADER).read()
    body = text[text.index("constexpr float %s[2][64]" % name):]
    body = body[body.index("{") + 1:body.index("};")]
    vals = [float.fromhex(v.strip().rstrip("f")) for v in body.replace("{", "").replace("}", "").split(",")
            if v.strip()]
    assert len(vals) == 128
    return np.array(vals).reshape(2, 64)


def test_float32_windows_cover_their_bounds():
    """kThr32 = float32(1/2 - W1) rounded down, W1 = E1 + EP/T + test rounding: an
    unflagged |d| <= kThr32 is more than W1 from a tie; the packed path's squared
    threshold must not exceed kThr32^2 (then |d| > kThr32 implies d^2 > kThr32Sq)."""
    e1, e2, ep, W1, W2 = dct_bounds.windows()
    thr, thr_sq = _header_floats("kThr32"), _header_floats("kThr32Sq")
    for t in range(2):
        w = W1[t].reshape(64)
        assert np.all(thr[t] <= 0.5 - w), t
        assert np.all(thr[t] > 0.5 - w - 2.0 ** -24), t  # tight: not rounded down by more than an ulp
        assert np.all(thr_sq[t] <= thr[t].astype(np.float64) ** 2), t
        assert np.all(w < 2.0 ** -9), t  # windows stay small: flags are rare
        # the float32 products / fma residuals the test relies on stay exact (|e| < 2^12)
    # the fallback tier's window (float64 dot product) sits inside its 2^-kW2Log2 test
    text = open(HEADER).read()
    k = int(text[text.index("kW2Log2 = ") + 10:].split(";")[0])
    assert W2.max() < 2.0 ** -k


def test_float32_constants_within_the_proof_model():
    """E1 (dct_bounds.py) models every float32 constant of the packed path as within
    2^-24 |c| of its real value: the four AAN factors (the packed kernel rounded dct_core.h's
    float64 kA1 / kA2 / kA4 / kA5 to float32) and the quantiser constants kR32 =
    float32(S_u S_v / T).  Checked against 50-digit values."""
    import re
    import mpmath as mp
    mp.mp.dps = 50
    core = open(os.path.join(REPO, "hiccup_amd", "csrc", "dct_core.h")).read()
    hexv = dict(re.findall(r"constexpr double (kA[1245]) = (0x[0-9a-fp.+-]+);", core))
    c8, c38 = mp.cos(mp.pi / 8), mp.cos(3 * mp.pi / 8)
    exact = {"kA1": mp.cos(mp.pi / 4), "kA2": c8 - c38, "kA4": c8 + c38, "kA5": c38}
    assert set(hexv) == set(exact)
    for name, h in hexv.items():
        k32 = float(np.float32(float.fromhex(h)))
        assert abs(mp.mpf(k32) - exact[name]) <= mp.mpf(2) ** -24 * abs(exact[name]), name
    r32 = _header_floats("kR32")
    S = [mp.mpf(2)] + [1 / mp.cos(k * mp.pi / 16) for k in range(1, 8)]
    for t in range(2):
        for i in range(64):
            R = S[i // 8] * S[i % 8] / dct_bounds.QT[t][i]
            assert abs(mp.mpf(float(r32[t, i])) - R) <= mp.mpf(2) ** -24 * R, (t, i)


def test_float64_fast_path_margin():
    """The float64 AAN path (k_encode420, dct_path 1): estimate + pocketfft + roundings
    < 2.5 * 2^-32, the qfast flag margin."""
    e64, ep = dct_bounds.E64(), dct_bounds.EP()
    for t in range(2):
        T = np.array(dct_bounds.QT[t], float).reshape(8, 8)
        tot = e64[t] + ep / T + 2.0 ** -33 + 2.0 ** -41
        tot[0, 0] = tot[4, 4] = 0.0  # computed exactly
        assert tot.max() < 2.5 * 2.0 ** -32, (t, math.log2(tot.max()))


def test_bounds_are_sensitive():
    """Sanity of the error model itself: dropping a rounding makes E1 smaller, and
    the float32 bound is orders above the float64 one."""
    e1 = dct_bounds.E1()
    e64 = dct_bounds.E64()
    assert np.all(e1[:, 1:, :] > 1e3 * e64[:, 1:, :])


def test_wire_widths_header_matches_proof():
    """The gather's wire widths (hiccup_amd/csrc/wire_widths.h) are what
    tools/check/wire_widths.py derives from the DCT bound, and every width holds
    the largest quantised value its slot can take (checked against a brute-force
    maximiser: the +-128 sign pattern of the slot's basis function)."""
    import wire_widths
    header = os.path.join(REPO, "hiccup_amd", "csrc", "wire_widths.h")
    assert wire_widths.emit() == open(header).read(), \
        "wire_widths.h differs from tools/check/wire_widths.py --emit: regenerate it"
    for t, table in enumerate((wire_widths.LUM, wire_widths.CHROMA)):
        w = wire_widths.widths(table)
        for z in range(64):
            u, v = divmod(wire_widths.ZZ[z], 8)
            cu = np.cos(np.pi * u * (2 * np.arange(8) + 1) / 16)
            cv = np.cos(np.pi * v * (2 * np.arange(8) + 1) / 16)
            # the pixel block maximising |y|: +-128 by the sign of the basis
            x = np.where(np.outer(cu, cv) >= 0, 127, -128)
            y = 4 * float(np.sum(x * np.outer(cu, cv)))
            q = abs(round(y / table[u][v]))
            assert q < (1 << (w[z] - 1)), (t, z, q, w[z])
        assert sum(w) == (637, 597)[t]
