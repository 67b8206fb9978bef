"""The integer-MFMA forward DCT + quantiser (dct_mfma.h, k_dct_mfma in dct.hip):
its constant matrices, the proof that an unflagged coefficient equals the
reference's, and a bit-level numpy emulation of the kernel's arithmetic.  Not
product code: `--emit` writes hiccup_amd/csrc/dct_mfma_tables.h, and
tests/test_dct_bounds.py re-runs the derivation and diffs the header.

The reference (hiccup/transform.py:67-84 dct2, quantization.py:47-52,80-81)
computes, per 8x8 block of centred pixels x_ij = p_ij - 128,
    y_uv = sum_ij C_uv,ij x_ij,   C_uv,ij = 4 cos(pi u (2i+1)/16) cos(pi v (2j+1)/16)
with scipy's pocketfft in float64 (y_pf), then q_uv = rint(fl(y_pf / T_uv)).

The kernel evaluates the whole 64 x 64 linear map as one integer contraction on
the matrix cores (v_mfma_i32_16x16x64_i8):
  * x = p XOR 0x80 is p - 128 as an exact int8;
  * A_z,k = round(2^32 C_uv,k / T_uv) (row z = zig-zag slot of (u, v), column k =
    8 i + j) is an integer below 2^31 in magnitude, split into four balanced
    base-256 digits a_0..a_3 in [-128, 127] (A = sum 2^(8d) a_d);
  * S_d = sum_k a_d,k x_k is computed EXACTLY (int8 x int8 -> int32 MFMA, |S_d| <= 2^20);
  * the four digit products are independent MFMAs (c0 and 2^15 ride in the
    accumulator inputs of digits 0 and 2) combined with ONE truncating shift:
        R = ((S_0 + c0 + (S_1 << 8)) >> 13) + ((S_2 + 2^15) << 3) + (S_3 << 11)
    so R = (S + c0) / 2^13 + 2^18 - eps with eps in [0, 1): R / 2^19 estimates
    y/T + 1/2 in units of 2^-19 (S = sum_d 2^(8d) S_d = sum_k A_k x_k; the 2^16 S_2
    and 2^24 S_3 terms are multiples of 2^13, so the floor only cuts S_0 + 2^8 S_1).
  * q = R >> 19 (floor), flagged when R mod 2^19 < L.
Proof (windows() below): |S / 2^32 - y/T| <= EA (A's rounding, summed exactly
over the 64 columns with |x| <= 128), |y/T - fl(y_pf/T)| <= EQ (pocketfft's
float64 error EP from dct_bounds.py, and the division's rounding).  With
o = c0 / 2^13 (R units) an unflagged R gives
    n + (L - o)/2^19 <= S/2^32 + 1/2 < n + 1 - (o - 1)/2^19,
so if (L - o) / 2^19 > EA + EQ and (o - 1) / 2^19 > EA + EQ the reference's
fl(y_pf/T) + 1/2 lies strictly inside (n, n + 1): its rint is n, no tie.
Special rows:
  * z = 0 (DC): A = 2^30 for both tables (the pixel sum, exact): the kernel
    recovers X = sum x = (R - 2^18) >> 17 and rounds 4 X / T itself (dc_quant);
  * (4,4) luminance (z = 39): y = 2 (a signed pixel sum), so y/T = K/34 is
    flagged exactly at its ties (K = 17 mod 34, ~3 % of random blocks), which
    pocketfft's own roundings decide (pf_y44 from the rows' signed sums);
  * everything else flagged sends the set to the float64 AAN path (dct_core.h).
"""
import math
import os
import sys

import mpmath
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import dct_bounds  # noqa: E402

mpmath.mp.dps = 60
QT = dct_bounds.QT
# transposed zig-zag: zig-zag slot -> raster index (dct_core.h ZZ, transform.py:106-124)
ZZ = [0, 8, 1, 2, 9, 16, 24, 17, 10, 3, 4, 11, 18, 25, 32, 40, 33, 26, 19, 12, 5, 6, 13, 20, 27, 34, 41, 48, 56, 49,
      42, 35, 28, 21, 14, 7, 15, 22, 29, 36, 43, 50, 57, 58, 51, 44, 37, 30, 23, 31, 38, 45, 52, 59, 60, 53, 46, 39,
      47, 54, 61, 62, 55, 63]
Z44 = ZZ.index(36)
SCALE = 32          # A = round(2^32 C / T)
RBITS = 19          # R = 2^19 (y/T + 1/2) - eps
HALF2 = 1 << 15     # 1/2 in S2's units (2^-16 of y/T)
DC_A = 1 << 30      # the DC row: 4 / 16 * 2^32 -> the exact pixel sum at 2^30


def _cexact(u, v, i, j):
    return 4 * mpmath.cos(mpmath.pi * u * (2 * i + 1) / 16) * mpmath.cos(mpmath.pi * v * (2 * j + 1) / 16)


def _round_half_even(x):
    f = mpmath.floor(x)
    d = x - f
    if d > 0.5 or (d == 0.5 and int(f) % 2 == 1):
        return int(f) + 1
    return int(f)


def amatrix(t):
    """A[z][k] (python ints) and the exact reals 2^32 C/T it rounds ([z][k])."""
    A, X = [], []
    for z in range(64):
        u, v = divmod(ZZ[z], 8)
        row, ex = [], []
        for k in range(64):
            i, j = divmod(k, 8)
            if z == 0:
                val = mpmath.mpf(DC_A)
            else:
                val = _cexact(u, v, i, j) * mpmath.mpf(2) ** SCALE / QT[t][ZZ[z]]
            a = _round_half_even(val)
            assert -(1 << 31) < a < (1 << 31)
            row.append(a)
            ex.append(val)
        A.append(row)
        X.append(ex)
    return A, X


def limbs(a):
    """Balanced base-256 digits d0..d3 in [-128, 127] with a = sum 256^k d_k."""
    out = []
    for _ in range(3):
        d = ((a + 128) & 255) - 128
        out.append(d)
        a = (a - d) >> 8
    assert -128 <= a <= 127
    out.append(a)
    return out


def EA(t):
    """|S / 2^32 - y/T| <= EA[z] over all centred blocks (|x| <= 128)."""
    A, X = amatrix(t)
    out = []
    for z in range(64):
        s = mpmath.fsum(abs(A[z][k] - X[z][k]) for k in range(64))
        out.append(float(s * 128 / mpmath.mpf(2) ** SCALE) * (1 + 2.0 ** -50))
    return np.array(out)


def ymax(t):
    """max |y/T| per zig-zag slot over the input box (x in [-128, 127])."""
    out = []
    for z in range(64):
        u, v = divmod(ZZ[z], 8)
        cu = np.cos(np.pi * u * (2 * np.arange(8) + 1) / 16)
        cv = np.cos(np.pi * v * (2 * np.arange(8) + 1) / 16)
        out.append(4 * 128 * np.abs(np.outer(cu, cv)).sum() / QT[t][ZZ[z]])
    return np.array(out)


def windows():
    """(o, L, margin): offset c0 = o 2^13, flag L, and the proof's slack (R units)."""
    ep = dct_bounds.EP().reshape(64)
    m = 0.0
    for t in range(2):
        ea = EA(t)
        T = np.array([QT[t][ZZ[z]] for z in range(64)], float)
        eq = np.array([ep[ZZ[z]] for z in range(64)]) / T + 2.0 ** -53 * ymax(t) + 2.0 ** -60
        tot = ea + eq
        tot[0] = 0.0                      # DC: exact, rounded apart
        m = max(m, float(tot.max()) * 2.0 ** RBITS)
    # o - 1 > m and L - o > m, o a multiple of 2^-13 (c0 an integer), L an integer
    o = 1.0 + m + 2.0 ** -6
    o = math.ceil(o * 2 ** 13) / 2 ** 13
    L = math.floor(o + m) + 1
    assert o - 1 > m and L - o > m
    return o, L, m


def bounds_ok():
    """Every accumulator and R stay inside int32 (asserts; returns the maxima)."""
    mx = {}
    for t in range(2):
        A, _ = amatrix(t)
        for z in range(64):
            d = limbs(A[z][0])  # noqa: F841  (range checked in limbs)
            s = [sum(abs(limbs(A[z][k])[dd]) for k in range(64)) * 128 for dd in range(4)]
            for dd in range(4):
                mx["S%d" % dd] = max(mx.get("S%d" % dd, 0), s[dd])
        yt = ymax(t).max() + 1
        mx["R"] = max(mx.get("R", 0), yt * 2 ** RBITS + 2 ** 18)
    assert mx["R"] < 2 ** 31 and all(mx["S%d" % d] <= 2 ** 20 for d in range(4))
    # D2 = S2 + 256 S3 + 2^15 <= R / 8 + ...: inside int32 with the R bound
    return mx


def emulate(x, t, c0):
    """The kernel's integer arithmetic on centred blocks x[n, 64] (raster k = 8i + j):
    returns (q[n, 64] zig-zag, fr[n, 64] = R mod 2^19, R[n, 64])."""
    A, _ = amatrix(t)
    L4 = np.array([[limbs(A[z][k]) for k in range(64)] for z in range(64)], dtype=np.int64)  # [z][k][d]
    x = x.astype(np.int64)
    S = [x @ L4[:, :, d].T for d in range(4)]  # [n, z]
    # every intermediate stays inside int32 (the kernel's arithmetic wraps nowhere)
    lo = (S[1] << 8) + S[0] + c0
    assert np.abs(lo).max() < 2 ** 31
    R = (lo >> 13) + ((S[2] + HALF2) << 3) + (S[3] << 11)
    assert np.abs(R).max() < 2 ** 31
    q = R >> RBITS
    fr = R & ((1 << RBITS) - 1)
    return q, fr, R


def dc_quant(X, T):
    """round-half-even(4 X / T) in integers (dct_core.h dc_quant)."""
    a = 8 * X + T
    q = np.floor_divide(a, 2 * T)
    tie = (a == q * 2 * T) & (q % 2 != 0)
    return np.where(tie, q - 1, q)


def emit(path):
    o, L, m = windows()
    bounds_ok()
    c0 = int(round(o * 2 ** 13))
    lines = ["// GENERATED by tools/check/dct_mfma.py --emit (do not edit): the integer-MFMA",
             "// forward DCT's constant matrices and flag window, with the proof in that script",
             "// (DESIGN.md section 5).  A[t][z][k] = round(2^32 C_uv,k / T[t][uv]), (u, v) = the",
             "// raster index of zig-zag slot z, k = 8 i + j the pixel of the block; row 0 is",
             "// 2^30 (the exact pixel sum) for both tables.",
             "#pragma once", "#include <stdint.h>", "", "namespace hic {", "namespace {", ""]
    lines.append("// proof slack: max (EA + EQ) = %.4f units of 2^-19; offset o = %.6f, flag L = %d" % (m, o, L))
    lines.append("constexpr int32_t kMfmaC0 = %d;  // o * 2^13: D0's accumulator input" % c0)
    lines.append("constexpr uint32_t kMfmaL = %du;  // flagged iff (R & (2^19 - 1)) < kMfmaL" % L)
    lines.append("constexpr int kMfmaZ44 = %d;  // zig-zag slot of (4,4)" % Z44)
    lines.append("constexpr int32_t kMfmaA[2][64][64] = {")
    for t in range(2):
        A, _ = amatrix(t)
        lines.append("  {")
        for z in range(64):
            lines.append("    {" + ", ".join(str(a) for a in A[z]) + "},")
        lines.append("  },")
    lines.append("};")
    lines += ["", "}  // namespace", "}  // namespace hic", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--emit":
        emit(sys.argv[2])
        sys.exit(0)
    o, L, m = windows()
    print("max (EA + EQ) = %.4f R units (2^%.2f); o = %.6f, L = %d" % (m, math.log2(m * 2.0 ** -19), o, L))
    for t in range(2):
        print("table", t, "log2 EA per slot:", np.round(np.log2(EA(t)[1:]), 2))
    print("int32 maxima:", {k: math.log2(v) for k, v in bounds_ok().items()})
    print("expected flags per block (random data, %d-unit window over 62 slots): %.2e" % (L, 62 * L * 2.0 ** -19))
