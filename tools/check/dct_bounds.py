"""Rigorous forward-error bounds for the DCT paths of the forward kernel (DESIGN.md
§5 "Why the fast path is exact").  Not product code: it prints the bounds and
emits tools/check/dct_windows.h, the float32 windows the round-5 packed kernel
compiled in (removed from the product; commit ae5c500).

Every intermediate is a linear functional L of the 64 pixels of a block (float64
coefficients; we only need magnitudes).  For each node we carry a bound E on
|computed - exact|.  A rounding to a format with unit roundoff u adds at most
u * (max|exact| + E).  max|exact| over the input box: raw bytes p in [0, 255] ->
255 * max(sum L+, sum |L-|); centred pixels x in [-128, 127] -> 128 * |L|_1.
An integer combination below 2^24 (f32) / 2^53 (f64) is exact.  A constant c
stored as K contributes |a| * |K - c|; |K - c| <= 1 ulp(c) is assumed for the
pocketfft twiddles (they are not all correctly rounded), 1/2 ulp for ours.

Four estimates of y/T are bounded (y = scipy.fftpack 2-D DCT-II of the centred
block, T the quantisation table entry):
  E64[t][u][v] the float64 AAN fast path (dct_core.h dct_block_aan: the production
               path of k_dct_planes and k_encode420)
  E1[t][u][v]  the float32 AAN fast path (dct_core.h dct_block_f32)
  E2[u][v]     the float64 separable dot product of the fallback (dct_coef_f64)
  EP[u][v]     pocketfft's own float64 result (the reference), vs the exact y
The fast path's window is W1 = E1 + EP + (rounding of the tie test), the
fallback's W2 = E2 + EP + (its test): outside its window a path's rint is the
reference's rint(fl(y_pf / T)).
"""
import math
import sys

import numpy as np

QT = [[16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56, 14, 17,
       22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92, 49, 64, 78,
       87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99],
      [17, 18, 24, 47] + [99] * 4 + [18, 21, 26, 66] + [99] * 4 + [24, 26, 56] + [99] * 5 + [47, 66] + [99] * 6
      + [99] * 32]


class Ctx:
    def __init__(self, u, exact_lim, raw, ulp_const):
        self.u, self.lim, self.raw, self.kc = u, exact_lim, raw, ulp_const

    def mag(self, L):
        if self.raw:
            return 255.0 * max(L[L > 0].sum(), -L[L < 0].sum())
        return 128.0 * np.abs(L).sum()


class N:
    __slots__ = ("L", "E", "i", "c")

    def __init__(self, c, L, E, i):
        self.c, self.L, self.E, self.i = c, L, E, i

    def mag(self):
        return self.c.mag(self.L)

    def _r(self, L, E, exact_int):
        n = N(self.c, L, E, exact_int)
        if exact_int and n.mag() < self.c.lim:
            n.E = 0.0
            return n
        n.i = False
        n.E = E + self.c.u * (n.mag() + E)
        return n

    def __add__(self, o):
        return self._r(self.L + o.L, self.E + o.E, self.i and o.i)

    def __sub__(self, o):
        return self._r(self.L - o.L, self.E + o.E, self.i and o.i)

    def __neg__(self):
        return N(self.c, -self.L, self.E, self.i)

    def scale(self, p):  # exact power-of-two scaling
        return N(self.c, self.L * p, self.E * abs(p), self.i)

    def mul(self, c, K=None):
        """round(self * K), K the stored constant for the real c"""
        dK = self.c.kc * abs(c)
        return self._r(self.L * c, (abs(c) + dK) * self.E + self.mag() * dK, False)

    def fma(self, c, b, s=1.0):
        """round(s * c * self + b)"""
        dK = self.c.kc * abs(c)
        return self._r(s * c * self.L + b.L, (abs(c) + dK) * self.E + self.mag() * dK + b.E, False)


def pixels(c):
    return [[N(c, np.eye(64)[8 * m + n], 0.0, True) for n in range(8)] for m in range(8)]


# ---- float32 AAN (dct_core.h dct_block_f32): raw bytes, fused z11/z13 and o2/o6
A1, A5 = math.cos(math.pi / 4), math.cos(3 * math.pi / 8)
A2, A4 = math.cos(math.pi / 8) - A5, math.cos(math.pi / 8) + A5


def aan(x):
    s0, s1, s2, s3 = x[0] + x[7], x[1] + x[6], x[2] + x[5], x[3] + x[4]
    t10, t13, t11, t12 = s0 + s3, s0 - s3, s1 + s2, s1 - s2
    o = [None] * 8
    o[0], o[4] = t10 + t11, t10 - t11
    w = t12 + t13
    o[2], o[6] = w.fma(A1, t13), w.fma(A1, t13, -1.0)
    d7, d6, d5, d4 = x[0] - x[7], x[1] - x[6], x[2] - x[5], x[3] - x[4]
    u10, u11, u12 = d4 + d5, d5 + d6, d6 + d7
    z5 = (u10 - u12).mul(A5)
    z2, z4 = u10.fma(A2, z5), u12.fma(A4, z5)
    z11, z13 = u11.fma(A1, d7), u11.fma(A1, d7, -1.0)
    o[5], o[3], o[1], o[7] = z13 + z2, z13 - z2, z11 + z4, z11 - z4
    return o


def aan_scale(k):
    return 2.0 if k == 0 else 1.0 / math.cos(k * math.pi / 16)  # AAN output k = y_k / S_k


def E1():
    c = Ctx(2.0 ** -24, 2.0 ** 24, True, 2.0 ** -24)
    px = pixels(c)
    rows = [aan(px[m]) for m in range(8)]
    out = np.zeros((2, 8, 8))
    for v in range(8):
        col = aan([rows[m][v] for m in range(8)])
        for u in range(8):
            n = col[u]
            for t in range(2):
                R = aan_scale(u) * aan_scale(v) / QT[t][8 * u + v]
                dR = 2.0 ** -24 * R
                # e = Y * Rf exactly inside the fma (no rounding of the product)
                out[t, u, v] = ((R + dR) * n.E + n.mag() * dR) / 1.0
    return out


# ---- pocketfft DCT-II (dct_core.h dct8h_int / dct8h), centred pixels
TW = [math.cos(math.pi * (i + 1) / 16) for i in range(7)]
WRc = math.cos(math.pi / 4)


def pf_dct8(x):
    c1, c2 = x[1] + x[2], x[2] - x[1]
    c3, c4 = x[3] + x[4], x[4] - x[3]
    c5, c6 = x[5] + x[6], x[6] - x[5]
    H0, H4 = x[0] + x[7], x[0] - x[7]
    h1, tr2, ti2, h2 = c1 + c5, c1 - c5, c2 + c6, c2 - c6
    h6 = ti2.mul(WRc) + tr2.mul(WRc)
    h5 = tr2.mul(WRc) - ti2.mul(WRc)
    T2, T1 = H0 + c3, H0 - c3
    D0, D4, D6, D2 = T2 + h1, T2 - h1, T1 + h2, T1 - h2
    U2, U1 = H4 - c4, H4 + c4
    D1, D5, D7, D3 = U2 + h5, U2 - h5, U1 + h6, U1 - h6
    y = [None] * 8

    def rot(a, b, ca, cb):  # P1 = ca*a + cb*b, P2 = ca*b - cb*a ; y = P1 + P2, P1 - P2
        P1 = a.mul(ca) + b.mul(cb)
        P2 = b.mul(ca) - a.mul(cb)
        return P1 + P2, P1 - P2
    y[1], y[7] = rot(D7, D1, TW[0], TW[6])
    y[2], y[6] = rot(D6, D2, TW[1], TW[5])
    y[3], y[5] = rot(D5, D3, TW[2], TW[4])
    y[0] = D0
    y[4] = D4.mul(TW[3])
    return y  # half-scaled: y[0], y[4] are y/2


def EP():
    c = Ctx(2.0 ** -53, 2.0 ** 53, False, 2.0 ** -52)
    px = pixels(c)
    rows = [pf_dct8(px[m]) for m in range(8)]
    out = np.zeros((8, 8))
    for v in range(8):
        col = pf_dct8([rows[m][v] for m in range(8)])
        for u in range(8):
            rho = (0.5 if u in (0, 4) else 1.0) * (0.5 if v in (0, 4) else 1.0)
            out[u, v] = col[u].E / rho  # error of the full-scale y
    return out


# ---- float64 fallback (dct_core.h dct_coef_f64), folded by symmetry:
# r_m = sum_{n<4} C_v(n) a_mn (a multiply, then an fma chain), a_mn = x_mn +- x_m,7-n
# (an exact integer); y = sum_{m<4} C_u(m) b_m, b_m = r_m +- r_7-m (rounded add)
def E2():
    c = Ctx(2.0 ** -53, 2.0 ** 53, False, 2.0 ** -53)
    px = pixels(c)
    out = np.zeros((8, 8))
    C = lambda k, n: 2.0 * math.cos(math.pi * k * (2 * n + 1) / 16)  # noqa: E731
    for u in range(8):
        for v in range(8):
            r = []
            for m in range(8):
                a = [px[m][n] + px[m][7 - n] if v % 2 == 0 else px[m][n] - px[m][7 - n] for n in range(4)]
                acc = a[0].mul(C(v, 0))
                for n in range(1, 4):
                    acc = a[n].fma(C(v, n), acc)
                r.append(acc)
            b = [r[m] + r[7 - m] if u % 2 == 0 else r[m] - r[7 - m] for m in range(4)]
            acc = b[0].mul(C(u, 0))
            for m in range(1, 4):
                acc = b[m].fma(C(u, m), acc)
            out[u, v] = acc.E
    return out


# ---- float64 AAN (dct_core.h aan_even / aan_odd / dct_block_aan, the production
# fast path): integer prefix on raw bytes (exact), then float64 with separate
# multiply and add where the source has them (z1, z3) and explicit fmas (z2, z4)
A1d, A2d, A4d, A5d = A1, A2, A4, A5


def aan64_even(x):
    s0, s1, s2, s3 = x[0] + x[7], x[1] + x[6], x[2] + x[5], x[3] + x[4]
    t10, t13, t11, t12 = s0 + s3, s0 - s3, s1 + s2, s1 - s2
    z1 = (t12 + t13).mul(A1d)
    return t10 + t11, t13 + z1, t10 - t11, t13 - z1  # outputs 0, 2, 4, 6


def aan64_odd(x):
    d7, d6, d5, d4 = x[0] - x[7], x[1] - x[6], x[2] - x[5], x[3] - x[4]
    u10, u11, u12 = d4 + d5, d5 + d6, d6 + d7
    z5 = (u10 - u12).mul(A5d)
    z2, z4 = u10.fma(A2d, z5), u12.fma(A4d, z5)
    z3 = u11.mul(A1d)
    z11, z13 = d7 + z3, d7 - z3
    return z11 + z4, z13 - z2, z13 + z2, z11 - z4  # outputs 1, 3, 5, 7


def aan64(x):
    e, o = aan64_even(x), aan64_odd(x)
    return [e[0], o[0], e[1], o[1], e[2], o[2], e[3], o[3]]


def E64():
    """|b * kRA - y / T| of dct_block_aan for every (t, u, v) but (0,0) and (4,4)
    (computed exactly there), b the AAN output, kRA = fl64(S_u S_v / T)."""
    c = Ctx(2.0 ** -53, 2.0 ** 53, True, 2.0 ** -53)
    px = pixels(c)
    rows = [aan64(px[m]) for m in range(8)]
    out = np.zeros((2, 8, 8))
    for v in range(8):
        col = aan64([rows[m][v] for m in range(8)])
        for u in range(8):
            n = col[u]
            for t in range(2):
                R = aan_scale(u) * aan_scale(v) / QT[t][8 * u + v]
                dR = 2.0 ** -53 * R  # kRA correctly rounded
                out[t, u, v] = (R + dR) * n.E + n.mag() * dR
    return out


def windows():
    e1, e2, ep = E1(), E2(), EP()
    W1 = np.zeros((2, 8, 8))
    W2 = np.zeros((2, 8, 8))
    for t in range(2):
        T = np.array(QT[t], float).reshape(8, 8)
        # fast-path test: d = fma(Y, Rf, -rint) is exact to 2^-25 (|d| <= 1/2 + E1);
        # fl(y_pf / T) is within 2^-53 |y/T| <= 2^-41 of y_pf / T
        W1[t] = e1[t] + ep / T + 2.0 ** -24 + 2.0 ** -40
        # fallback test: b = y2 * (1/T) rounded (fma with the 2^32 magic below) to 2^-32;
        # 1/T stored to 2^-53 relative -> |y/T| 2^-52
        W2[t] = e2 / T + ep / T + 2.0 ** -31 + 2.0 ** -40
    return e1, e2, ep, W1, W2


def emit(path):
    e1, e2, ep, W1, W2 = windows()
    S = [aan_scale(k) for k in range(8)]
    lines = ["// GENERATED by tools/check/dct_bounds.py --emit (do not edit): the float32 fast",
             "// path's quantiser constants and tie windows, from the rigorous forward-error",
             "// bounds derived there (DESIGN.md §5).",
             "#pragma once", "", "namespace hic {", "namespace {", ""]
    lines.append("// R[t][u*8+v] = float32(S_u S_v / T[t][u][v]) (AAN output scale S_0 = 2, S_k = 1/cos(k pi/16))")
    lines.append("constexpr float kR32[2][64] = {")
    for t in range(2):
        vals = [float(np.float32(S[i // 8] * S[i % 8] / QT[t][i])) for i in range(64)]
        lines.append("    {" + ", ".join(v.hex() + "f" for v in vals) + "},")
    lines.append("};")
    lines.append("// fast-path flag threshold: |d| > kThr32 flags (d = Y*R - rint(Y*R));")
    lines.append("// kThr32 = float32 rounded down of 1/2 - W1, W1 = E1 + EP/T + 2^-24 + 2^-40")
    lines.append("constexpr float kThr32[2][64] = {")
    thr = [[], []]
    for t in range(2):
        vals = []
        for i in range(64):
            th = np.float32(0.5 - W1[t].flat[i])
            if float(th) > 0.5 - W1[t].flat[i]:
                th = np.nextafter(th, np.float32(0))
            vals.append(float(th))
        thr[t] = vals
        lines.append("    {" + ", ".join(v.hex() + "f" for v in vals) + "},")
    lines.append("};")
    # the packed path tests d^2 > c instead of |d| > thr: c must not exceed thr^2, so
    # every |d| > thr is still flagged (fl(c - d*d) in one fma has d*d's exact sign)
    lines.append("// packed-path threshold: d*d > kThr32Sq flags; kThr32Sq = float32 rounded down of kThr32^2")
    lines.append("constexpr float kThr32Sq[2][64] = {")
    for t in range(2):
        vals = []
        for th in thr[t]:
            sq = np.float32(th * th)
            if float(sq) > th * th:  # float64 th*th is exact (24-bit th)
                sq = np.nextafter(sq, np.float32(0))
            vals.append(float(sq))
        lines.append("    {" + ", ".join(v.hex() + "f" for v in vals) + "},")
    lines.append("};")
    m2 = float(W2.max())
    k = math.ceil(-math.log2(m2)) - 1
    lines.append("// fallback (float64) window: the largest W2 over both tables is 2^%.2f; the" % math.log2(m2))
    lines.append("// test uses 2^-%d (kW2Log2)" % k)
    lines.append("constexpr int kW2Log2 = %d;" % k)
    lines += ["", "}  // namespace", "}  // namespace hic", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--emit":
        emit(sys.argv[2])
        sys.exit(0)
    e1, e2, ep, W1, W2 = windows()
    np.set_printoptions(linewidth=160, precision=1)
    for t in range(2):
        print("table", t, "log2 W1:\n", np.log2(W1[t]))
        print("  expected fast-path flags per block (2 W1 summed over AC):", round(2 * (W1[t].sum() - W1[t, 0, 0]), 4))
    print("log2 E2 (y):\n", np.log2(e2))
    print("log2 EP (y):\n", np.log2(ep))
    print("max W2 = 2^%.2f" % math.log2(W2.max()))
    # the float64 fast path: qfast rounds b * kRA + 1/2 + 2^-30 to a multiple of 2^-32
    # (2^-33 error) and flags a low word <= 6, so an unflagged value lies more than
    # 2.5 * 2^-32 (above) / 4 * 2^-32 (below) from the next integer; its rint equals
    # rint(fl(y_pf / T)) if the estimate's error + pocketfft's + the division's stays
    # below that margin
    e64 = E64()
    for t in range(2):
        T = np.array(QT[t], float).reshape(8, 8)
        tot = e64[t] + ep / T + 2.0 ** -33 + 2.0 ** -41
        tot[0, 0] = tot[4, 4] = 0.0  # exact paths
        print("table", t, "float64 AAN: max |estimate - y_pf/T| + roundings = 2^%.2f  (margin 2.5 * 2^-32 = 2^%.2f)"
              % (math.log2(tot.max()), math.log2(2.5 * 2.0 ** -32)))
        assert tot.max() < 2.5 * 2.0 ** -32
