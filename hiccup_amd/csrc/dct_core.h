// dct_core.h -- the bit-exact 8x8 DCT-II / DCT-III + quantizer building blocks
// shared by the transform kernels (dct.hip) and the fused plane encoder
// (encode.hip).  See dct.hip for the design notes and reference citations.
#pragma once
#include "hic_common.h"

namespace hic {
namespace {

// pocketfft sincos_2pibyn constants (n = 8 radix-2 twiddle, n = 16 DCT twiddles)
constexpr double WR = 0x1.6a09e667f3bccp-1;
constexpr double WI = 0x1.6a09e667f3bcdp-1;
constexpr double TW0 = 0x1.f6297cff75cb0p-1;
constexpr double TW1 = 0x1.d906bcf328d46p-1;
constexpr double TW2 = 0x1.a9b66290ea1a3p-1;
constexpr double TW3 = 0x1.6a09e667f3bccp-1;
constexpr double TW4 = 0x1.1c73b39ae68c8p-1;
constexpr double TW5 = 0x1.87de2a6aea963p-2;
constexpr double TW6 = 0x1.8f8b83c69a60ap-3;
constexpr double TW3x2 = 2.0 * TW3;  // exact

// quantization.py:14-37 (JPEG Annex K), raster [u][v]
constexpr int QT[2][64] = {
    {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
     14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
     18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
     49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99},
    {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
     24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99}};

// transposed zig-zag: zig-zag position -> raster index (transform.py:106-124)
constexpr int ZZ[64] = {0,  8,  1,  2,  9,  16, 24, 17, 10, 3,  4,  11, 18, 25, 32, 40,
                        33, 26, 19, 12, 5,  6,  13, 20, 27, 34, 41, 48, 56, 49, 42, 35,
                        28, 21, 14, 7,  15, 22, 29, 36, 43, 50, 57, 58, 51, 44, 37, 30,
                        23, 31, 38, 45, 52, 59, 60, 53, 46, 39, 47, 54, 61, 62, 55, 63};

// rho(k): the half-scaled transform returns outputs 0 and 4 at half scale.
constexpr double rho(int k) { return (k == 0 || k == 4) ? 0.5 : 1.0; }

constexpr bool pow2(double d) {
  if (d <= 0) return false;
  while (d > 1.0) d *= 0.5;
  while (d < 1.0) d *= 2.0;
  return d == 1.0;
}

// D[u][v] = rho(u) rho(v) T[u][v]: b'/D == b/T as real numbers (exact scaling).
struct QConst {
  double d[2][64];
  double r[2][64];
  constexpr QConst() : d(), r() {
    for (int t = 0; t < 2; ++t)
      for (int i = 0; i < 64; ++i) {
        d[t][i] = rho(i / 8) * rho(i % 8) * (double)QT[t][i];
        r[t][i] = 1.0 / d[t][i];
      }
  }
};
constexpr QConst kQ{};

// ---------------------------------------------------------------------------
// Half-scaled pocketfft DCT-II, n = 8.  Returns y' with y'[0] = y[0]/2,
// y'[4] = y[4]/2 and y'[k] = y[k] otherwise, where y = scipy.fftpack.dct(x).
// Integer-input variant: x are exact small integers.
__device__ __forceinline__ void dct8h_int(const int (&x)[8], int &y0, double (&y)[8]) {
  const int c1 = x[1] + x[2], c2 = x[2] - x[1];
  const int c3 = x[3] + x[4], c4 = x[4] - x[3];
  const int c5 = x[5] + x[6], c6 = x[6] - x[5];
  const int H0 = x[0] + x[7], H4 = x[0] - x[7];
  const int h1 = c1 + c5, tr2 = c1 - c5, ti2 = c2 + c6, h2 = c2 - c6;
  const double dtr2 = (double)tr2, dti2 = (double)ti2;
  const double h6 = WR * dti2 + WI * dtr2;
  const double h5 = WR * dtr2 - WI * dti2;
  const int T2 = H0 + c3, T1 = H0 - c3;
  const int D0 = T2 + h1, D4 = T2 - h1, D6 = T1 + h2, D2 = T1 - h2;
  const double U2 = (double)(H4 - c4), U1 = (double)(H4 + c4);
  const double D1 = U2 + h5, D5 = U2 - h5, D7 = U1 + h6, D3 = U1 - h6;
  double P1 = TW0 * D7 + TW6 * D1, P2 = TW0 * D1 - TW6 * D7;
  y[1] = P1 + P2;
  y[7] = P1 - P2;
  const double dD6 = (double)D6, dD2 = (double)D2;
  P1 = TW1 * dD6 + TW5 * dD2;
  P2 = TW1 * dD2 - TW5 * dD6;
  y[2] = P1 + P2;
  y[6] = P1 - P2;
  P1 = TW2 * D5 + TW4 * D3;
  P2 = TW2 * D3 - TW4 * D5;
  y[3] = P1 + P2;
  y[5] = P1 - P2;
  y0 = D0;
  y[0] = (double)D0;
  y[4] = (double)D4 * TW3;
}

// Float64-input variant (column pass).
__device__ __forceinline__ void dct8h(const double (&x)[8], double (&y)[8]) {
  const double c1 = x[1] + x[2], c2 = x[2] - x[1];
  const double c3 = x[3] + x[4], c4 = x[4] - x[3];
  const double c5 = x[5] + x[6], c6 = x[6] - x[5];
  const double H0 = x[0] + x[7], H4 = x[0] - x[7];
  const double h1 = c1 + c5, tr2 = c1 - c5, ti2 = c2 + c6, h2 = c2 - c6;
  const double h6 = WR * ti2 + WI * tr2;
  const double h5 = WR * tr2 - WI * ti2;
  const double T2 = H0 + c3, T1 = H0 - c3;
  const double D0 = T2 + h1, D4 = T2 - h1, D6 = T1 + h2, D2 = T1 - h2;
  const double U2 = H4 - c4, U1 = H4 + c4;
  const double D1 = U2 + h5, D5 = U2 - h5, D7 = U1 + h6, D3 = U1 - h6;
  double P1 = TW0 * D7 + TW6 * D1, P2 = TW0 * D1 - TW6 * D7;
  y[1] = P1 + P2;
  y[7] = P1 - P2;
  P1 = TW1 * D6 + TW5 * D2;
  P2 = TW1 * D2 - TW5 * D6;
  y[2] = P1 + P2;
  y[6] = P1 - P2;
  P1 = TW2 * D5 + TW4 * D3;
  P2 = TW2 * D3 - TW4 * D5;
  y[3] = P1 + P2;
  y[5] = P1 - P2;
  y[0] = D0;
  y[4] = D4 * TW3;
}

// pocketfft DCT-III, n = 8 (scipy.fftpack.idct, type 2, norm=None).
template <typename In>
__device__ __forceinline__ void idct8(const In (&c)[8], double (&y)[8]) {
  double C1, C7, C2, C6, C3, C5;
  {
    const In t1 = c[1] + c[7], t2 = c[1] - c[7];
    C1 = TW0 * (double)t2 + TW6 * (double)t1;
    C7 = TW0 * (double)t1 - TW6 * (double)t2;
  }
  {
    const In t1 = c[2] + c[6], t2 = c[2] - c[6];
    C2 = TW1 * (double)t2 + TW5 * (double)t1;
    C6 = TW1 * (double)t1 - TW5 * (double)t2;
  }
  {
    const In t1 = c[3] + c[5], t2 = c[3] - c[5];
    C3 = TW2 * (double)t2 + TW4 * (double)t1;
    C5 = TW2 * (double)t1 - TW4 * (double)t2;
  }
  const double C4 = (double)c[4] * TW3x2;
  const double C0 = (double)c[0];
  // radix-4 then radix-2 (ido = 4)
  double tr1 = C6 + C2;
  const double h2 = C6 - C2;
  double tr2 = C0 + C4;
  const double h1 = C0 - C4;
  const double h0 = tr2 + tr1, h3 = tr2 - tr1;
  tr1 = C7 + C3;
  const double h6 = C7 - C3;
  tr2 = C1 + C5;
  const double h5 = C1 - C5;
  const double h4 = tr2 + tr1, h7 = tr2 - tr1;
  const double d0 = h0 + h4, d7 = h0 - h4;
  const double r2 = WR * h5 + WI * h6;
  const double i2 = WR * h6 - WI * h5;
  const double d1 = h1 + r2, d5 = h1 - r2, d2 = i2 + h2, d6 = i2 - h2;
  y[0] = d0;
  y[1] = d1 - d2;
  y[2] = d2 + d1;
  y[3] = h3 + h7;  // d3 - d4 with d4 = -h7
  y[4] = h3 - h7;  // d4 + d3
  y[5] = d5 - d6;
  y[6] = d6 + d5;
  y[7] = d7;
}

// rint(b / D[t][i]) as numpy computes it (fp64 divide, round half to even).
template <int TABLE>
__device__ __forceinline__ int quantize(double b, int i) {
  const double p = b * kQ.r[TABLE][i];
  double r = __builtin_rint(p);
  if (i != 0) {  // DC: b' is an exact integer and D is 4 or 17/4 -> never near a tie
    if (__builtin_fabs(p - r) > 0.5 - 0x1p-30) r = __builtin_rint(b / kQ.d[TABLE][i]);
  }
  return (int)r;
}

__device__ __forceinline__ void put16(uint32_t (&pk)[32], int slot, int q) {
  const uint32_t v = (uint32_t)q & 0xFFFFu;
  if (slot & 1)
    pk[slot >> 1] |= v << 16;
  else
    pk[slot >> 1] |= v;
}

// position of raster index i in the output packing of `LAYOUT`
template <int LAYOUT>
struct SlotOf {
  int s[64];
  constexpr SlotOf() : s() {
    for (int z = 0; z < 64; ++z) {
      if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16)
        s[ZZ[z]] = z;
      else
        s[z] = z;
    }
  }
};

template <int TABLE>
__device__ __forceinline__ int quant_fast(double b, int i) {
  if (pow2(kQ.d[TABLE][i])) return (int)__builtin_rint(b * kQ.r[TABLE][i]);  // exact product
  // one rounding of the exact product b*(1/D) to a multiple of 2^-19 (FMA: the
  // tie test below is then about b*(1/D) itself, within 2^-53 relative of b/D)
  const double t = __builtin_fma(b, kQ.r[TABLE][i], 0x1.8p33);
  const int n = (int)(uint32_t)(unsigned long long)__double_as_longlong(t);
  const int sft = n + (1 << 18);
  int q = sft >> 19;
  if ((sft & 0x7FFFF) == 0) q = (int)__builtin_rint(b / kQ.d[TABLE][i]);
  return q;
}

constexpr int kStagePad = 9;  // uint4 per block in the LDS stage (8 + 1 pad: conflict-free)

// One 8x8 block (this lane's eight 8-byte pixel rows) -> quantized int16
// coefficients written to st[slot] in the order of LAYOUT (stage row of this lane).
// Two phases: the row transform's even outputs (0, 2, 4, 6: the k=0 butterfly +
// the (2,6) twiddle pair) feed the four even-column transforms, then the odd
// outputs (1, 3, 5, 7) the odd columns.  Live state is ~half of a one-pass
// block, at the cost of recomputing 4 integer sums per row.
template <int TABLE, int LAYOUT>
__device__ __forceinline__ void dct_block_2ph(uint2 (&w)[8], int16_t *st) {
  constexpr SlotOf<LAYOUT> kSlot{};
  auto px = [&](int r, int n) -> int {
    return (int)(((n < 4 ? w[r].x : w[r].y) >> (8 * (n & 3))) & 0xFFu) - 128;
  };
  // ---- phase A: even row outputs -> even columns
  {
    int e0[8];
    double e2[8], e4[8], e6[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int c1 = px(r, 1) + px(r, 2), c2 = px(r, 2) - px(r, 1);
      const int c3 = px(r, 3) + px(r, 4);
      const int c5 = px(r, 5) + px(r, 6), c6 = px(r, 6) - px(r, 5);
      const int H0 = px(r, 0) + px(r, 7);
      const int h1 = c1 + c5, h2 = c2 - c6;
      const int T2 = H0 + c3, T1 = H0 - c3;
      const double D6 = (double)(T1 + h2), D2 = (double)(T1 - h2);
      e0[r] = T2 + h1;
      e4[r] = (double)(T2 - h1) * TW3;
      const double P1 = TW1 * D6 + TW5 * D2, P2 = TW1 * D2 - TW5 * D6;
      e2[r] = P1 + P2;
      e6[r] = P1 - P2;
    }
    {
      int b0;
      double b[8];
      dct8h_int(e0, b0, b);
      st[kSlot.s[0]] = (int16_t)quant_fast<TABLE>((double)b0, 0);
#pragma unroll
      for (int u = 1; u < 8; ++u) st[kSlot.s[u * 8]] = (int16_t)quant_fast<TABLE>(b[u], u * 8);
    }
    double b[8];
    dct8h(e2, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 2]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 2);
    dct8h(e4, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 4]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 4);
    dct8h(e6, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 6]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 6);
  }
  // ---- phase B: odd row outputs -> odd columns.  Re-unpack the pixels (the asm
  // makes w opaque, so the compiler cannot keep 64 unpacked ints live across phases)
#pragma unroll
  for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(w[r].x), "+v"(w[r].y));
  {
    double o1[8], o3[8], o5[8], o7[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int c1 = px(r, 1) + px(r, 2), c2 = px(r, 2) - px(r, 1);
      const int c4 = px(r, 4) - px(r, 3);
      const int c5 = px(r, 5) + px(r, 6), c6 = px(r, 6) - px(r, 5);
      const int H4 = px(r, 0) - px(r, 7);
      const double tr2 = (double)(c1 - c5), ti2 = (double)(c2 + c6);
      const double h6 = WR * ti2 + WI * tr2;
      const double h5 = WR * tr2 - WI * ti2;
      const double U2 = (double)(H4 - c4), U1 = (double)(H4 + c4);
      const double D1 = U2 + h5, D5 = U2 - h5, D7 = U1 + h6, D3 = U1 - h6;
      double P1 = TW0 * D7 + TW6 * D1, P2 = TW0 * D1 - TW6 * D7;
      o1[r] = P1 + P2;
      o7[r] = P1 - P2;
      P1 = TW2 * D5 + TW4 * D3;
      P2 = TW2 * D3 - TW4 * D5;
      o3[r] = P1 + P2;
      o5[r] = P1 - P2;
    }
    double b[8];
    dct8h(o1, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 1]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 1);
    dct8h(o3, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 3]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 3);
    dct8h(o5, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 5]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 5);
    dct8h(o7, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 7]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 7);
  }
}

}  // namespace
}  // namespace hic
