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
__host__ __device__ __forceinline__ void dct8h_int(const int (&x)[8], int &y0, double (&y)[8]) {
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
__host__ __device__ __forceinline__ void dct8h(const double (&x)[8], double (&y)[8]) {
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
__host__ __device__ __forceinline__ void idct8(const In (&c)[8], double (&y)[8]) {
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
__host__ __device__ __forceinline__ int quantize(double b, int i) {
  const double p = b * kQ.r[TABLE][i];
  double r = __builtin_rint(p);
  if (i != 0) {  // DC: b' is an exact integer and D is 4 or 17/4 -> never near a tie
    if (__builtin_fabs(p - r) > 0.5 - 0x1p-30) r = __builtin_rint(b / kQ.d[TABLE][i]);
  }
  return (int)r;
}

__host__ __device__ __forceinline__ void put16(uint32_t (&pk)[32], int slot, int q) {
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

// TABLE >= 0: the table is a compile-time constant; TABLE == -1: it is `trt`
// (wave-uniform at run time, so the constants become scalar loads).  The same
// convention holds for every TABLE-templated block function below.
template <int TABLE>
__host__ __device__ __forceinline__ int quant_fast(double b, int i, int trt = 0) {
  constexpr int kT = TABLE >= 0 ? TABLE : 0;
  const int t = TABLE >= 0 ? TABLE : trt;
  if (TABLE >= 0 && pow2(kQ.d[kT][i])) return (int)__builtin_rint(b * kQ.r[kT][i]);  // exact product
  // one rounding of the exact product b*(1/D) to a multiple of 2^-19 (FMA: the
  // tie test below is then about b*(1/D) itself, within 2^-53 relative of b/D;
  // a power-of-two D makes the product exact and the test exact too)
  const double tt = __builtin_fma(b, kQ.r[t][i], 0x1.8p33);
  const int n = (int)(uint32_t)__builtin_bit_cast(unsigned long long, tt);
  const int sft = n + (1 << 18);
  int q = sft >> 19;
  if ((sft & 0x7FFFF) == 0) q = (int)__builtin_rint(b / kQ.d[t][i]);
  return q;
}

// LDS stage row of one block: 128 B of coefficients + 8 B pad (17 x 8 B).  The
// quantiser writes it 2 B at a time (ds_write_b16, banks (a/4) mod 32): a 34-dword
// lane stride puts a half-wave's 32 lanes on 16 banks, a 2-way conflict, which
// costs a b16 store nothing (a 36-dword stride was 4-way, 2x); it is read back
// 8 B at a time (ds_read_b64)
constexpr int kStageU2 = 17;

// One 8x8 block (this lane's eight 8-byte pixel rows) -> quantized int16
// coefficients written to st[slot] in the order of LAYOUT (stage row of this lane).
// Two phases: the row transform's even outputs (0, 2, 4, 6: the k=0 butterfly +
// the (2,6) twiddle pair) feed the four even-column transforms, then the odd
// outputs (1, 3, 5, 7) the odd columns.  Live state is ~half of a one-pass
// block, at the cost of recomputing 4 integer sums per row.
template <int TABLE, int LAYOUT>
__host__ __device__ __forceinline__ void dct_block_2ph(uint2 (&w)[8], int16_t *st, int trt = 0) {
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
      st[kSlot.s[0]] = (int16_t)quant_fast<TABLE>((double)b0, 0, trt);
#pragma unroll
      for (int u = 1; u < 8; ++u) st[kSlot.s[u * 8]] = (int16_t)quant_fast<TABLE>(b[u], u * 8, trt);
    }
    double b[8];
    dct8h(e2, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 2]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 2, trt);
    dct8h(e4, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 4]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 4, trt);
    dct8h(e6, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 6]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 6, trt);
  }
  // ---- phase B: odd row outputs -> odd columns.  Re-unpack the pixels (the asm
  // makes w opaque, so the compiler cannot keep 64 unpacked ints live across phases)
#pragma unroll
  for (int r = 0; r < 8; ++r) {
#ifdef __HIP_DEVICE_COMPILE__
    asm volatile("" : "+v"(w[r].x), "+v"(w[r].y));  // register-pressure barrier (device code only)
#endif
  }
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
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 1]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 1, trt);
    dct8h(o3, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 3]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 3, trt);
    dct8h(o5, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 5]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 5, trt);
    dct8h(o7, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + 7]] = (int16_t)quant_fast<TABLE>(b[u], u * 8 + 7, trt);
  }
}

// ---------------------------------------------------------------------------
// Fast path: Arai-Agui-Nakajima (AAN) factorised 8-point DCT-II, 5 multiplies
// (2 fused) and 29 adds per 1-D transform, ~45% of the float64 operations of
// the pocketfft replica.  Its outputs are y_k / S_k with S_0 = 2 and
// S_k = 1 / cos(k*pi/16); the 2-D scale S_u S_v is folded into the quantiser
// constant kRA = S_u S_v / T.  The fast result differs from pocketfft's float64
// value only by rounding, so rint(y / T) agrees wherever y / T is not within the
// quantiser's tie window (2^-31 of a half-integer, see qfast).  A block with a
// coefficient inside the window is reported to the caller: the (2,2) class apart
// (dct_fix26), anything else for a redo on the exact pocketfft path
// (dct_block_2ph).  (0,0) (an integer) and (4,4) (an integer times cos(pi/4)^2)
// are computed here with pocketfft's own operation sequence.
constexpr double kA1 = 0x1.6a09e667f3bcdp-1;  // cos(pi/4)
constexpr double kA2 = 0x1.1517a7bdb3895p-1;  // cos(pi/8) - cos(3pi/8)
constexpr double kA4 = 0x1.4e7ae9144f0fcp+0;  // cos(pi/8) + cos(3pi/8)
constexpr double kA5 = 0x1.87de2a6aea963p-2;  // cos(3pi/8)
// S_u S_v / T[u][v] (raster [u][v]), correctly rounded
constexpr double kRA[2][64] = {
    {0x1.0000000000000p-2, 0x1.7ba89eae3f7bep-3, 0x1.bb590c62b8dbbp-3, 0x1.33e37a1e0173ep-3,
     0x1.e2b7dddfefa66p-4, 0x1.70a158c8e0aadp-4, 0x1.a3bd60ba1cf0ap-4, 0x1.582fdb4eee6fbp-3,
     0x1.5c053c1fba319p-3, 0x1.62d6acad3f2e3p-4, 0x1.42e18fe92cb18p-4, 0x1.085aa551e1e43p-4,
     0x1.c650cb793af71p-5, 0x1.0335588fc721ep-5, 0x1.6bc4bca389533p-5, 0x1.853696338f32ep-4,
     0x1.3cad51fd5f785p-3, 0x1.5bb7d60ecdab8p-4, 0x1.2bec333018867p-4, 0x1.bc5773154fbb4p-5,
     0x1.397e885588782p-5, 0x1.180073dce05b3p-5, 0x1.4fcdd1fff4a04p-5, 0x1.95cee8190983dp-4,
     0x1.5fdf66fdb8847p-3, 0x1.27745e6a930e1p-4, 0x1.e4bc7d8b9ccc4p-5, 0x1.9899cc29aafa9p-5,
     0x1.1134702de0ef1p-5, 0x1.97ad1a1a0b168p-6, 0x1.41d21671728f1p-5, 0x1.974603fed046ep-4,
     0x1.41cfe93ff5199p-3, 0x1.0c758f81d1637p-4, 0x1.52e9a8251de9bp-5, 0x1.f19f832efe45bp-6,
     0x1.e1e1e1e1e1e1ep-6, 0x1.7e9f206fde8a9p-6, 0x1.25eb551855053p-5, 0x1.819c35037af83p-4,
     0x1.33311f52108e6p-3, 0x1.ad8b9a12d4f65p-5, 0x1.222f03b65ce0dp-5, 0x1.1517a7bdb3895p-5,
     0x1.01716341c9e20p-5, 0x1.fe65cc24132b7p-6, 0x1.54fbad46dbf8cp-5, 0x1.9ac4cea9f4378p-4,
     0x1.b4df3ae10e72ap-4, 0x1.550870d950be0p-5, 0x1.290eafec44b53p-5, 0x1.27ed526e34604p-5,
     0x1.25eb551855053p-5, 0x1.3e70538a1bb58p-5, 0x1.d22769d10a86dp-5, 0x1.0f9a260bd6d97p-3,
     0x1.239a52b1183b1p-3, 0x1.d15d17c33658bp-5, 0x1.de6d31f7ca8b4p-5, 0x1.01a9aeef9370cp-4,
     0x1.091b6472648aap-4, 0x1.79e8434032997p-4, 0x1.0a540c73ff6a6p-3, 0x1.0fc3ce4ae56f5p-2},
    {0x1.e1e1e1e1e1e1ep-3, 0x1.d006fad4f8422p-4, 0x1.7174dfa79a0c6p-4, 0x1.a340a6498a25fp-5,
     0x1.d41724ba1eb0ep-6, 0x1.29e20edb36d7ap-5, 0x1.b0758a722d550p-5, 0x1.a82649bbc6276p-4,
     0x1.d006fad4f8422p-4, 0x1.9587a0c5ff104p-5, 0x1.5bb7d60ecdab8p-5, 0x1.30686147041e0p-6,
     0x1.dd42c63c1ee9ap-7, 0x1.2fb80aada3823p-6, 0x1.b8ee780c0b4d9p-6, 0x1.b0758a722d550p-5,
     0x1.7174dfa79a0c6p-4, 0x1.5bb7d60ecdab8p-5, 0x1.56c4ccc94099ap-6, 0x1.aee06f988b604p-7,
     0x1.faa84b87a640ep-7, 0x1.426d2091bc880p-6, 0x1.d41724ba1eb0ep-6, 0x1.cb189f24151bap-5,
     0x1.a340a6498a25fp-5, 0x1.30686147041e0p-6, 0x1.aee06f988b604p-7, 0x1.dec3b8eb013a5p-7,
     0x1.197bd86d545b2p-6, 0x1.6642c95cb4692p-6, 0x1.040e9dc5b1e80p-5, 0x1.fe1eceb3862a3p-5,
     0x1.d41724ba1eb0ep-6, 0x1.dd42c63c1ee9ap-7, 0x1.faa84b87a640ep-7, 0x1.197bd86d545b2p-6,
     0x1.4afd6a052bf5bp-6, 0x1.a5452e0e902c0p-6, 0x1.31cb779043c4cp-5, 0x1.2beb45ad5fa49p-4,
     0x1.29e20edb36d7ap-5, 0x1.2fb80aada3823p-6, 0x1.426d2091bc880p-6, 0x1.6642c95cb4692p-6,
     0x1.a5452e0e902c0p-6, 0x1.0c167065b2265p-5, 0x1.8533f45377333p-5, 0x1.7db97a3baca55p-4,
     0x1.b0758a722d550p-5, 0x1.b8ee780c0b4d9p-6, 0x1.d41724ba1eb0ep-6, 0x1.040e9dc5b1e80p-5,
     0x1.31cb779043c4cp-5, 0x1.8533f45377333p-5, 0x1.1a847e311da71p-4, 0x1.1516cc4f4f8dbp-3,
     0x1.a82649bbc6276p-4, 0x1.b0758a722d550p-5, 0x1.cb189f24151bap-5, 0x1.fe1eceb3862a3p-5,
     0x1.2beb45ad5fa49p-4, 0x1.7db97a3baca55p-4, 0x1.1516cc4f4f8dbp-3, 0x1.0fc3ce4ae56f5p-2},
};

// Even half of the AAN transform.  T = int: exact integer prefix (rows, and the
// columns whose inputs are row outputs 0 / 4); T = double: float64.
template <typename T>
__host__ __device__ __forceinline__ void aan_even(T x0, T x1, T x2, T x3, T x4, T x5, T x6, T x7, T &o0, T &o4,
                                                   double &o2, double &o6) {
  const T s0 = x0 + x7, s1 = x1 + x6, s2 = x2 + x5, s3 = x3 + x4;
  const T t10 = s0 + s3, t13 = s0 - s3, t11 = s1 + s2, t12 = s1 - s2;
  o0 = t10 + t11;
  o4 = t10 - t11;
  const double z1 = (double)(t12 + t13) * kA1;
  o2 = (double)t13 + z1;
  o6 = (double)t13 - z1;
}
template <typename T>
__host__ __device__ __forceinline__ void aan_odd(T x0, T x1, T x2, T x3, T x4, T x5, T x6, T x7, double &o1,
                                                  double &o3, double &o5, double &o7) {
  const T d7 = x0 - x7, d6 = x1 - x6, d5 = x2 - x5, d4 = x3 - x4;
  const T u10 = d4 + d5, u11 = d5 + d6, u12 = d6 + d7;
  const double z5 = (double)(u10 - u12) * kA5;
  const double z2 = __builtin_fma(kA2, (double)u10, z5);
  const double z4 = __builtin_fma(kA4, (double)u12, z5);
  const double z3 = (double)u11 * kA1;
  const double z11 = (double)d7 + z3, z13 = (double)d7 - z3;
  o5 = z13 + z2;
  o3 = z13 - z2;
  o1 = z11 + z4;
  o7 = z11 - z4;
}

// Fast quantiser: q = round(b * r).  t = fma(b, r, 1.5*2^20 + 1/2 + 2^-30) rounds
// b*r + 1/2 + 2^-30 to a multiple of 2^-32 (|b*r| < 2^19).  The high word of its bit
// pattern is the constant's exponent over 2^19 + floor(b*r + 1/2 + 2^-30), so its
// low 16 bits are q's (all an int16 output needs: no shift, no subtract); the low
// word is the rounded fraction in units of 2^-32, offset by 4.  b*r + 1/2 within
// 2^-31 of an integer (a quantiser tie) gives a low word of 2..6, and the 2^-30
// offset can only change q where the fraction was within 2^-30 below an integer,
// which gives 0..4: `tie` keeps the minimum low word, and any value <= kTieMax
// flags the block.  The fast estimate of y/T is within 2^-41 of pocketfft's
// (tools/check/aan_err.hip, 4M blocks incl. saturated patterns), three orders of
// magnitude inside the window, so an unflagged q is pocketfft's q.
constexpr double kQMagic = 0x1.8p20 + 0.5 + 0x1p-30;
constexpr uint32_t kQHi = (uint32_t)(__builtin_bit_cast(unsigned long long, 0x1.8p20) >> 32);
constexpr uint32_t kTieMax = 6;
__host__ __device__ __forceinline__ int qfast(double b, double r, uint32_t &tie) {
  const unsigned long long t = __builtin_bit_cast(unsigned long long, __builtin_fma(b, r, kQMagic));
  const uint32_t lo = (uint32_t)t;
  tie = tie < lo ? tie : lo;
  return (int)((uint32_t)(t >> 32) - kQHi);
}

// One block on the fast path; returns true if it must be redone exactly.
template <int TABLE, int LAYOUT>
__host__ __device__ __forceinline__ bool dct_block_aan(uint2 (&w)[8], int16_t *st, bool *tie26_out = nullptr,
                                                       double *dbg = nullptr, int trt = 0) {
  const int tb = TABLE >= 0 ? TABLE : trt;
  constexpr SlotOf<LAYOUT> kSlot{};
  // dbg (host error analysis only): b * kRA, i.e. this path's estimate of y / T
  // (2,2), (2,6), (6,2), (6,6): y = A + B*sqrt(2) with rational A, B, an exact tie
  // when B = 0 (~1e-4 of random blocks).  Their ties are reported apart
  // (*tie26_out) for dct_fix26, which recomputes just these four coefficients.
  uint32_t tie26 = 0xFFFFFFFFu;
  auto qf = [&](double b, int i, uint32_t &t) {
    if (dbg) dbg[i] = b * kRA[tb][i];
    const bool c26 = (i == 18 || i == 22 || i == 50 || i == 54);
    return qfast(b, kRA[tb][i], c26 ? tie26 : t);
  };
  // raw bytes: the -128 offset of dct_channel only reaches row output 0 (the
  // DCT's other basis rows sum to zero), corrected there by -8 * 128 per row
  auto px = [&](int r, int n) -> int { return (int)(((n < 4 ? w[r].x : w[r].y) >> (8 * (n & 3))) & 0xFFu); };
  uint32_t tie = 0xFFFFFFFFu;
  // ---- even row outputs (0, 2, 4, 6) -> columns 0, 2, 4, 6
  {
    int e0[8], e4[8];
    double e2[8], e6[8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
    {
      aan_even<int>(px(r, 0), px(r, 1), px(r, 2), px(r, 3), px(r, 4), px(r, 5), px(r, 6), px(r, 7), e0[r], e4[r],
                    e2[r], e6[r]);
      e0[r] -= 8 * 128;
    }
    // column 0: integer prefix; (0,0) = the pixel sum, pocketfft's exact DC (half scale)
    {
      int c0, c4;
      double c[8];
      aan_even<int>(e0[0], e0[1], e0[2], e0[3], e0[4], e0[5], e0[6], e0[7], c0, c4, c[2], c[6]);
      aan_odd<int>(e0[0], e0[1], e0[2], e0[3], e0[4], e0[5], e0[6], e0[7], c[1], c[3], c[5], c[7]);
      st[kSlot.s[0]] = (int16_t)quant_fast<TABLE>((double)c0, 0, trt);
      st[kSlot.s[32]] = (int16_t)qf((double)c4, 32, tie);
#pragma unroll
      for (int u = 1; u < 8; ++u)
        if (u != 4) st[kSlot.s[u * 8]] = (int16_t)qf(c[u], u * 8, tie);
    }
    // column 4: integer prefix; (4,4) with pocketfft's own operation sequence
    {
      int c0, c4;
      double c[8];
      aan_even<int>(e4[0], e4[1], e4[2], e4[3], e4[4], e4[5], e4[6], e4[7], c0, c4, c[2], c[6]);
      aan_odd<int>(e4[0], e4[1], e4[2], e4[3], e4[4], e4[5], e4[6], e4[7], c[1], c[3], c[5], c[7]);
      st[kSlot.s[4]] = (int16_t)qf((double)c0, 4, tie);
#pragma unroll
      for (int u = 1; u < 8; ++u)
        if (u != 4) st[kSlot.s[u * 8 + 4]] = (int16_t)qf(c[u], u * 8 + 4, tie);
      double y[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) y[r] = (double)e4[r] * TW3;  // pocketfft row output 4 (half scale)
      const double c1 = y[1] + y[2], c3 = y[3] + y[4], c5 = y[5] + y[6], H0 = y[0] + y[7];
      const double h1 = c1 + c5, T2 = H0 + c3;
      st[kSlot.s[36]] = (int16_t)quant_fast<TABLE>((T2 - h1) * TW3, 36, trt);
    }
    // columns 2, 6
#pragma unroll
    for (int v = 2; v < 8; v += 4) {
      const double(&x)[8] = v == 2 ? e2 : e6;
      double c0, c4, c[8];
      aan_even<double>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], c0, c4, c[2], c[6]);
      aan_odd<double>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], c[1], c[3], c[5], c[7]);
      c[0] = c0;
      c[4] = c4;
#pragma unroll
      for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + v]] = (int16_t)qf(c[u], u * 8 + v, tie);
    }
  }
  // ---- odd row outputs (1, 3, 5, 7) -> columns 1, 3, 5, 7.  Re-unpack the pixels
  // (opaque w: the compiler must not keep 64 unpacked ints live across phases)
#ifdef __HIP_DEVICE_COMPILE__
  for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(w[r].x), "+v"(w[r].y));
#endif
  {
    double o[4][8];  // [v/2][row]
#pragma unroll
    for (int r = 0; r < 8; ++r)
      aan_odd<int>(px(r, 0), px(r, 1), px(r, 2), px(r, 3), px(r, 4), px(r, 5), px(r, 6), px(r, 7), o[0][r], o[1][r],
                   o[2][r], o[3][r]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int v = 2 * k + 1;
      const double(&x)[8] = o[k];
      double c0, c4, c[8];
      aan_even<double>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], c0, c4, c[2], c[6]);
      aan_odd<double>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], c[1], c[3], c[5], c[7]);
      c[0] = c0;
      c[4] = c4;
#pragma unroll
      for (int u = 0; u < 8; ++u) st[kSlot.s[u * 8 + v]] = (int16_t)qf(c[u], u * 8 + v, tie);
    }
  }
  if (tie26_out) *tie26_out = tie26 <= kTieMax;
  return tie <= kTieMax;
}

// The four (2,2)-class coefficients with pocketfft's own operations (rows' outputs
// 2 and 6, then columns 2 and 6), quantised exactly; q[] = raster (2,2), (2,6),
// (6,2), (6,6).
template <int TABLE>
__host__ __device__ __forceinline__ void dct_fix26(const uint2 (&w)[8], int (&q)[4], int trt = 0) {
  auto px = [&](int r, int n) -> int { return (int)(((n < 4 ? w[r].x : w[r].y) >> (8 * (n & 3))) & 0xFFu); };
  double y2[8], y6[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    // offsets cancel in these differences: raw bytes
    const int c2 = px(r, 2) - px(r, 1), c6 = px(r, 6) - px(r, 5);
    const int T1 = (px(r, 0) + px(r, 7)) - (px(r, 3) + px(r, 4)), h2 = c2 - c6;
    const double D6 = (double)(T1 + h2), D2 = (double)(T1 - h2);
    const double P1 = TW1 * D6 + TW5 * D2, P2 = TW1 * D2 - TW5 * D6;
    y2[r] = P1 + P2;
    y6[r] = P1 - P2;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const double(&X)[8] = k == 0 ? y2 : y6;
    const int v = k == 0 ? 2 : 6;
    const double c2 = X[2] - X[1], c6 = X[6] - X[5];
    const double T1 = (X[0] + X[7]) - (X[3] + X[4]), h2 = c2 - c6;
    const double D6 = T1 + h2, D2 = T1 - h2;
    const double P1 = TW1 * D6 + TW5 * D2, P2 = TW1 * D2 - TW5 * D6;
    q[k] = quant_fast<TABLE>(P1 + P2, 16 + v, trt);
    q[2 + k] = quant_fast<TABLE>(P1 - P2, 48 + v, trt);
  }
}


// ---------------------------------------------------------------------------
// round-half-even(4 X / T[0][0]) for the centred pixel sum X (|X| <= 8192), in
// integers: the DC is exact, and its ties (X = 2 mod 4 for T = 16) are real.
template <int TABLE>
__host__ __device__ __forceinline__ int dc_quant(int X) {
  constexpr int T = QT[TABLE][0];
  const int a = 8 * X + T;                        // 2 (4X) + T
  const int q = (a >= 0 ? a : a - (2 * T - 1)) / (2 * T);  // floor(a / 2T)
  return (a == q * 2 * T && (q & 1)) ? q - 1 : q;  // exact tie: to even
}

}  // namespace
}  // namespace hic
