// dct.hip -- 8x8 block DCT-II + quantize (encode) and dequantize + DCT-III (decode)
// for MI355X (gfx950), bit-exact against hiccup's scipy/numpy path.
//
// Reference: transform.dct_channel / inv_dct_channel (transform.py:169-193),
// transform.dct2 / idct2 (transform.py:67-103) -> scipy.fftpack.dct / idct
// (pocketfft, scipy 1.15.3), quantization.jpeg_quantize / invert_jpeg_quantize
// (quantization.py:47-57,80-81).
//
// Design (DESIGN.md "forward kernel"):
//  * one 8x8 block per lane, 64 consecutive raster-order blocks per wave, so each
//    row load (8 B/lane) and each coefficient-row store (16 B/lane) of a wave is
//    one contiguous 512 B / 1 KiB segment of HBM; no LDS, no cross-lane traffic;
//  * float64 throughout, replicating pocketfft's length-8 operation order exactly
//    (built with -ffp-contract=off; the only FMAs are explicit ones whose product
//    is exact, e.g. y*2^-8);
//  * "half-scaled" DCT-II: pocketfft's x2 / x0.5 steps are exact power-of-two
//    scalings, so they are dropped and folded into the quantizer divisor
//    (DESIGN.md derives the bookkeeping: outputs 0 and 4 come out halved);
//  * the integer-exact prefix of each row transform (pixel sums/differences) runs
//    in int32, converting to float64 only where pocketfft first rounds;
//  * quantize = rint(b * (1/D)) with a near-tie guard: when the product lies
//    within 2^-30 of a half-integer (exact .5 ties occur at DC and at (4,4)), the
//    lane recomputes rint(b / D) with the IEEE-correct divide, which is what
//    numpy does.  The guard is > 10^3 x the reciprocal's error bound.
#include <stdlib.h>

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

template <int TABLE, int LAYOUT, bool FAST>
__global__ __launch_bounds__(256) void k_dct_quant(const uint8_t *__restrict__ plane, int H, int W,
                                                   int64_t stride, int nbx, int nblk,
                                                   void *__restrict__ out) {
  constexpr SlotOf<LAYOUT> kSlot{};
  const int blk = blockIdx.x * 256 + threadIdx.x;
  if (blk >= nblk) return;
  const int bi = blk / nbx, bj = blk - bi * nbx;
  const int y0 = bi * 8, x0 = bj * 8;

  // ---- row pass (rows of the 8x8 block) ----
  int col0[8];   // y'[r][0], exact integers
  double a[8][8];  // y'[r][1..7]  (a[r][0] unused)
  if (FAST) {
    const uint8_t *p = plane + (int64_t)y0 * stride + x0;
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + r * stride);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      int x[8];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        x[n] = (int)((w[r].x >> (8 * n)) & 0xFFu) - 128;
        x[n + 4] = (int)((w[r].y >> (8 * n)) & 0xFFu) - 128;
      }
      dct8h_int(x, col0[r], a[r]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      int x[8];
      const int yy = y0 + r;
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const int xx = x0 + n;
        // pad_matrix pads the (pixel - 128) plane with 0 (transform.py:17-30)
        x[n] = (yy < H && xx < W) ? (int)plane[(int64_t)yy * stride + xx] - 128 : 0;
      }
      dct8h_int(x, col0[r], a[r]);
    }
  }

  // ---- column pass + quantize, packed to int16 in the output order ----
  uint32_t pk[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) pk[k] = 0;
  {
    int b0;
    double b[8];
    dct8h_int(col0, b0, b);
    put16(pk, kSlot.s[0], quantize<TABLE>((double)b0, 0));
#pragma unroll
    for (int u = 1; u < 8; ++u) put16(pk, kSlot.s[u * 8], quantize<TABLE>(b[u], u * 8));
  }
#pragma unroll
  for (int v = 1; v < 8; ++v) {
    double xc[8], b[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) xc[r] = a[r][v];
    dct8h(xc, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) put16(pk, kSlot.s[u * 8 + v], quantize<TABLE>(b[u], u * 8 + v));
  }

  // ---- store ----
  if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
    if (!FAST && (y0 + 8 > H || x0 + 8 > W)) {
      // positions cropped by merge_blocks are 0 when jpeg_encode re-pads
#pragma unroll
      for (int z = 0; z < 64; ++z) {
        const int u = ZZ[z] / 8, v = ZZ[z] % 8;
        if (y0 + u >= H || x0 + v >= W) pk[z >> 1] &= (z & 1) ? 0x0000FFFFu : 0xFFFF0000u;
      }
    }
    uint4 *o = reinterpret_cast<uint4 *>(static_cast<int16_t *>(out) + (int64_t)blk * 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = make_uint4(pk[4 * k], pk[4 * k + 1], pk[4 * k + 2], pk[4 * k + 3]);
  } else if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
    int16_t *o = static_cast<int16_t *>(out);
    if (FAST) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        *reinterpret_cast<uint4 *>(o + (int64_t)(y0 + u) * W + x0) =
            make_uint4(pk[4 * u], pk[4 * u + 1], pk[4 * u + 2], pk[4 * u + 3]);
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int v = 0; v < 8; ++v)
          if (y0 + u < H && x0 + v < W)
            o[(int64_t)(y0 + u) * W + x0 + v] = (int16_t)(pk[(u * 8 + v) >> 1] >> (16 * (v & 1)));
    }
  } else {  // RASTER_I32
    int32_t *o = static_cast<int32_t *>(out);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int q[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) q[v] = (int)(int16_t)(pk[(u * 8 + v) >> 1] >> (16 * (v & 1)));
      if (FAST) {
        int4 *row = reinterpret_cast<int4 *>(o + (int64_t)(y0 + u) * W + x0);
        row[0] = make_int4(q[0], q[1], q[2], q[3]);
        row[1] = make_int4(q[4], q[5], q[6], q[7]);
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v)
          if (y0 + u < H && x0 + v < W) o[(int64_t)(y0 + u) * W + x0 + v] = q[v];
      }
    }
  }
}

// ---------------------------------------------------------------------------
template <int TABLE, int LAYOUT, bool FAST>
__global__ __launch_bounds__(256) void k_dequant_idct(const void *__restrict__ coef, int H, int W,
                                                      int nbx, int nblk, uint8_t *__restrict__ out,
                                                      int64_t ostride) {
  const int blk = blockIdx.x * 256 + threadIdx.x;
  if (blk >= nblk) return;
  const int bi = blk / nbx, bj = blk - bi * nbx;
  const int y0 = bi * 8, x0 = bj * 8;

  int q[64];  // raster [u][v]
  if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
    const uint4 *src = reinterpret_cast<const uint4 *>(static_cast<const int16_t *>(coef) + (int64_t)blk * 64);
    uint32_t w[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 t = src[k];
      w[4 * k] = t.x;
      w[4 * k + 1] = t.y;
      w[4 * k + 2] = t.z;
      w[4 * k + 3] = t.w;
    }
#pragma unroll
    for (int z = 0; z < 64; ++z) q[ZZ[z]] = (int)(int16_t)(w[z >> 1] >> (16 * (z & 1)));
    if (!FAST && (y0 + 8 > H || x0 + 8 > W)) {
#pragma unroll
      for (int i = 0; i < 64; ++i)
        if (y0 + i / 8 >= H || x0 + i % 8 >= W) q[i] = 0;
    }
  } else if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
    const int16_t *c = static_cast<const int16_t *>(coef);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (FAST) {
        const uint4 t = *reinterpret_cast<const uint4 *>(c + (int64_t)(y0 + u) * W + x0);
        const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int v = 0; v < 8; ++v) q[u * 8 + v] = (int)(int16_t)(w[v >> 1] >> (16 * (v & 1)));
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v)
          q[u * 8 + v] = (y0 + u < H && x0 + v < W) ? (int)c[(int64_t)(y0 + u) * W + x0 + v] : 0;
      }
    }
  } else {
    const int32_t *c = static_cast<const int32_t *>(coef);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (FAST) {
        const int4 *row = reinterpret_cast<const int4 *>(c + (int64_t)(y0 + u) * W + x0);
        const int4 t0 = row[0], t1 = row[1];
        q[u * 8 + 0] = t0.x; q[u * 8 + 1] = t0.y; q[u * 8 + 2] = t0.z; q[u * 8 + 3] = t0.w;
        q[u * 8 + 4] = t1.x; q[u * 8 + 5] = t1.y; q[u * 8 + 6] = t1.z; q[u * 8 + 7] = t1.w;
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v)
          q[u * 8 + v] = (y0 + u < H && x0 + v < W) ? c[(int64_t)(y0 + u) * W + x0 + v] : 0;
      }
    }
  }

  // dequantize (q * T, exact in int32) and row pass
  double a[8][8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    int c[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) c[v] = q[u * 8 + v] * QT[TABLE][u * 8 + v];
    idct8<int>(c, a[u]);
  }
  // column pass, /256 (exact) + 128, truncate toward zero, wrap mod 256
  uint32_t px[16];  // row r: bytes v = 0..3 in px[2r], 4..7 in px[2r+1]
#pragma unroll
  for (int k = 0; k < 16; ++k) px[k] = 0;
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    double xc[8], yv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xc[u] = a[u][v];
    idct8<double>(xc, yv);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double p = __builtin_fma(yv[r], 0x1p-8, 128.0);  // == fl(y/256 + 128): y*2^-8 exact
      const uint32_t b = (uint32_t)__double2int_rz(p) & 0xFFu;
      px[2 * r + (v >> 2)] |= b << (8 * (v & 3));
    }
  }
  if (FAST) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      *reinterpret_cast<uint2 *>(out + (int64_t)(y0 + r) * ostride + x0) = make_uint2(px[2 * r], px[2 * r + 1]);
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int v = 0; v < 8; ++v)
        if (y0 + r < H && x0 + v < W)
          out[(int64_t)(y0 + r) * ostride + x0 + v] = (uint8_t)(px[2 * r + (v >> 2)] >> (8 * (v & 3)));
  }
}

// ---------------------------------------------------------------------------
// Streaming forward kernel for aligned planes (the production path).
//  * one 8x8 block per lane (the instruction-cheapest mapping: ~19 fp64 wave
//    instructions per block), 64 consecutive raster-order blocks ("a set") per
//    wave iteration;
//  * persistent grid (~2 waves per SIMD, what the 220-VGPR body allows) with the
//    next set's eight 8-byte row loads issued before the current set's math, so
//    HBM latency hides under ~5k cycles of float64 work;
//  * quantizer: fma(b, 1/D, 1.5*2^33) rounds b/D to 2^-19 in the low mantissa
//    bits, giving q = (N + 2^18) >> 19 and an exact integer near-tie test (low 19
//    bits == 2^18 <=> |b/D - (k + 1/2)| <~ 2^-20, 10^6 x the reciprocal's error
//    bound); flagged lanes recompute numpy's rint(b / D) with the IEEE divide;
//  * zig-zag output staged through LDS so every store instruction writes one
//    contiguous 1 KiB segment.
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

template <int TABLE, int LAYOUT>
__global__ __launch_bounds__(256) void k_dct_quant_stream(const uint8_t *__restrict__ plane, int64_t stride, int W,
                                                          int nbx, int nblk, int nsets, void *__restrict__ out) {
  __shared__ uint4 s_stage[LAYOUT == HIC_LAYOUT_ZIGZAG_I16 ? 4 * 64 * kStagePad : 1];
  constexpr SlotOf<LAYOUT> kSlot{};
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  int set = blockIdx.x * 4 + wv;

  auto load_rows = [&](int st, uint2(&w)[8]) {
    int blk = st * 64 + lane;
    if (blk >= nblk) blk = nblk - 1;
    const int bi = blk / nbx, bj = blk - bi * nbx;
    const uint8_t *p = plane + (int64_t)bi * 8 * stride + bj * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + r * stride);
  };

  uint2 nxt[8];
  if (set < nsets) load_rows(set, nxt);
  for (; set < nsets; set += nwaves) {
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = nxt[r];
    if (set + nwaves < nsets) load_rows(set + nwaves, nxt);
    const int blk = set * 64 + lane;

    int col0[8];
    double a[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      int x[8];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        x[n] = (int)((w[r].x >> (8 * n)) & 0xFFu) - 128;
        x[n + 4] = (int)((w[r].y >> (8 * n)) & 0xFFu) - 128;
      }
      dct8h_int(x, col0[r], a[r]);
    }
    uint32_t pk[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) pk[k] = 0;
    {
      int b0;
      double b[8];
      dct8h_int(col0, b0, b);
      put16(pk, kSlot.s[0], quant_fast<TABLE>((double)b0, 0));
#pragma unroll
      for (int u = 1; u < 8; ++u) put16(pk, kSlot.s[u * 8], quant_fast<TABLE>(b[u], u * 8));
    }
#pragma unroll
    for (int v = 1; v < 8; ++v) {
      double xc[8], b[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) xc[r] = a[r][v];
      dct8h(xc, b);
#pragma unroll
      for (int u = 0; u < 8; ++u) put16(pk, kSlot.s[u * 8 + v], quant_fast<TABLE>(b[u], u * 8 + v));
    }

    if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
      uint4 *st = s_stage + wv * 64 * kStagePad;
#pragma unroll
      for (int k = 0; k < 8; ++k) st[lane * kStagePad + k] = make_uint4(pk[4 * k], pk[4 * k + 1], pk[4 * k + 2], pk[4 * k + 3]);
      __builtin_amdgcn_wave_barrier();
      uint4 *o = reinterpret_cast<uint4 *>(static_cast<int16_t *>(out) + (int64_t)set * 64 * 64);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int b = 8 * k + (lane >> 3);  // block (within the set) of this lane's 16 bytes
        const uint4 v = st[b * kStagePad + (lane & 7)];
        if (set * 64 + b < nblk) o[64 * k + lane] = v;
      }
      __builtin_amdgcn_wave_barrier();
    } else if (blk < nblk) {
      const int bi = blk / nbx, bj = blk - bi * nbx;
      if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
        int16_t *o = static_cast<int16_t *>(out) + (int64_t)bi * 8 * W + bj * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          *reinterpret_cast<uint4 *>(o + (int64_t)u * W) = make_uint4(pk[4 * u], pk[4 * u + 1], pk[4 * u + 2], pk[4 * u + 3]);
      } else {
        int32_t *o = static_cast<int32_t *>(out) + (int64_t)bi * 8 * W + bj * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          int q[8];
#pragma unroll
          for (int v = 0; v < 8; ++v) q[v] = (int)(int16_t)(pk[(u * 8 + v) >> 1] >> (16 * (v & 1)));
          int4 *row = reinterpret_cast<int4 *>(o + (int64_t)u * W);
          row[0] = make_int4(q[0], q[1], q[2], q[3]);
          row[1] = make_int4(q[4], q[5], q[6], q[7]);
        }
      }
    }
  }
}

// Two-phase variant: the row transform is split into its even outputs
// (0, 2, 4, 6: the k=0 butterfly + the (2,6) twiddle pair) and odd outputs
// (1, 3, 5, 7: k=1 butterfly + the (1,7), (3,5) pairs).  Phase A computes the
// even outputs of all 8 rows and runs the four even-column transforms; phase B
// the odd ones.  Quantized coefficients go straight to their zig-zag slot in an
// LDS stage.  Live state is ~half of the one-pass kernel's, so ~4 waves fit per
// SIMD, at the cost of recomputing 4 integer sums per row.
template <int TABLE, int LAYOUT>
__global__ __launch_bounds__(256) void k_dct_quant_2ph(const uint8_t *__restrict__ plane, int64_t stride, int W,
                                                       int nbx, int nblk, int nsets, void *__restrict__ out) {
  __shared__ uint4 s_stage[4 * 64 * kStagePad];
  constexpr SlotOf<LAYOUT> kSlot{};
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  uint4 *st4 = s_stage + wv * 64 * kStagePad;
  int16_t *st = reinterpret_cast<int16_t *>(st4 + lane * kStagePad);

  for (int set = blockIdx.x * 4 + wv; set < nsets; set += nwaves) {
    int blk = set * 64 + lane;
    const int cblk = blk < nblk ? blk : nblk - 1;
    const int bi = cblk / nbx, bj = cblk - bi * nbx;
    const uint8_t *p = plane + (int64_t)bi * 8 * stride + bj * 8;
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + r * stride);
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
    __builtin_amdgcn_wave_barrier();
    if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
      uint4 *o = reinterpret_cast<uint4 *>(static_cast<int16_t *>(out) + (int64_t)set * 64 * 64);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int b = 8 * k + (lane >> 3);
        const uint4 v = st4[b * kStagePad + (lane & 7)];
        if (set * 64 + b < nblk) o[64 * k + lane] = v;
      }
    } else if (blk < nblk) {
      if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
        int16_t *o = static_cast<int16_t *>(out) + (int64_t)bi * 8 * W + bj * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u) *reinterpret_cast<uint4 *>(o + (int64_t)u * W) = st4[lane * kStagePad + u];
      } else {
        int32_t *o = static_cast<int32_t *>(out) + (int64_t)bi * 8 * W + bj * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint4 t = st4[lane * kStagePad + u];
          const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
          int q[8];
#pragma unroll
          for (int v = 0; v < 8; ++v) q[v] = (int)(int16_t)(wd[v >> 1] >> (16 * (v & 1)));
          int4 *row = reinterpret_cast<int4 *>(o + (int64_t)u * W);
          row[0] = make_int4(q[0], q[1], q[2], q[3]);
          row[1] = make_int4(q[4], q[5], q[6], q[7]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

inline int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      n = prop.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

// ---------------------------------------------------------------------------
// Block-level helpers (transform.dct2 / idct2, quantization.jpeg_quantize /
// invert_jpeg_quantize on arbitrary float64 / int blocks): one block per lane.
__global__ __launch_bounds__(256) void k_dct2_f64(const double *__restrict__ in, int64_t nblk, double *__restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  const double *p = in + b * 64;
  double a[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    double x[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) x[n] = p[r * 8 + n];
    dct8h(x, a[r]);
  }
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    double xc[8], y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) xc[r] = a[r][v];
    dct8h(xc, y);
#pragma unroll
    for (int u = 0; u < 8; ++u) out[b * 64 + u * 8 + v] = y[u] / (rho(u) * rho(v));  // exact power-of-2 rescale
  }
}

__global__ __launch_bounds__(256) void k_idct2_f64(const double *__restrict__ in, int64_t nblk, double *__restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  const double *p = in + b * 64;
  double a[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    double x[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) x[n] = p[r * 8 + n];
    idct8<double>(x, a[r]);
  }
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    double xc[8], y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) xc[r] = a[r][v];
    idct8<double>(xc, y);
#pragma unroll
    for (int r = 0; r < 8; ++r) out[b * 64 + r * 8 + v] = y[r] * 0x1p-8;  // == y / 256
  }
}

__global__ void k_quantize_f64(const double *__restrict__ in, int64_t n, int table, int32_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (int32_t)__builtin_rint(in[i] / (double)QT[table][i & 63]);
}

__global__ void k_dequantize_i32(const int32_t *__restrict__ in, int64_t n, int table, int64_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (int64_t)in[i] * QT[table][i & 63];
}

// ---------------------------------------------------------------------------
// Paired-lane forward kernel (interior / aligned planes).  Lanes l and l+32 of a
// wave share one 8x8 block: lane l does the row pass of rows 0-3, lane l+32 of
// rows 4-7; one v_permlane32_swap per dword then hands each lane the four
// columns it transforms in the column pass (l: columns 0-3, l+32: columns 4-7).
// Half the per-lane state of the one-lane-per-block kernel -> twice the waves.
__device__ __forceinline__ void swap_halves(double &x, double &y) {
  // lanes 32-63 of x <-> lanes 0-31 of y
  const unsigned long long xb = (unsigned long long)__double_as_longlong(x);
  const unsigned long long yb = (unsigned long long)__double_as_longlong(y);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)xb, (unsigned)yb, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(xb >> 32), (unsigned)(yb >> 32), false, false);
  x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}

__device__ __forceinline__ void swap_halves_u32(uint32_t &x, uint32_t &y) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

// quantize coefficient with raster index i0 (lanes 0-31) or i1 (lanes 32-63)
template <int TABLE>
__device__ __forceinline__ int quantize_sel(double b, bool hi, int i0, int i1) {
  const double r = hi ? kQ.r[TABLE][i1] : kQ.r[TABLE][i0];
  const double p = b * r;
  double q = __builtin_rint(p);
  // the product is exact when D is a power of two (rint is then already numpy's answer)
  const bool exact = hi ? pow2(kQ.d[TABLE][i1]) : pow2(kQ.d[TABLE][i0]);
  if (!exact && __builtin_fabs(p - q) > 0.5 - 0x1p-30) {
    const double d = hi ? kQ.d[TABLE][i1] : kQ.d[TABLE][i0];
    q = __builtin_rint(b / d);
  }
  return (int)q;
}

template <int TABLE, int LAYOUT>
__global__ __launch_bounds__(256) void k_dct_quant_pair(const uint8_t *__restrict__ plane, int64_t stride, int W,
                                                        int nbx, int nblk, void *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const bool hi = h != 0;
  int blk = ((blockIdx.x * 256 + threadIdx.x) >> 6) * 32 + (lane & 31);
  const bool active = blk < nblk;
  if (!active) blk = nblk - 1;  // every lane stays alive for the cross-lane swaps
  const int bi = blk / nbx, bj = blk - bi * nbx;
  const int y0 = bi * 8, x0 = bj * 8;

  const uint8_t *p = plane + (int64_t)(y0 + 4 * h) * stride + x0;
  uint2 w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = *reinterpret_cast<const uint2 *>(p + i * stride);
  double A[4][4], B[4][4];  // B: columns 0-3, A: columns 4-7 of this lane's four rows
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int x[8];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      x[n] = (int)((w[i].x >> (8 * n)) & 0xFFu) - 128;
      x[n + 4] = (int)((w[i].y >> (8 * n)) & 0xFFu) - 128;
    }
    int c0;
    double y[8];
    dct8h_int(x, c0, y);
    B[i][0] = (double)c0;
#pragma unroll
    for (int j = 1; j < 4; ++j) B[i][j] = y[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) A[i][j] = y[4 + j];
  }
  // lanes 0-31 keep B (rows 0-3) and receive rows 4-7 of columns 0-3 into A;
  // lanes 32-63 keep A (rows 4-7) and receive rows 0-3 of columns 4-7 into B.
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) swap_halves(B[i][j], A[i][j]);

  uint32_t pk[16];  // raster int16 of this lane's 4 columns: row u -> pk[2u], pk[2u+1]
#pragma unroll
  for (int k = 0; k < 16; ++k) pk[k] = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double xc[8] = {B[0][j], B[1][j], B[2][j], B[3][j], A[0][j], A[1][j], A[2][j], A[3][j]};
    double b[8];
    dct8h(xc, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = quantize_sel<TABLE>(b[u], hi, u * 8 + j, u * 8 + 4 + j);
      pk[2 * u + (j >> 1)] |= ((uint32_t)q & 0xFFFFu) << (16 * (j & 1));
    }
  }

  if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
    uint32_t L[16], R[16];  // after the swap: L = columns 0-3, R = columns 4-7 (all lanes)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      L[k] = pk[k];
      R[k] = pk[k];
      swap_halves_u32(L[k], R[k]);
    }
    // value at raster index r as a 16-bit field
    auto field = [&](int r) -> uint32_t {
      const int u = r / 8, v = r % 8;
      const uint32_t wd = v < 4 ? L[2 * u + (v >> 1)] : R[2 * u + ((v - 4) >> 1)];
      return (v & 1) ? (wd >> 16) : (wd & 0xFFFFu);
    };
    uint32_t zw[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t lo = field(ZZ[2 * k]) | (field(ZZ[2 * k + 1]) << 16);
      const uint32_t up = field(ZZ[32 + 2 * k]) | (field(ZZ[32 + 2 * k + 1]) << 16);
      zw[k] = hi ? up : lo;
    }
    if (active) {
      uint4 *o = reinterpret_cast<uint4 *>(static_cast<int16_t *>(out) + (int64_t)blk * 64 + 32 * h);
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = make_uint4(zw[4 * k], zw[4 * k + 1], zw[4 * k + 2], zw[4 * k + 3]);
    }
  } else if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
    if (active) {
      int16_t *o = static_cast<int16_t *>(out) + (int64_t)y0 * W + x0 + 4 * h;
#pragma unroll
      for (int u = 0; u < 8; ++u) *reinterpret_cast<uint2 *>(o + (int64_t)u * W) = make_uint2(pk[2 * u], pk[2 * u + 1]);
    }
  } else {
    if (active) {
      int32_t *o = static_cast<int32_t *>(out) + (int64_t)y0 * W + x0 + 4 * h;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        *reinterpret_cast<int4 *>(o + (int64_t)u * W) =
            make_int4((int)(int16_t)pk[2 * u], (int)(int16_t)(pk[2 * u] >> 16), (int)(int16_t)pk[2 * u + 1],
                      (int)(int16_t)(pk[2 * u + 1] >> 16));
    }
  }
}

// Paired-lane inverse kernel (interior / aligned planes): lane l dequantizes and
// row-transforms coefficient rows 0-3, lane l+32 rows 4-7; after the half swap
// lane l column-transforms pixel columns 0-3 and lane l+32 columns 4-7.
template <int TABLE, int LAYOUT>
__global__ __launch_bounds__(256) void k_dequant_idct_pair(const void *__restrict__ coef, int W, int nbx, int nblk,
                                                           uint8_t *__restrict__ out, int64_t ostride) {
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const bool hi = h != 0;
  int blk = ((blockIdx.x * 256 + threadIdx.x) >> 6) * 32 + (lane & 31);
  const bool active = blk < nblk;
  if (!active) blk = nblk - 1;
  const int bi = blk / nbx, bj = blk - bi * nbx;
  const int y0 = bi * 8, x0 = bj * 8;

  int q[4][8];  // coefficient rows 4h + i
  if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
    const uint4 *src = reinterpret_cast<const uint4 *>(static_cast<const int16_t *>(coef) + (int64_t)blk * 64 + 32 * h);
    uint32_t L[16], R[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 t = src[k];
      L[4 * k] = t.x; L[4 * k + 1] = t.y; L[4 * k + 2] = t.z; L[4 * k + 3] = t.w;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      R[k] = L[k];
      swap_halves_u32(L[k], R[k]);  // now L = zig-zag words 0-15, R = words 16-31
    }
    auto zfield = [&](int z) -> int {
      const uint32_t wd = z < 32 ? L[z >> 1] : R[(z - 32) >> 1];
      return (int)(int16_t)((z & 1) ? (wd >> 16) : (wd & 0xFFFFu));
    };
    constexpr SlotOf<HIC_LAYOUT_ZIGZAG_I16> kZ{};  // raster index -> zig-zag position
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int v = 0; v < 8; ++v) q[i][v] = hi ? zfield(kZ.s[(4 + i) * 8 + v]) : zfield(kZ.s[i * 8 + v]);
  } else if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
    const int16_t *c = static_cast<const int16_t *>(coef) + (int64_t)(y0 + 4 * h) * W + x0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 t = *reinterpret_cast<const uint4 *>(c + (int64_t)i * W);
      const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int v = 0; v < 8; ++v) q[i][v] = (int)(int16_t)(wd[v >> 1] >> (16 * (v & 1)));
    }
  } else {
    const int32_t *c = static_cast<const int32_t *>(coef) + (int64_t)(y0 + 4 * h) * W + x0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int4 t0 = reinterpret_cast<const int4 *>(c + (int64_t)i * W)[0];
      const int4 t1 = reinterpret_cast<const int4 *>(c + (int64_t)i * W)[1];
      q[i][0] = t0.x; q[i][1] = t0.y; q[i][2] = t0.z; q[i][3] = t0.w;
      q[i][4] = t1.x; q[i][5] = t1.y; q[i][6] = t1.z; q[i][7] = t1.w;
    }
  }

  double A[4][4], B[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int c[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int t = hi ? QT[TABLE][(4 + i) * 8 + v] : QT[TABLE][i * 8 + v];
      c[v] = q[i][v] * t;
    }
    double y[8];
    idct8<int>(c, y);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      B[i][j] = y[j];
      A[i][j] = y[4 + j];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) swap_halves(B[i][j], A[i][j]);

  uint32_t px[8];  // pixel row r: bytes of columns 4h .. 4h+3
#pragma unroll
  for (int r = 0; r < 8; ++r) px[r] = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double xc[8] = {B[0][j], B[1][j], B[2][j], B[3][j], A[0][j], A[1][j], A[2][j], A[3][j]};
    double yv[8];
    idct8<double>(xc, yv);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double pv = __builtin_fma(yv[r], 0x1p-8, 128.0);  // == fl(y/256 + 128)
      px[r] |= ((uint32_t)__double2int_rz(pv) & 0xFFu) << (8 * j);
    }
  }
  if (active) {
    uint8_t *o = out + (int64_t)y0 * ostride + x0 + 4 * h;
#pragma unroll
    for (int r = 0; r < 8; ++r) *reinterpret_cast<uint32_t *>(o + (int64_t)r * ostride) = px[r];
  }
}

inline bool aligned(const void *p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

// Dev/A-B knob (not part of the ABI contract): HIC_DCT_VARIANT=single forces the
// one-lane-per-block kernel on aligned planes.
inline int dct_variant() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("HIC_DCT_VARIANT");
    v = !e ? 3 : (e[0] == 's' && e[1] == 'i') ? 1 : (e[0] == 'p') ? 2 : (e[0] == 's' && e[1] == 't') ? 0 : 3;
  }
  return v;
}

template <int TABLE, int LAYOUT>
int launch_fwd(const uint8_t *plane, int H, int W, int64_t stride, void *out, hipStream_t s) {
  const int nbx = (W + 7) / 8, nby = (H + 7) / 8, nblk = nbx * nby;
  const bool fast = (H % 8 == 0) && (W % 8 == 0) && (stride % 8 == 0) && aligned(plane, 8) && aligned(out, 16);
  const dim3 grid((nblk + 255) / 256), block(256);
  if (fast && dct_variant() == 3) {
    const int nsets = (nblk + 63) / 64;
    const int waves = nsets < 16 * cu_count() ? nsets : 16 * cu_count();  // ~4 waves per SIMD
    hipLaunchKernelGGL((k_dct_quant_2ph<TABLE, LAYOUT>), dim3((waves + 3) / 4), block, 0, s, plane, stride, W, nbx,
                       nblk, nsets, out);
  } else if (fast && dct_variant() == 0) {
    const int nsets = (nblk + 63) / 64;
    const int waves = nsets < 8 * cu_count() ? nsets : 8 * cu_count();  // ~2 waves per SIMD
    hipLaunchKernelGGL((k_dct_quant_stream<TABLE, LAYOUT>), dim3((waves + 3) / 4), block, 0, s, plane, stride, W, nbx,
                       nblk, nsets, out);
  } else if (fast && dct_variant() == 1) {
    hipLaunchKernelGGL((k_dct_quant<TABLE, LAYOUT, true>), grid, block, 0, s, plane, H, W, stride, nbx, nblk, out);
  } else if (fast) {
    const dim3 pgrid((nblk + 127) / 128);  // 32 blocks per wave, 4 waves per workgroup
    hipLaunchKernelGGL((k_dct_quant_pair<TABLE, LAYOUT>), pgrid, block, 0, s, plane, stride, W, nbx, nblk, out);
  } else
    hipLaunchKernelGGL((k_dct_quant<TABLE, LAYOUT, false>), grid, block, 0, s, plane, H, W, stride, nbx, nblk, out);
  return check_launch("k_dct_quant");
}

template <int TABLE, int LAYOUT>
int launch_inv(const void *coef, int H, int W, uint8_t *out, int64_t ostride, hipStream_t s) {
  const int nbx = (W + 7) / 8, nby = (H + 7) / 8, nblk = nbx * nby;
  const bool fast = (H % 8 == 0) && (W % 8 == 0) && (ostride % 8 == 0) && aligned(out, 8) && aligned(coef, 16);
  const dim3 grid((nblk + 255) / 256), block(256);
  if (fast && dct_variant() != 2) {
    hipLaunchKernelGGL((k_dequant_idct<TABLE, LAYOUT, true>), grid, block, 0, s, coef, H, W, nbx, nblk, out, ostride);
  } else if (fast) {
    const dim3 pgrid((nblk + 127) / 128);
    hipLaunchKernelGGL((k_dequant_idct_pair<TABLE, LAYOUT>), pgrid, block, 0, s, coef, W, nbx, nblk, out, ostride);
  } else
    hipLaunchKernelGGL((k_dequant_idct<TABLE, LAYOUT, false>), grid, block, 0, s, coef, H, W, nbx, nblk, out, ostride);
  return check_launch("k_dequant_idct");
}

bool dims_ok(int64_t H, int64_t W) {
  // one lane per block, int32 block / element indices
  return H > 0 && W > 0 && H < (1 << 20) && W < (1 << 20) && ((H + 7) / 8) * ((W + 7) / 8) < (1LL << 31) / 256;
}

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" int hic_dct_quant_u8(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                                int layout, void *out, void *stream) {
  if (!plane || !out) return arg_error("null pointer");
  if (!dims_ok(H, W) || stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  hipStream_t s = as_stream(stream);
  const int h = (int)H, w = (int)W;
#define HIC_FWD(T, L) return launch_fwd<T, L>(plane, h, w, stride, out, s)
  if (table_id == 0) {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_FWD(0, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_FWD(0, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_FWD(0, HIC_LAYOUT_ZIGZAG_I16);
  } else {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_FWD(1, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_FWD(1, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_FWD(1, HIC_LAYOUT_ZIGZAG_I16);
  }
#undef HIC_FWD
  return arg_error("layout");
}

extern "C" int hic_dequant_idct_u8(const void *coef, int layout, int64_t H, int64_t W, int table_id,
                                   uint8_t *out, int64_t out_stride, void *stream) {
  if (!coef || !out) return arg_error("null pointer");
  if (!dims_ok(H, W) || out_stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  hipStream_t s = as_stream(stream);
  const int h = (int)H, w = (int)W;
#define HIC_INV(T, L) return launch_inv<T, L>(coef, h, w, out, out_stride, s)
  if (table_id == 0) {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_INV(0, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_INV(0, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_INV(0, HIC_LAYOUT_ZIGZAG_I16);
  } else {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_INV(1, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_INV(1, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_INV(1, HIC_LAYOUT_ZIGZAG_I16);
  }
#undef HIC_INV
  return arg_error("layout");
}

extern "C" int hic_dct2_f64(const double *in, int64_t nblk, double *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  hipLaunchKernelGGL(k_dct2_f64, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, as_stream(stream), in, nblk, out);
  return check_launch("k_dct2_f64");
}

extern "C" int hic_idct2_f64(const double *in, int64_t nblk, double *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  hipLaunchKernelGGL(k_idct2_f64, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, as_stream(stream), in, nblk, out);
  return check_launch("k_idct2_f64");
}

extern "C" int hic_quantize_f64(const double *in, int64_t nblk, int table_id, int32_t *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (table_id != 0 && table_id != 1) return arg_error("table_id");
  const int64_t n = nblk * 64;
  hipLaunchKernelGGL(k_quantize_f64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), in, n,
                     table_id, out);
  return check_launch("k_quantize_f64");
}

extern "C" int hic_dequantize_i32(const int32_t *in, int64_t nblk, int table_id, int64_t *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (table_id != 0 && table_id != 1) return arg_error("table_id");
  const int64_t n = nblk * 64;
  hipLaunchKernelGGL(k_dequantize_i32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), in, n,
                     table_id, out);
  return check_launch("k_dequantize_i32");
}
