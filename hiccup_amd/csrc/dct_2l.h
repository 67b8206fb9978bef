// dct_2l.h -- the float64 AAN forward 8x8 DCT + quantiser with TWO lanes per block
// (k_dct_2l in dct.hip; DESIGN.md section 5 "Two lanes per block, round 5").
//
// Reference: transform.dct_channel (transform.py:182-193) = dct2 (:67-84, scipy's
// pocketfft DCT-II) + jpeg_quantize (quantization.py:47-52: round-half-even(y / T)).
//
// The arithmetic is dct_block_aan's (dct_core.h), operation for operation, so its
// proof (tools/check/dct_bounds.py, E64: an unflagged q equals numpy's) holds
// unchanged; only the lane mapping differs.  dct_block_aan holds one block per lane
// (~150 VGPRs: 3 waves per SIMD).  Here lane l of a wave owns half of block
// b = l & 31 of a 32-block half set, h = l >> 5:
//   rows:    lane h runs the row transform of pixel rows 4h .. 4h + 3 (the integer
//            prefix, outputs 0 / 4 as int, the rest float64);
//   swap:    one v_permlane32_swap per 32-bit word hands lane b the rows 4..7 of
//            row outputs 0..3 and lane b + 32 the rows 0..3 of outputs 4..7
//            (28 swaps per lane);
//   columns: lane h transforms columns 4h .. 4h + 3 (all eight rows) and quantises
//            its 32 coefficients: the constants kRA[table][8u + 4h + c] are per
//            lane, so they come from an LDS copy (ds_read_b64 at an immediate
//            offset from a per-lane base), and the int16 results go to the block's
//            stage row in raster order (offset 16h + 2(8u + c): per-lane base,
//            immediate offset); the zig-zag permutation happens on the way out
//            (a gather of 8 int16 per 16-byte output chunk, dct.hip).
// Column slot c = 0 is an integer column in both halves (column 0: the DC, exact
// (pixel sum) ; column 4: the (4,4) coefficient with pocketfft's own operations), so
// the two halves execute the same instructions apart from those two coefficients.
#pragma once
#include "dct_core.h"

namespace hic {
namespace {

// v_permlane32_swap of one 32-bit word pair (a: the lane's column-c value, b: its
// column-(c + 4) value): afterwards, in both halves, a holds row r and b row r + 4 of
// the lane's own column c + 4h
__device__ __forceinline__ void swap_2l(uint32_t &a, uint32_t &b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void swap_2l(int &a, int &b) {
  uint32_t x = (uint32_t)a, y = (uint32_t)b;
  swap_2l(x, y);
  a = (int)x;
  b = (int)y;
}
__device__ __forceinline__ void swap_2l(double &a, double &b) {
  uint64_t x = __builtin_bit_cast(uint64_t, a), y = __builtin_bit_cast(uint64_t, b);
  uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32), yl = (uint32_t)y, yh = (uint32_t)(y >> 32);
  swap_2l(xl, yl);
  swap_2l(xh, yh);
  a = __builtin_bit_cast(double, (uint64_t)xh << 32 | xl);
  b = __builtin_bit_cast(double, (uint64_t)yh << 32 | yl);
}

// Lane's half of one block: pixel rows 4h .. 4h + 3 (w), quantised coefficients of
// columns 4h .. 4h + 3 written to the block's raster stage row (st: the row's byte
// address + 8h, i.e. column 4h of row u at st + 16u), the quantiser constants from
// the LDS table kra (kRA[table][0..63], double).  tie / tie26 as in dct_block_aan:
// the minimum low word of every qfast (the (2,2)-class coefficients apart); the
// block needs the exact replica if either half's tie <= kTieMax, dct_fix26 if only
// a tie26 is.  TABLE: -1 = `trt` at run time.
template <int TABLE>
__device__ __forceinline__ void dct_half_2l(uint2 (&w)[4], uint8_t *st, const double *kra, int h, uint32_t &tie,
                                            uint32_t &tie26, int trt) {
  auto px = [&](int r, int n) -> int { return (int)(((n < 4 ? w[r].x : w[r].y) >> (8 * (n & 3))) & 0xFFu); };
  auto put = [&](int u, int c, int q) { *reinterpret_cast<int16_t *>(st + 16 * u + 2 * c) = (int16_t)q; };
  auto qf = [&](double b, int u, int c, uint32_t &t) { return qfast(b, kra[8 * u + c], t); };
  // one float64 column slot cs (column cs + 4h) from its eight row values
  auto column = [&](const double (&X)[8], int cs) {
    double c0, c4, c[8];
    aan_even<double>(X[0], X[1], X[2], X[3], X[4], X[5], X[6], X[7], c0, c4, c[2], c[6]);
    aan_odd<double>(X[0], X[1], X[2], X[3], X[4], X[5], X[6], X[7], c[1], c[3], c[5], c[7]);
    c[0] = c0;
    c[4] = c4;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      // (2,2), (2,6), (6,2), (6,6): column slot 2, rows 2 and 6, in both halves
      const bool c26 = cs == 2 && (u == 2 || u == 6);
      put(u, cs, qf(c[u], u, cs, c26 ? tie26 : tie));
    }
  };
  // Two phases, as dct_block_aan: the rows' even outputs (0, 2, 4, 6) feed column
  // slots 0 and 2, then the odd outputs (1, 3, 5, 7) slots 1 and 3 (the pixels stay
  // live and are unpacked again: half the row state at a time)
  {
    int e0[4], e4[4];
    double e2[4], e6[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      aan_even<int>(px(r, 0), px(r, 1), px(r, 2), px(r, 3), px(r, 4), px(r, 5), px(r, 6), px(r, 7), e0[r], e4[r],
                    e2[r], e6[r]);
      e0[r] -= 8 * 128;
    }
    // ---- column slot 0: column 0 (h = 0) or 4 (h = 1), integer inputs
    int X[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int a = e0[r], b = e4[r];
      swap_2l(a, b);
      X[r] = a;
      X[r + 4] = b;
    }
    int c0, c4;
    double c[8];
    aan_even<int>(X[0], X[1], X[2], X[3], X[4], X[5], X[6], X[7], c0, c4, c[2], c[6]);
    aan_odd<int>(X[0], X[1], X[2], X[3], X[4], X[5], X[6], X[7], c[1], c[3], c[5], c[7]);
    // u = 0: (0,0) = the pixel sum (quant_fast, exact) / (0,4) the fast quantiser;
    // u = 4: (4,0) the fast quantiser / (4,4) pocketfft's operations on the rows'
    // integer outputs 4 (the upper half's X)
    int q0, q4;
    if (h == 0) {
      q0 = quant_fast<TABLE>((double)c0, 0, trt);
      q4 = qf((double)c4, 4, 0, tie);
    } else {
      q0 = qf((double)c0, 0, 0, tie);
      double y[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) y[r] = (double)X[r] * TW3;
      const double f1 = y[1] + y[2], f3 = y[3] + y[4], f5 = y[5] + y[6], H0 = y[0] + y[7];
      const double h1 = f1 + f5, T2 = H0 + f3;
      q4 = quant_fast<TABLE>((T2 - h1) * TW3, 36, trt);
    }
    put(0, 0, q0);
    put(4, 0, q4);
#pragma unroll
    for (int u = 1; u < 8; ++u)
      if (u != 4) put(u, 0, qf(c[u], u, 0, tie));
    // ---- column slot 2: column 2 (h = 0) or 6 (h = 1)
    double Y[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double a = e2[r], b = e6[r];
      swap_2l(a, b);
      Y[r] = a;
      Y[r + 4] = b;
    }
    column(Y, 2);
  }
  // ---- column slots 1 and 3: columns 1, 3 (h = 0) or 5, 7 (h = 1)
#ifdef __HIP_DEVICE_COMPILE__
  for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(w[r].x), "+v"(w[r].y));
#endif
  {
    double o[4][4];  // [row][k]: row outputs 1, 3, 5, 7
#pragma unroll
    for (int r = 0; r < 4; ++r)
      aan_odd<int>(px(r, 0), px(r, 1), px(r, 2), px(r, 3), px(r, 4), px(r, 5), px(r, 6), px(r, 7), o[r][0], o[r][1],
                   o[r][2], o[r][3]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      double Y[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double a = o[r][k], b = o[r][k + 2];
        swap_2l(a, b);
        Y[r] = a;
        Y[r + 4] = b;
      }
      column(Y, 2 * k + 1);
    }
  }
}

// zig-zag position z -> byte offset of its int16 in a raster stage row (2 ZZ[z])
struct ZzOff {
  uint16_t o[64];
  constexpr ZzOff() : o() {
    for (int z = 0; z < 64; ++z) o[z] = (uint16_t)(2 * ZZ[z]);
  }
};
__device__ const ZzOff kZzOff{};

}  // namespace
}  // namespace hic
