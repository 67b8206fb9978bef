// dct_mfma.h -- the integer-MFMA forward DCT + quantiser of 64-block passes,
// shared by the plane kernel (k_dct_mfma, dct.hip) and the fused 4:2:0 encoder
// (k_encode420, encode.hip).  The proof, the constant matrices and a bit-level
// emulation live in tools/check/dct_mfma.py (pinned by tests/test_dct_mfma.py);
// see dct.hip above k_dct_mfma for the arithmetic.
#pragma once
#include "dct_core.h"
#include "dct_mfma_tables.h"
#include "rle_core.h"

namespace hic {
namespace {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int16_t s16x2 __attribute__((ext_vector_type(2)));

constexpr int32_t mfma_digit(int32_t a, int d) {
  for (int k = 0; k < d; ++k) {
    const int32_t dk = ((a + 128) & 255) - 128;
    a = (a - dk) / 256;  // exact
  }
  return d < 3 ? ((a + 128) & 255) - 128 : a;
}

// A's digits in MFMA fragment order: w[t][mt][d][lane][c] = dword c of lane
// `lane`'s A operand for M-tile mt (slots 16 mt ..), digit d.  Byte j of lane
// (zl = lane & 15, g = lane >> 4) is digit d of A[t][16 mt + zl][16 g + j]: pixel
// 16 g + j = row 2 g + j / 8, column j % 8 -- the same (g, j) the B operand's
// pixel rows use.
struct MfmaFrag {
  uint32_t w[2][4][4][64][4];
  static constexpr int slot(int mt, int r) { return 16 * mt + r; }
  constexpr MfmaFrag() : w() {
    for (int t = 0; t < 2; ++t)
      for (int mt = 0; mt < 4; ++mt)
        for (int d = 0; d < 4; ++d)
          for (int l = 0; l < 64; ++l)
            for (int c = 0; c < 4; ++c) {
              uint32_t v = 0;
              for (int b = 0; b < 4; ++b) {
                const int32_t a = kMfmaA[t][slot(mt, l & 15)][16 * (l >> 4) + 4 * c + b];
                v |= (uint32_t)(uint8_t)(int8_t)mfma_digit(a, d) << (8 * b);
              }
              w[t][mt][d][l][c] = v;
            }
  }
};
__device__ const MfmaFrag kMfmaFragDev{};

__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// pocketfft's half-scaled y'[4][4] from the rows' signed sums k_r (pf_y44 with the
// integer prefix done): a luminance (4,4) tie is decided by these roundings
__device__ __forceinline__ double pf_y44_k(const int (&k)[8]) {
  double y[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) y[r] = (double)k[r] * TW3;
  const double c1 = y[1] + y[2], c3 = y[3] + y[4], c5 = y[5] + y[6], H0 = y[0] + y[7];
  const double h1 = c1 + c5, T2 = H0 + c3;
  return (T2 - h1) * TW3;
}

// this lane's A operand digits for `table` (16 x 16 B, L2-resident)
__device__ __forceinline__ void mfma_load_A(int table, int lane, i32x4 (&A)[4][4]) {
  const uint4 *f = reinterpret_cast<const uint4 *>(&kMfmaFragDev.w[table][0][0][0][0]);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint4 v = f[(mt * 4 + d) * 64 + lane];
      A[mt][d] = i32x4{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
    }
}

// A pixel fragment: rows 2g, 2g + 1 (8 bytes each) of a block, centred (p XOR 0x80
// is p - 128 as an int8)
__device__ __forceinline__ i32x4 mfma_pixels(uint2 r0, uint2 r1) {
  return i32x4{(int)(r0.x ^ 0x80808080u), (int)(r0.y ^ 0x80808080u), (int)(r1.x ^ 0x80808080u),
               (int)(r1.y ^ 0x80808080u)};
}

// One pass over 64 blocks: B[nt] holds (lane n = lane & 15, g = lane >> 4) rows 2g,
// 2g + 1 of block 16 nt + n; the quantised zig-zag coefficients of block b go to
// stage row b (kStageU2 uint2 per row).  Returns true (wave-uniform) if any
// coefficient but the DCs and the luminance (4,4) ties is flagged: the caller then
// redoes the pass on the float64 AAN path.  m44 (table 0): bit b = block b's (4,4)
// is a tie, its stage value provisional (the caller decides it: pf_y44).
// PIPE: the next group's four MFMAs are issued before this group's epilogue (32
// accumulator VGPRs instead of 16; the epilogue never waits on a just-issued MFMA)
template <bool PIPE = false>
__device__ __forceinline__ bool mfma_pass(const i32x4 (&A)[4][4], const i32x4 (&B)[4], uint2 *st2, int lane,
                                          int table, uint64_t &m44) {
  const int n = lane & 15, g = lane >> 4;
  const i32x4 c0v = {kMfmaC0, kMfmaC0, kMfmaC0, kMfmaC0}, zero = {0, 0, 0, 0};
  const i32x4 halfv = {1 << 15, 1 << 15, 1 << 15, 1 << 15};
  const uint32_t dcmask = g == 0 ? 0x7FFFFu : 0u;
  const uint32_t z44mask = (g == 1 && table == 0) ? 0x7FFFFu : 0u;
  uint32_t fmin = 0xFFFFFFFFu;
  m44 = 0;
  // group k = (N-tile k >> 2, M-tile k & 3): four independent digit products (no
  // MFMA -> VALU -> MFMA chain); c0 and the 1/2 ride in the accumulator inputs of
  // digits 0 and 2
  i32x4 S[PIPE ? 2 : 1][4];
  auto issue = [&](int k, i32x4 (&s)[4]) {
    const int nt = k >> 2, mt = k & 3;
    s[0] = mfma_i8(A[mt][0], B[nt], c0v);
    s[1] = mfma_i8(A[mt][1], B[nt], zero);
    s[2] = mfma_i8(A[mt][2], B[nt], halfv);
    s[3] = mfma_i8(A[mt][3], B[nt], zero);
  };
  if (PIPE) issue(0, S[0]);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int nt = k >> 2, mt = k & 3;
    i32x4 (&s)[4] = S[PIPE ? (k & 1) : 0];
    if (PIPE) {
      if (k + 1 < 16) issue(k + 1, S[PIPE ? ((k + 1) & 1) : 0]);
    } else {
      issue(k, s);
    }
    // R = floor((S0 + c0 + 2^8 S1) / 2^13) + 2^3 (S2 + 2^15) + 2^11 S3
    const i32x4 R = (s[3] << 11) + (s[2] << 3) + (((s[1] << 8) + s[0]) >> 13);
    uint32_t f0 = (uint32_t)R.x & 0x7FFFFu, f3 = (uint32_t)R.w & 0x7FFFFu;
    if (mt == 0) f0 |= dcmask;
    if (mt == 2) {
      if (table == 0) {
        const uint64_t b = __builtin_amdgcn_ballot_w64(g == 1 && f3 < kMfmaL);
        m44 |= ((b >> 16) & 0xFFFFull) << (16 * nt);
      }
      f3 |= z44mask;
    }
    fmin = min(min(fmin, f0), (uint32_t)R.y & 0x7FFFFu);  // v_min3_u32
    fmin = min(min(fmin, (uint32_t)R.z & 0x7FFFFu), f3);
    // q = R >> 19 as int16 pairs: the high halves, then >> 3 per half
    s16x2 q01 = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((uint32_t)R.y, (uint32_t)R.x, 0x07060302u));
    s16x2 q23 = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((uint32_t)R.w, (uint32_t)R.z, 0x07060302u));
    q01 = q01 >> (s16x2){3, 3};
    q23 = q23 >> (s16x2){3, 3};
    uint32_t w01 = __builtin_bit_cast(uint32_t, q01);
    if (mt == 0) {
      // DC: the exact pixel sum X = (R - 2^18) >> 17, rounded as numpy does
      const int X = (R.x - (1 << 18)) >> 17;
      const int qdc = table == 0 ? dc_quant<0>(X) : dc_quant<1>(X);
      if (g == 0) w01 = (w01 & 0xFFFF0000u) | ((uint32_t)qdc & 0xFFFFu);
    }
    st2[(16 * nt + n) * kStageU2 + g + 4 * mt] = make_uint2(w01, __builtin_bit_cast(uint32_t, q23));
    // one group (two with PIPE) in flight keeps the live accumulators at 16 (32)
    // VGPRs (the other waves of the SIMD cover the latency)
    __builtin_amdgcn_sched_barrier(0);
  }
  return __builtin_amdgcn_ballot_w64(fmin < kMfmaL) != 0;
}


}  // namespace
}  // namespace hic
