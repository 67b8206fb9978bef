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
// ROWS 1 ("direct" layout): M-tile mt's local row r is zig-zag slot 16 (r >> 2) +
// 4 mt + (r & 3), so output lane (n, g) ends with slots 16 g .. 16 g + 15 of its
// block over the four M-tiles: 32 contiguous bytes, stored straight from registers.
template <int ROWS>
struct MfmaFrag {
  uint32_t w[2][4][4][64][4];
  static constexpr int slot(int mt, int r) { return ROWS == 0 ? 16 * mt + r : 16 * (r >> 2) + 4 * mt + (r & 3); }
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
__device__ const MfmaFrag<0> kMfmaFragDev{};
__device__ const MfmaFrag<1> kMfmaFragDevD{};

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

// this lane's A operand digits for `table` (16 x 16 B, L2-resident); DIRECT: the
// direct layout's row order
template <bool DIRECT = false>
__device__ __forceinline__ void mfma_load_A(int table, int lane, i32x4 (&A)[4][4]) {
  const uint4 *f = reinterpret_cast<const uint4 *>(DIRECT ? &kMfmaFragDevD.w[table][0][0][0][0]
                                                          : &kMfmaFragDev.w[table][0][0][0][0]);
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
__device__ __forceinline__ bool mfma_pass(const i32x4 (&A)[4][4], const i32x4 (&B)[4], uint2 *st2, int lane,
                                          int table, uint64_t &m44) {
  const int n = lane & 15, g = lane >> 4;
  const i32x4 c0v = {kMfmaC0, kMfmaC0, kMfmaC0, kMfmaC0}, zero = {0, 0, 0, 0};
  const i32x4 halfv = {1 << 15, 1 << 15, 1 << 15, 1 << 15};
  const uint32_t dcmask = g == 0 ? 0x7FFFFu : 0u;
  const uint32_t z44mask = (g == 1 && table == 0) ? 0x7FFFFu : 0u;
  uint32_t fmin = 0xFFFFFFFFu;
  m44 = 0;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    uint2 *row = st2 + (16 * nt + n) * kStageU2 + g;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      // four independent digit products (no MFMA -> VALU -> MFMA chain); c0 and
      // the 1/2 ride in the accumulator inputs of digits 0 and 2
      const i32x4 S0 = mfma_i8(A[mt][0], B[nt], c0v);
      const i32x4 S1 = mfma_i8(A[mt][1], B[nt], zero);
      const i32x4 S2 = mfma_i8(A[mt][2], B[nt], halfv);
      const i32x4 S3 = mfma_i8(A[mt][3], B[nt], zero);
      // R = floor((S0 + c0 + 2^8 S1) / 2^13) + 2^3 (S2 + 2^15) + 2^11 S3
      const i32x4 R = (S3 << 11) + (S2 << 3) + (((S1 << 8) + S0) >> 13);
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
      row[4 * mt] = make_uint2(w01, __builtin_bit_cast(uint32_t, q23));
      // one (N-tile, M-tile) group at a time: four MFMAs in flight keep the live
      // accumulators at 16 VGPRs (the other waves of the SIMD cover the latency)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  return __builtin_amdgcn_ballot_w64(fmin < kMfmaL) != 0;
}


// The direct pass (row layout 1): lane (n, g) of N-tile nt computes slots 16 g ..
// 16 g + 15 of block 16 nt + n and stores them as two 16-byte stores at
// out + (16 nt + n) * 64 + 16 g (int16 units): no LDS stage.  The luminance (4,4)
// ties are decided per N-tile before its stores (the rows' signed sums go through
// k44, 4 int2 per block); every lane's 16-bit nonzero mask of its slots goes to
// nzm[block][g] for the set's tile record.  Returns true (wave-uniform) if any
// other coefficient is flagged: the caller redoes the set (which stores again).
// blk_ok: this lane's block exists (its stores are skipped otherwise).
// BUF: the stores go through the buffer resource `orsrc` (the plane's output, its
// size as the record count) at scalar offset `soff` (the set's first byte): always
// issued -- out-of-range lanes are dropped by the hardware -- so a set issues a
// fixed number of vector-memory instructions (the DMA kernel's vmcnt bookkeeping)
template <bool BUF = false>
__device__ __forceinline__ bool mfma_pass_direct(const i32x4 (&A)[4][4], const i32x4 (&B)[4], int16_t *out_set,
                                                 int lane, int table, int nvalid, int2 *k44, uint16_t *nzm,
                                                 __amdgpu_buffer_rsrc_t orsrc, uint32_t soff) {
  const int n = lane & 15, g = lane >> 4;
  const i32x4 c0v = {kMfmaC0, kMfmaC0, kMfmaC0, kMfmaC0}, zero = {0, 0, 0, 0};
  const i32x4 halfv = {1 << 15, 1 << 15, 1 << 15, 1 << 15};
  const uint32_t dcmask = g == 0 ? 0x7FFFFu : 0u;
  const bool luma = table == 0;
  const uint32_t z44mask = (g == 2 && luma) ? 0x7FFFFu : 0u;
  uint32_t fmin = 0xFFFFFFFFu;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    uint32_t wq[8];
    bool t44 = false;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const i32x4 S0 = mfma_i8(A[mt][0], B[nt], c0v);
      const i32x4 S1 = mfma_i8(A[mt][1], B[nt], zero);
      const i32x4 S2 = mfma_i8(A[mt][2], B[nt], halfv);
      const i32x4 S3 = mfma_i8(A[mt][3], B[nt], zero);
      const i32x4 R = (S3 << 11) + (S2 << 3) + (((S1 << 8) + S0) >> 13);
      uint32_t f0 = (uint32_t)R.x & 0x7FFFFu, f3 = (uint32_t)R.w & 0x7FFFFu;
      if (mt == 0) f0 |= dcmask;
      if (mt == 1) {
        t44 = luma && g == 2 && f3 < kMfmaL;
        f3 |= z44mask;
      }
      fmin = min(min(fmin, f0), (uint32_t)R.y & 0x7FFFFu);  // v_min3_u32
      fmin = min(min(fmin, (uint32_t)R.z & 0x7FFFFu), f3);
      s16x2 q01 = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((uint32_t)R.y, (uint32_t)R.x, 0x07060302u));
      s16x2 q23 = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm((uint32_t)R.w, (uint32_t)R.z, 0x07060302u));
      q01 = q01 >> (s16x2){3, 3};
      q23 = q23 >> (s16x2){3, 3};
      uint32_t w01 = __builtin_bit_cast(uint32_t, q01);
      if (mt == 0) {
        const int X = (R.x - (1 << 18)) >> 17;
        const int qdc = table == 0 ? dc_quant<0>(X) : dc_quant<1>(X);
        if (g == 0) w01 = (w01 & 0xFFFF0000u) | ((uint32_t)qdc & 0xFFFFu);
      }
      wq[2 * mt] = w01;
      wq[2 * mt + 1] = __builtin_bit_cast(uint32_t, q23);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (__builtin_amdgcn_ballot_w64(t44)) {
      // luminance (4,4) ties of this N-tile: the rows' signed sums of each block to its
      // lane (n, 2), pocketfft's own roundings, the exact q into slot 39 (high half
      // of wq[3])
      constexpr int kS = 0x01FFFF01;  // int8 (+1, -1, -1, +1)
      const int ka = __builtin_amdgcn_sdot4(B[nt].y, kS, __builtin_amdgcn_sdot4(B[nt].x, kS, 0, false), false);
      const int kb = __builtin_amdgcn_sdot4(B[nt].w, kS, __builtin_amdgcn_sdot4(B[nt].z, kS, 0, false), false);
      k44[n * 4 + g] = make_int2(ka, kb);
      __builtin_amdgcn_wave_barrier();
      if (t44) {
        int k[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int2 v = k44[n * 4 + r];
          k[2 * r] = v.x;
          k[2 * r + 1] = v.y;
        }
        const int q = quant_fast<0>(pf_y44_k(k), 36);
        wq[3] = (wq[3] & 0xFFFFu) | ((uint32_t)q << 16);
      }
      __builtin_amdgcn_wave_barrier();
    }
    // this lane's 16 slots: 32 contiguous bytes of block 16 nt + n
    if (BUF) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const uint32_t vo = (uint32_t)(((16 * nt + n) * 64 + 16 * g) * 2);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){wq[0], wq[1], wq[2], wq[3]}, orsrc, vo, soff, 2);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){wq[4], wq[5], wq[6], wq[7]}, orsrc, vo + 16, soff, 2);
    } else if (16 * nt + n < nvalid) {
      uint4 *o = reinterpret_cast<uint4 *>(out_set + (16 * nt + n) * 64 + 16 * g);
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store((u32x4){wq[0], wq[1], wq[2], wq[3]}, reinterpret_cast<u32x4 *>(o));
      __builtin_nontemporal_store((u32x4){wq[4], wq[5], wq[6], wq[7]}, reinterpret_cast<u32x4 *>(o + 1));
    }
    if (nzm) {
      // nonzero mask of slots 16 g .. 16 g + 15: v_pk_min_u16(w, 1) per pair, even
      // slots in bits 0..7, odd in 16..23, then interleaved
      uint32_t acc = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc |= pk_min_u16(wq[k], 0x00010001u) << k;
      nzm[(16 * nt + n) * 4 + g] = (uint16_t)zip16(acc & 0xFFu, acc >> 16);
    }
  }
  return __builtin_amdgcn_ballot_w64(fmin < kMfmaL) != 0;
}

}  // namespace
}  // namespace hic
