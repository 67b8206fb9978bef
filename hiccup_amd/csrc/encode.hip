// encode.hip -- the fused 4:2:0 encoder front end for MI355X (gfx950): one pass
// over the RGB image computes cvtColor(RGB2YCrCb), pyrDown of Cr / Cb, the 8x8
// DCT + quantize + transposed zig-zag of all three planes and the planes' RLE
// tile records.  The Y / Cr / Cb planes never exist in HBM.
//
// Reference: compression.jpeg_compression (compression.py:16-39) = cv2.cvtColor
// (:21) + transform.down_sample (pyrDown, transform.py:151-157) + dct_channel x3
// (transform.py:182-193), and the zig-zag / tile pass of codec.jpeg_encode
// (codec.py:286-301, transform.py:106-148).  Bit-exact with the unfused chain
// (color.hip + dct.hip): the same colour arithmetic (color_core.h, OpenCV 8U
// restatement, PARITY UNPINNED), the same float64 AAN DCT with exact tie
// handling (dct_core.h), the same tile records (rle_core.h).
//
// Work unit: a "strip" of 512 pixel columns x 16 image rows.  Lane l owns pixel
// columns [8 l, 8 l + 8) of the strip, i.e. Y block column l of the strip's two
// block rows (a 64-block RLE tile each when W % 512 == 0) and half of chroma block
// column l / 2.  Any W % 16 == 0: the last strip is ragged (W mod 512 columns;
// its lanes past W compute on whatever the loads return and store nothing, the
// right-border pixel goes to its last lane); its block rows then straddle RLE
// tiles, so the tile records come from a tile pass after the launch.  One wave
// per unit:
//   1. colour: 19 RGB rows (the 16 rows + the 2 + 1 rows of pyrDown's vertical
//      taps), 24 B per lane per row (1.5 KiB contiguous per wave-row, buffer loads
//      at a scalar row offset); YCC by v_dot4 (ycc8); Y of rows 0..15 stays in
//      registers (two 8x8 blocks per lane); Cr / Cb per pixel, the horizontal
//      [1 4 6 4 1] at even columns with the neighbour pixels by DPP wave shifts
//      (the strip's edge pixels converted once per unit, one row per lane, and
//      written into lane 0 / 63 by v_writelane), the vertical taps over a 5-row
//      window -> 8 chroma rows x 4 columns per lane and plane;
//   2. DCT of Y block row 0 and row 1 (lane = block; after all 19 colour rows):
//      coefficients to the LDS stage at their zig-zag slot, copied out in 1 KiB
//      stores, the tile record from the stage;
//   3. chroma: the colour stage left the chroma rows in a 4 KiB LDS area per wave;
//      chroma block m of Cr is read into lane m and of Cb into lane 32 + m (a
//      block spans the columns of lanes 2m, 2m + 1), one DCT pass with the
//      chrominance table, 4 KiB of Cr and 4 KiB of Cb blocks out, and two 32-block
//      half-tile records (hic_rle_job16.records_per_tile = 2).
// Exact-tie fallbacks (dct_block_2ph, dct_fix26) run in place on the pixels still
// in registers: a unit never revisits HBM.
// RGB traffic: 19/16 of the image fetched by the waves (the vertical halo rows are
// re-read by the unit above / below), of which the default unit order (knob
// encode_order 6: XCD-major workgroups, odd unit rows bottom-up) has the L2 serve
// most re-reads: 109.6 MB from HBM per 8K launch against the image's 99.5 MB;
// coefficient writes 3 B per pixel.
#include "color_core.h"
#include "dct_core.h"
#include "rle_core.h"
#include "slots.h"

namespace hic {
namespace {

struct Enc420 {
  const uint8_t *rgb;  // image rows [in_row0, in_row0 + in_rows), W * 3 bytes each
  int in_row0, in_rows, H, W, out_row0, out_rows;
  int16_t *coef[3];  // ZIGZAG_I16 blocks of the shard's Y, Cr, Cb planes
  int64_t *rec[3];   // tile records: Y per 64-block tile, Cr / Cb per 32-block half tile
  int M;
  int nstrips, nunits;  // nunits: waves (one unit each)
  int xcd;              // 1: workgroups remapped XCD-major (xcd_block)
  int alt;              // 1: odd unit rows run their colour rows bottom-up
  int wlast;            // pixel columns of the last strip (16 .. 512)
  // slot layout (k_encode420<15, true>, hic_encode420_slots_u8; slots.h): per plane
  // the symbol slots, the DC differences and the records' last DCs; coef unused
  uint8_t *slen[3];
  int16_t *sval[3];
  int32_t *dc[3];
  int32_t *rdc[3];
  const int32_t *nsym[3];  // hic_probe_encode420_slots: the record index (n_r) it replays
};

constexpr int kZZ = HIC_LAYOUT_ZIGZAG_I16;

// Workgroup b of n, as dispatched round-robin over the 8 XCDs (b % 8), -> the logical
// block that puts consecutive logical blocks on one XCD (its own L2): XCD x takes
// blocks x * q + min(x, r) .. (q = n / 8, r = n % 8), so the pixel rows and strip-edge
// lines neighbouring units share are fetched once into that L2.
__device__ __forceinline__ int xcd_block(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7, i = b >> 3;
  return x * q + (x < r ? x : r) + i;
}

// Exact fallbacks, out of line (cold; by-value pixel rows keep them in VGPRs).
template <int TABLE>
__device__ __attribute__((noinline)) void enc_exact_block(uint2 w0, uint2 w1, uint2 w2, uint2 w3, uint2 w4, uint2 w5,
                                                          uint2 w6, uint2 w7, int16_t *st) {
  uint2 w[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  dct_block_2ph<TABLE, kZZ>(w, st);
}
template <int TABLE>
__device__ __attribute__((noinline)) void enc_fix26_block(uint2 w0, uint2 w1, uint2 w2, uint2 w3, uint2 w4, uint2 w5,
                                                          uint2 w6, uint2 w7, int16_t *st) {
  const uint2 w[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  int q[4];
  dct_fix26<TABLE>(w, q);
  constexpr SlotOf<kZZ> kSlot{};
  st[kSlot.s[18]] = (int16_t)q[0];
  st[kSlot.s[22]] = (int16_t)q[1];
  st[kSlot.s[50]] = (int16_t)q[2];
  st[kSlot.s[54]] = (int16_t)q[3];
}

// One block per lane -> quantized zig-zag coefficients in this lane's stage row,
// exact in every case (fast AAN path; the rare tie sets fall back in place).
template <int TABLE>
__device__ __forceinline__ void enc_dct(uint2 (&w)[8], int16_t *st) {
  bool t26 = false;
  const bool f = dct_block_aan<TABLE, kZZ>(w, st, &t26);
  if (__builtin_amdgcn_ballot_w64(f)) {
    enc_exact_block<TABLE>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], st);
  } else if (__builtin_amdgcn_ballot_w64(t26)) {
    enc_fix26_block<TABLE>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], st);
  }
}

#ifndef HIC_ENC_WPB
#define HIC_ENC_WPB 4  // waves per workgroup
#endif
#ifndef HIC_ENC_LA3
#define HIC_ENC_LA3 3  // colour rows' load lookahead
#endif

// 16 B chunk k of stage row b
__device__ __forceinline__ uint4 enc_st16(const uint2 *st2, int b, int k) {
  const uint2 lo = st2[b * kStageU2 + 2 * k], hi = st2[b * kStageU2 + 2 * k + 1];
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// stage rows 0..31 -> o_lo (32 blocks), rows 32..63 -> o_hi: 1 KiB per store
// instruction, nontemporal (the coefficients are not re-read by this kernel; with 3
// waves per SIMD and 4 images in flight nontemporal stores won against cached ones
// in 3 of 3 alternating pairs, 0.0999-0.1033 vs 0.1041-0.1051 ms/step,
// profiles/r03/s2/nt/).  n_lo / n_hi (wave-uniform): blocks of o_lo / o_hi that
// exist (32 but in a ragged strip)
__device__ __forceinline__ void enc_store(const uint2 *st2, int lane, int16_t *o_lo, int16_t *o_hi, int n_lo = 32,
                                          int n_hi = 32) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const bool full = (n_lo & n_hi) == 32;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 t = enc_st16(st2, 8 * k + (lane >> 3), lane & 7);
    const u32x4 v = {t.x, t.y, t.z, t.w};
    u32x4 *o = reinterpret_cast<u32x4 *>(k < 4 ? o_lo : o_hi) + 64 * (k & 3) + lane;
    if (!full && 8 * (k & 3) + (lane >> 3) >= (k < 4 ? n_lo : n_hi)) continue;
    __builtin_nontemporal_store(v, o);
  }
}

__device__ __forceinline__ void enc_stage_row(const uint2 *st2, int lane, uint32_t (&zw)[32]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 t = enc_st16(st2, lane, k);
    zw[4 * k] = t.x; zw[4 * k + 1] = t.y; zw[4 * k + 2] = t.z; zw[4 * k + 3] = t.w;
  }
}

// Packed 16-bit helpers: both chroma planes in one dword (Cr low half, Cb high
// half); pyrDown's sums stay below 2^16 (horizontal <= 16 * 255, vertical + 128 <=
// 65408), so v_pk_*_u16 does both planes at once.  The multipliers arrive as
// opaque registers (opq): a literal 4 is strength-reduced to a shift + an add.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_mad16(uint32_t a, uint32_t k, uint32_t c) {  // a * k + c per half
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, k) +
                                          __builtin_bit_cast(u16x2, c));
}
__device__ __forceinline__ uint32_t opq(uint32_t k) {
  asm volatile("" : "+s"(k));
  return k;
}
// [1 4 6 4 1] over five packed taps (k4 = 4 | 4 << 16, k6 = 6 | 6 << 16)
__device__ __forceinline__ uint32_t pk_taps5(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e, uint32_t k4,
                                             uint32_t k6) {
  return pk_mad16(c, k6, pk_mad16(pk_add16(b, d), k4, pk_add16(a, e)));
}

// cvtColor RGB2YCrCb of the 8 pixels in 24 RGB bytes wd[0..5]: color_core.h's
// rgb2ycc restated for the dot-product unit (equal on all 2^24 inputs,
// tools/check/colour_dot4.py):
//   4 (4899 r + 9617 g + 1868 b) + 2^15 = 256 (rgb . HI) + (rgb . LO) + 2^15, HI / LO
//   the high / low bytes of the 4x coefficients: two v_dot4_u32_u8, the second
//   accumulating the first >> 8, leave y = descale14(4899 r + ...) in byte 1 (Yh);
//   Cr = sat8(descale14((r - y) 11682 + 2^21)) is byte 2 of
//   clamp((r - y) 46728 + 4 (2^21 + 2^13), 0, 2^24 - 1), likewise Cb, and one
//   v_perm packs Cr | Cb << 16 (c).
// Pixel k's bytes start at 3k: pixels 0, 4 (byte 0 of a dword) and 3, 7 (byte 1)
// are read in place, pixels 1, 2, 5, 6 through v_alignbyte.
constexpr uint32_t kYLo = 140u | 68u << 8 | 48u << 16, kYHi = 76u | 150u << 8 | 29u << 16;
constexpr int kCr4 = 4 * kYCRI, kCb4 = 4 * kYCBI, kCC4 = 4 * ((128 << 14) + (1 << 13));
struct YccK {  // dot4 weights in SGPRs (VOP3P takes no literals), addends in VGPRs
  uint32_t lo0, lo1, hi0, hi1, acc, cc4;
};
// Stage by stage over the 8 pixels (a v_dot4 result read by the next instruction
// costs wait states: independent pixels fill them)
__device__ __forceinline__ void ycc8(const uint32_t (&wd)[6], const YccK &K, uint32_t (&Yh)[8], uint32_t (&c)[8]) {
  uint32_t x[8], L[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int q = k & 3, d0 = (k >> 2) * 3;
    x[k] = q == 0 ? wd[d0]
           : q == 1 ? __builtin_amdgcn_alignbyte(wd[d0 + 1], wd[d0], 3)
           : q == 2 ? __builtin_amdgcn_alignbyte(wd[d0 + 2], wd[d0 + 1], 2)
                    : wd[d0 + 2];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) L[k] = __builtin_amdgcn_udot4(x[k], (k & 3) == 3 ? K.lo1 : K.lo0, K.acc, false);
#pragma unroll
  for (int k = 0; k < 8; ++k) Yh[k] = __builtin_amdgcn_udot4(x[k], (k & 3) == 3 ? K.hi1 : K.hi0, L[k] >> 8, false);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int sh = (k & 3) == 3 ? 8 : 0;
    const int y = (int)((Yh[k] >> 8) & 255u);
    const int r = (int)((x[k] >> sh) & 255u), b = (int)((x[k] >> (sh + 16)) & 255u);
    // opaque addend: a literal one is split off into a v_add after the clamp
    int vr = (r - y) * kCr4 + (int)K.cc4, vb = (b - y) * kCb4 + (int)K.cc4;
    vr = vr < 0 ? 0 : (vr > 0xFFFFFF ? 0xFFFFFF : vr);
    vb = vb < 0 ? 0 : (vb > 0xFFFFFF ? 0xFFFFFF : vb);
    c[k] = __builtin_amdgcn_perm((uint32_t)vb, (uint32_t)vr, 0x07060302u);
  }
}
// bytes 1 of Yh[k0 .. k0 + 3] -> one dword of four Y bytes
__device__ __forceinline__ uint32_t ypack4(const uint32_t (&Yh)[8], int k0) {
  const uint32_t lo = __builtin_amdgcn_perm(Yh[k0 + 1], Yh[k0], 0x0C0C0501u);
  const uint32_t hi = __builtin_amdgcn_perm(Yh[k0 + 3], Yh[k0 + 2], 0x0C0C0501u);
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// The lane index made afresh (v_mbcnt), opaque to CSE: the 3-wave kernel would
// otherwise keep lane-derived values live from the colour stage into the DCT passes
// and spill them
__device__ __forceinline__ int fresh_lane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ uint32_t opv(uint32_t k) {  // a constant held in a VGPR
  asm volatile("" : "+v"(k));
  return k;
}
// v's value in lane L replaced by s (v_writelane_b32: no builtin in this compiler)
template <int L>
__device__ __forceinline__ uint32_t set_lane(uint32_t v, int s) {
  asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s), "n"(L));
  return v;
}
// the same with a wave-uniform lane index (writelane cannot take the value and the
// lane from two SGPRs: one constant-bus read per instruction)
__device__ __forceinline__ uint32_t set_lane_s(uint32_t v, int s, int lane, int l) {
  return lane == l ? (uint32_t)s : v;
}
// wave shifts for the horizontal taps (the edge lane is overwritten by v_writelane)
__device__ __forceinline__ uint32_t wshr1(uint32_t v) {  // lane i <- lane i - 1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wshl1(uint32_t v) {  // lane i <- lane i + 1
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);
}

// Colour stage of one unit (image rows y0 .. y0 + 15 of strip s), run in two row
// ranges around the DCT of Y block row 0 (rows() below): Y rows -> yq, pyrDown'd
// chroma rows (4 columns per lane, packed bytes) -> the wave's LDS chroma area
// s_chroma[plane][row][lane] (so chroma block m's row i is the 8 bytes at
// s_chroma[plane][i][2m]).  Input row r (image row y0 + r - 2) arrives by a buffer
// load whose row offset is a scalar (no per-row address arithmetic on the vector
// unit); the strip-edge pixels (the neighbour strips', or reflect-101's at the
// image border) are converted once up front and written into lane 0 / 63 by
// v_writelane.
#ifndef HIC_ENC_LA
#define HIC_ENC_LA 6
#endif
// NR input rows: 19 for one 16-row unit, 35 for two vertically adjacent units
// (VG = 2: the second unit reuses the first's bottom halo rows).
template <int NR, int LA = HIC_ENC_LA, bool PIN_Y = false>
struct EncColour {
  static_assert(NR % 2 == 1, "the bottom-up chroma rows assume an odd row count");
  // rows stream through a ring of kLA + 1 loads in flight (sched_barrier keeps the
  // compiler from hoisting all 19 rows' loads: 114 VGPRs)
  static constexpr int kLA = LA;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  int lane, roff, voff, rlane;  // rlane: the strip's last lane (63 but in a ragged strip)
  uint32_t hal_l2, hal_l1, hal_r;
  __amdgpu_buffer_rsrc_t rsrc;
  YccK K;
  uint32_t k4, k6, k128;
  u32x4 ring_a[kLA + 1];
  u32x2 ring_b[kLA + 1];
  uint32_t h[NR][4];  // horizontal pyrDown sums of input row r, chroma column j (packed)

#ifndef HIC_ENC_LOAD_AUX
#define HIC_ENC_LOAD_AUX 0
#endif
  // input row r into ring slot t % (kLA + 1) (t: the row's turn)
  __device__ __forceinline__ void load_row_at(int r, int t) {
    const int so = __builtin_amdgcn_readlane(roff, r);
    ring_a[t % (kLA + 1)] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, so, HIC_ENC_LOAD_AUX);
    ring_b[t % (kLA + 1)] = __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff + 16, so, HIC_ENC_LOAD_AUX);
  }

  __device__ __forceinline__ void init(const Enc420 &E, int y0, int s, int lane_, int nb, bool rev = false) {
    lane = lane_;
    rlane = __builtin_amdgcn_readfirstlane(nb - 1);
    const int W = E.W, H = E.H, pitch = 3 * W;
    const int in_row1 = E.in_row0 + E.in_rows;
    const int xs = 512 * s;
    // byte offset of input row rr (image row y0 + rr - 2, rr = 0 .. NR - 1) in the
    // input rows, computed by lane rr (read back per row by v_readlane): one
    // reflect-101 step suffices for every row a unit uses (its last row <= H, H >=
    // 16), then the shard's clamp (which also keeps the rows of a missing second
    // unit, loaded ahead but never used, inside the buffer)
    {
      int sy = y0 + lane - 2;
      sy = sy < 0 ? -sy : (sy >= H ? 2 * H - 2 - sy : sy);
      sy = sy < E.in_row0 ? E.in_row0 : (sy >= in_row1 ? in_row1 - 1 : sy);
      roff = (sy - E.in_row0) * pitch;
    }
    // edge pixels, packed (cr | cb << 16): lane r converts input row r's x = xs - 2,
    // xs - 1 (or 2, 1 at the left border) and x = xs + 512 (or W - 2 at the right,
    // also for a ragged last strip)
    hal_l2 = hal_l1 = hal_r = 0;
    if (lane < NR) {
      const uint8_t *row = E.rgb + roff;
      const int xl = xs >= 2 ? xs - 2 : 2, xl1 = xs >= 2 ? xs - 1 : 1, xr = xs + 512 < W ? xs + 512 : W - 2;
      const YCC a = rgb2ycc(row[3 * xl], row[3 * xl + 1], row[3 * xl + 2]);
      const YCC b = rgb2ycc(row[3 * xl1], row[3 * xl1 + 1], row[3 * xl1 + 2]);
      const YCC c = rgb2ycc(row[3 * xr], row[3 * xr + 1], row[3 * xr + 2]);
      hal_l2 = a.cr | a.cb << 16;
      hal_l1 = b.cr | b.cb << 16;
      hal_r = c.cr | c.cb << 16;
    }
    const uint64_t base = reinterpret_cast<uint64_t>(E.rgb) + 3 * xs;
    const uint32_t base_lo = __builtin_amdgcn_readfirstlane((uint32_t)base),
                   base_hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>((uint64_t)base_hi << 32 | base_lo), 0,
                                             __builtin_amdgcn_readfirstlane(E.in_rows * pitch - 3 * xs), 0x00020000);
    voff = 24 * lane;
    K = YccK{opq(kYLo), opq(kYLo << 8), opq(kYHi), opq(kYHi << 8), opv(32768u), opv((uint32_t)kCC4)};
    k4 = opq(0x00040004u);
    k6 = opq(0x00060006u);
    k128 = opq(0x00800080u);
    // rev: the rows run bottom-up (rows_rev)
#pragma unroll
    for (int t = 0; t < kLA; ++t) load_row_at(rev ? NR - 1 - t : t, t);
  }

  // all NR input rows, top-down, or bottom-up (rev, wave-uniform; init(.., rev)): a
  // unit row's bottom halo rows are then fetched while the unit row below, running
  // the other way, fetches them as its top rows (not ~20 us apart, after the L2 has
  // turned over).  One code path: row t of the pass is input row r = t or NR - 1 - t,
  // and as the pyrDown filter is symmetric only the Y slot and the chroma row a turn
  // fills depend on the direction.
  __device__ __forceinline__ void rows(uint2 (&yq)[16], uint32_t *s_chroma, bool rev) {
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      const int r = rev ? NR - 1 - t : t;  // wave-uniform
      if (t + kLA < NR) load_row_at(rev ? NR - 1 - (t + kLA) : t + kLA, t + kLA);
      const u32x4 qa = ring_a[t % (kLA + 1)];
      const u32x2 qb = ring_b[t % (kLA + 1)];
      const uint32_t wd[6] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y};
      uint32_t Yh[8], c[8];
      ycc8(wd, K, Yh, c);
      // Y rows of the unit: input rows 2 .. NR - 2, slot r - 2 (top-down: turns
      // 2 .. NR - 2, slot t - 2; bottom-up: turns 1 .. NR - 3, slot NR - 3 - t)
      const uint2 yv = make_uint2(ypack4(Yh, 0), ypack4(Yh, 4));
      if (t >= 2 && t <= NR - 2) {
        uint2 &q = yq[(t - 2) & 15];
        q = rev ? q : yv;
        // PIN_Y: pack now (the compiler otherwise sinks the packing v_perms to the
        // DCT and keeps the row's eight Yh dwords live, spilling them at 168 VGPRs)
        if constexpr (PIN_Y) asm volatile("" : "+v"(q.x), "+v"(q.y));
      }
      if (t >= 1 && t <= NR - 3) {
        uint2 &q = yq[(NR - 3 - t) & 15];
        q = rev ? yv : q;
        if constexpr (PIN_Y) asm volatile("" : "+v"(q.x), "+v"(q.y));
      }
      // neighbour pixels x0 - 2, x0 - 1 (left lane) and x0 + 8 (right lane)
      const uint32_t l2 = set_lane<0>(wshr1(c[6]), __builtin_amdgcn_readlane((int)hal_l2, r));
      const uint32_t l1 = set_lane<0>(wshr1(c[7]), __builtin_amdgcn_readlane((int)hal_l1, r));
      const uint32_t r0 = set_lane_s(wshl1(c[0]), __builtin_amdgcn_readlane((int)hal_r, r), lane, rlane);
      h[t][0] = pk_taps5(l2, l1, c[0], c[1], c[2], k4, k6);
      h[t][1] = pk_taps5(c[0], c[1], c[2], c[3], c[4], k4, k6);
      h[t][2] = pk_taps5(c[2], c[3], c[4], c[5], c[6], k4, k6);
      h[t][3] = pk_taps5(c[4], c[5], c[6], c[7], r0, k4, k6);
      // chroma row i has all five input rows 2 i .. 2 i + 4: the turns t - 4 .. t
      // (t even; i = t / 2 - 2, or bottom-up (NR - 1 - t) / 2)
      if (t >= 4 && t % 2 == 0) {
        const int a = t - 4, i = rev ? (NR - 1 - t) / 2 : t / 2 - 2;  // NR odd
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)  // sum + 128 < 2^16: (sum + 128) >> 8 is the high byte
          v[j] = pk_add16(pk_taps5(h[a][j], h[a + 1][j], h[a + 2][j], h[a + 3][j], h[a + 4][j], k4, k6), k128);
        // high bytes: x01 = (cr0, cr1, cb0, cb1), x23 = (cr2, cr3, cb2, cb3)
        const uint32_t x01 = __builtin_amdgcn_perm(v[1], v[0], 0x07030501u);
        const uint32_t x23 = __builtin_amdgcn_perm(v[3], v[2], 0x07030501u);
        s_chroma[(i & 7) * 64 + lane] = __builtin_amdgcn_perm(x23, x01, 0x05040100u);
        s_chroma[512 + (i & 7) * 64 + lane] = __builtin_amdgcn_perm(x23, x01, 0x07060302u);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // hic_probe_encode420: the same NR row loads in the same order, no arithmetic --
  // each row's words (and the edge pixels) folded into the Y slots so the probe's
  // stores carry what its loads fetched
  __device__ __forceinline__ void fold_rows(uint2 (&yq)[16], bool rev) {
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      if (t + kLA < NR) load_row_at(rev ? NR - 1 - (t + kLA) : t + kLA, t + kLA);
      const u32x4 qa = ring_a[t % (kLA + 1)];
      const u32x2 qb = ring_b[t % (kLA + 1)];
      yq[t & 15].x ^= qa.x ^ qa.z ^ qb.x;
      yq[t & 15].y ^= qa.y ^ qa.w ^ qb.y;
    }
    yq[0].x ^= hal_l2 ^ hal_l1 ^ hal_r;
  }
};

// One wave per unit, 3 waves per SIMD (<= 168 VGPRs): all 19 colour rows first, so
// no DCT runs while the row ring and the pyrDown window are live (the other waves of
// the SIMD hide the loads instead); each packed Y row is pinned where it is made;
// the DCT passes take the lane index afresh.  Round 3 measured this against the
// 2-wave budget (colour rows 0..9, Y block row 0, rows 10..18): 8K bench
// 0.1017-0.1041 vs 0.1043-0.1063 ms/step in 5 alternating pairs
// (profiles/r03/s2/enc_w3/).  Measured slower and removed (git history): the 2-wave
// kernel, the float32 / packed-float32 / integer-MFMA transforms (the packed one
// again in round 5, with proven windows and a cooperative float64 redo: 70.5-74.9
// vs 55.6-57.7 us, commit ae5c500), cached stores, the one-pass (look-back +
// emission) variant and vertically stacked units.
//
// SLOTS (TMF 15, whole images with W % 512 == 0; hic_encode420_slots_u8): each pass
// emits its record's AC symbols and DC differences into the slot layout (slots.h)
// instead of storing the int16 coefficients: no coefficient ever reaches HBM.
// One unit (wave g of the launch's E): the kernels below map their waves to units.
template <int TMF, bool SLOTS>
__device__ __forceinline__ void encode_unit(const Enc420 &E, int g, int lane, uint2 *st2, uint32_t *s_chroma) {
  static_assert(!SLOTS || TMF == kSlotM, "the slot layout packs 4-bit lengths (max_len 15)");
  int16_t *st = reinterpret_cast<int16_t *>(st2 + lane * kStageU2);
  const int u0 = __builtin_amdgcn_readfirstlane(g / E.nstrips);
  const int s = __builtin_amdgcn_readfirstlane(g - u0 * E.nstrips);
  const int y0 = E.out_row0 + 16 * u0;
  // Y blocks of this strip's block rows (64 but in a ragged last strip)
  const int nb = __builtin_amdgcn_readfirstlane(s == E.nstrips - 1 ? E.wlast >> 3 : 64);
  const int nbx = E.W >> 3, nbxc = E.W >> 4;

  uint2 yq[16];
  // Y block row br: blocks 64 s .. 64 s + 63 of block row 2 u0 + br (one RLE tile),
  // from yq slots 8 br .. 8 br + 7
  auto y_blocks = [&](int br) {
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = yq[8 * br + r];
    enc_dct<0>(w, st);
    const int64_t b0 = (int64_t)(2 * u0 + br) * nbx + 64 * s;
    __builtin_amdgcn_wave_barrier();
    if constexpr (SLOTS) {
      uint32_t zw[32];
      enc_stage_row(st2, fresh_lane(), zw);
      const int64_t r = b0 >> 6;  // W % 512 == 0: block row segments are whole tiles
      const SlotRec A{E.slen[0] + r * kSlotY, E.sval[0] + r * kSlotY, E.dc[0] + b0, E.rec[0] + r * 3, E.rdc[0] + r,
                      b0 * 63};
      slot_pass<false, true>(zw, st2, lane, A, A);
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
    int16_t *o = E.coef[0] + b0 * 64;
    enc_store(st2, fresh_lane(), o, o + 32 * 64, nb < 32 ? nb : 32, nb > 32 ? nb - 32 : 0);
    if (TMF >= 0 && E.rec[0]) {
      uint32_t zw[32];
      enc_stage_row(st2, fresh_lane(), zw);
      // one record per strip segment of the block row (64 blocks, or the ragged last
      // strip's nb): record (2 u0 + br) * nstrips + s (= b0 / 64 when W % 512 == 0)
      tile_record16<TMF>(zw, lane < nb, b0 + lane, E.M, E.rec[0] + ((2 * u0 + br) * E.nstrips + s) * 3);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // chroma: block m of Cr -> stage row m, of Cb -> row 32 + m (block m spans the
  // chroma columns of lanes 2m and 2m + 1 of this strip; its row i is the 8 bytes
  // at uint2 i * 32 + m of the plane's LDS area), one block per lane (Cr block m in
  // lane m, Cb in lane 32 + m)
  auto c_blocks = [&]() {
    __builtin_amdgcn_wave_barrier();
    const uint2 *sc = reinterpret_cast<const uint2 *>(s_chroma + (lane >> 5) * 512) + (lane & 31);
    uint2 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = sc[i * 32];
    enc_dct<1>(w, st);
    const int64_t b0 = (int64_t)u0 * nbxc + 32 * s;
    __builtin_amdgcn_wave_barrier();
    if constexpr (SLOTS) {
      uint32_t zw[32];
      enc_stage_row(st2, fresh_lane(), zw);
      const int64_t r = b0 >> 5;  // one record per 32-block half tile
      const SlotRec A{E.slen[1] + r * kSlotC, E.sval[1] + r * kSlotC, E.dc[1] + b0, E.rec[1] + r * 3, E.rdc[1] + r,
                      b0 * 63};
      const SlotRec B{E.slen[2] + r * kSlotC, E.sval[2] + r * kSlotC, E.dc[2] + b0, E.rec[2] + r * 3, E.rdc[2] + r,
                      b0 * 63};
      slot_pass<true, false>(zw, st2, lane, A, B);
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
    enc_store(st2, fresh_lane(), E.coef[1] + b0 * 64, E.coef[2] + b0 * 64, nb >> 1, nb >> 1);
    if (TMF >= 0 && E.rec[1]) {
      uint32_t zw[32];
      enc_stage_row(st2, fresh_lane(), zw);
      const int64_t rc = (int64_t)u0 * E.nstrips + s;  // = b0 / 32 when W % 512 == 0
      tile_record16_half<TMF>(zw, b0, E.M, E.rec[1] + rc * 3, E.rec[2] + rc * 3, nb >> 1);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  EncColour<19, HIC_ENC_LA3, true> C;
  const bool rev = E.alt && (u0 & 1);  // wave-uniform
  // the colour stage (its row loads) at issue priority 1 over the SIMD's waves in
  // their DCT / emission passes: kernel 72.6-73.4 vs 73.6-74.3 us, step 0.0728-0.0740
  // vs 0.0742-0.0760 ms in 5 alternating rounds (priority 2 / 3 within that range;
  // profiles/r06/enc_prio/)
  __builtin_amdgcn_s_setprio(1);
  C.init(E, y0, s, lane, nb, rev);
  C.rows(yq, s_chroma, rev);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
  y_blocks(0);
  y_blocks(1);
  c_blocks();
}

template <int TMF, bool SLOTS = false>
__global__ __launch_bounds__(64 * HIC_ENC_WPB) __attribute__((amdgpu_waves_per_eu(3))) void k_encode420(Enc420 E) {
  __shared__ __attribute__((aligned(16))) uint2 s_stage[HIC_ENC_WPB * 64 * kStageU2];
  __shared__ uint32_t s_chroma_all[HIC_ENC_WPB][2 * 8 * 64];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bx = __builtin_amdgcn_readfirstlane(E.xcd ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x);
  // wave g: strip s of unit row u0
  const int g = __builtin_amdgcn_readfirstlane(bx * HIC_ENC_WPB + wv);
  if (g >= E.nunits) return;  // wave-uniform
  encode_unit<TMF, SLOTS>(E, g, lane, s_stage + wv * 64 * kStageU2, s_chroma_all[wv]);
}

// Several encodes in ONE launch (hic_encode420_batch_u8: the row shards of a
// multi-GPU group, one per image): job j owns waves [unit0[j], unit0[j + 1]).  A
// shard is 1/N of an image -- 506 waves at N = 8, a sixth of the chip's 3072 wave
// slots -- so N launches in a row ran ~2.4x the time of one whole-image launch.
constexpr int kEncBatchMax = 8;
struct Enc420Batch {
  Enc420 e[kEncBatchMax];
  int unit0[kEncBatchMax + 1];
  int n, xcd;
};

template <int TMF>
__global__ __launch_bounds__(64 * HIC_ENC_WPB) __attribute__((amdgpu_waves_per_eu(3))) void k_encode420_batch(
    Enc420Batch B) {
  __shared__ __attribute__((aligned(16))) uint2 s_stage[HIC_ENC_WPB * 64 * kStageU2];
  __shared__ uint32_t s_chroma_all[HIC_ENC_WPB][2 * 8 * 64];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bx = __builtin_amdgcn_readfirstlane(B.xcd ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x);
  const int g = __builtin_amdgcn_readfirstlane(bx * HIC_ENC_WPB + wv);
  if (g >= B.unit0[B.n]) return;  // wave-uniform
  int j = 0;
  while (j + 1 < B.n && g >= B.unit0[j + 1]) ++j;  // wave-uniform
  encode_unit<TMF, false>(B.e[j], g - B.unit0[j], lane, s_stage + wv * 64 * kStageU2, s_chroma_all[wv]);
}

// Memory-only probe of k_encode420's byte pattern (bench.py's in-run floor for the
// fused kernel): the same grid, unit order and 19 row loads per unit, the LDS stage
// and the three passes' 1 KiB nontemporal stores plus their records, no colour
// conversion, pyrDown, DCT or RLE summary.  SLOTS: the slot layout's outputs instead
// -- each record's n_r symbols (read from the index of an earlier real encode into
// the same buffers) copied out of the stage in the kernel's 16 + 32 B nontemporal
// stores, the DC differences, the record and its last DC.
__device__ __forceinline__ void probe_slot_out(const uint2 *st2, int lane, int n, uint8_t *len, int16_t *val) {
  // slot_pass's copy-out: 16 lengths (from 32 B of the stage) and 8 values (16 B) per
  // lane per store, each store instruction 1 KiB contiguous
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint4 *src = reinterpret_cast<const uint4 *>(st2);
  for (int c = lane; 16 * c < n; c += 64) {
    const uint4 p = src[(2 * c) & 511], q = src[(2 * c + 1) & 511];
    __builtin_nontemporal_store(u32x4{p.x ^ q.y, p.y ^ q.x, p.z ^ q.w, p.w ^ q.z}, reinterpret_cast<u32x4 *>(len) + c);
  }
  for (int c = lane; 8 * c < n; c += 64) {
    const uint4 p = src[c & 511];
    __builtin_nontemporal_store(u32x4{p.x, p.y, p.z, p.w}, reinterpret_cast<u32x4 *>(val) + c);
  }
}

template <bool SLOTS = false>
__global__ __launch_bounds__(64 * HIC_ENC_WPB) __attribute__((amdgpu_waves_per_eu(3))) void k_probe_encode420(
    Enc420 E) {
  __shared__ __attribute__((aligned(16))) uint2 s_stage[HIC_ENC_WPB * 64 * kStageU2];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bx = __builtin_amdgcn_readfirstlane(E.xcd ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x);
  const int g = __builtin_amdgcn_readfirstlane(bx * HIC_ENC_WPB + wv);
  if (g >= E.nunits) return;  // wave-uniform
  const int u0 = __builtin_amdgcn_readfirstlane(g / E.nstrips), s = __builtin_amdgcn_readfirstlane(g - u0 * E.nstrips);
  const int y0 = E.out_row0 + 16 * u0, nbx = E.W >> 3, nbxc = E.W >> 4;
  uint2 *st2 = s_stage + wv * 64 * kStageU2;
  uint2 yq[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) yq[r] = make_uint2(0, 0);
  EncColour<19, HIC_ENC_LA3, true> C;
  const bool rev = E.alt && (u0 & 1);
  C.init(E, y0, s, lane, 64, rev);
  C.fold_rows(yq, rev);
  for (int p = 0; p < 3; ++p) {  // Y block rows 0 and 1, then Cr | Cb
    uint2 *row = st2 + lane * kStageU2;
#pragma unroll
    for (int k = 0; k < 16; ++k) row[k] = make_uint2(yq[k].x ^ p, yq[k].y);
    __builtin_amdgcn_wave_barrier();
    if constexpr (SLOTS) {
      const int64_t b0 = p < 2 ? (int64_t)(2 * u0 + p) * nbx + 64 * s : (int64_t)u0 * nbxc + 32 * s;
      const int64_t r = p < 2 ? b0 >> 6 : b0 >> 5;
      const int np = p < 2 ? 1 : 2;
      for (int h = 0; h < np; ++h) {
        const int k = p < 2 ? 0 : 1 + h, cap = p < 2 ? kSlotY : kSlotC;
        const int n = __builtin_amdgcn_readfirstlane(E.nsym[k][4 * r]);
        probe_slot_out(st2, lane, n, E.slen[k] + r * cap, E.sval[k] + r * cap);
        if (lane < (p < 2 ? 64 : 32)) E.dc[k][b0 + lane] = (int)yq[lane & 15].x;
        if (lane < 3) E.rec[k][r * 3 + lane] = yq[p].y;
        if (lane == 0) E.rdc[k][r] = (int)yq[p].x;
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    int16_t *lo, *hi;
    int64_t *rec;
    if (p < 2) {
      const int64_t b0 = (int64_t)(2 * u0 + p) * nbx + 64 * s;
      lo = E.coef[0] + b0 * 64;
      hi = lo + 32 * 64;
      rec = E.rec[0] + (b0 >> 6) * 3;
    } else {
      const int64_t b0 = (int64_t)u0 * nbxc + 32 * s;
      lo = E.coef[1] + b0 * 64;
      hi = E.coef[2] + b0 * 64;
      rec = E.rec[1] + (b0 >> 5) * 3;
    }
    enc_store(st2, lane, lo, hi);
    if (lane == 0) {
      rec[0] = yq[p].x;
      rec[1] = yq[p].y;
      rec[2] = p;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace
}  // namespace hic

using namespace hic;

// checks one encode's arguments and fills its kernel argument (no launch)
static int prep420(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H, int64_t W, int64_t out_row0,
                   int64_t out_rows, int16_t *coef_y, int16_t *coef_cr, int16_t *coef_cb, void *ws_y, void *ws_cr,
                   void *ws_cb, int max_len, bool seg, int64_t wsb_y, int64_t wsb_c, Enc420 &E, bool &recs,
                   bool &aligned) {
  if (!rgb_rows || !coef_y || !coef_cr || !coef_cb) return arg_error("null pointer");
  if (H < 16 || W < 16 || H >= (1 << 20) || W >= (1 << 20)) return arg_error("image shape");
  if (W % 16 || H % 16) return arg_error("hic_encode420_u8 needs W %% 16 == 0 and H %% 16 == 0");
  if (out_row0 < 0 || out_rows < 16 || out_row0 % 16 || out_rows % 16 || out_row0 + out_rows > H)
    return arg_error("output row range (multiples of 16)");
  const int64_t need0 = out_row0 >= 2 ? out_row0 - 2 : 0;
  const int64_t need1 = out_row0 + out_rows + 1 < H ? out_row0 + out_rows + 1 : H;
  if (in_row0 > need0 || in_row0 + in_rows < need1) return arg_error("input rows do not cover the pyrDown halo");
  if (reinterpret_cast<uintptr_t>(rgb_rows) % 8) return arg_error("rgb must be 8-byte aligned");
  // the RGB rows are read through a buffer resource with 32-bit offsets
  if (in_rows * W * 3 > INT32_MAX) return arg_error("hic_encode420_u8: input rows exceed 2 GiB (use the unfused chain)");
  if ((reinterpret_cast<uintptr_t>(coef_y) | reinterpret_cast<uintptr_t>(coef_cr) |
       reinterpret_cast<uintptr_t>(coef_cb)) % 16)
    return arg_error("coefficient buffers must be 16-byte aligned");
  recs = ws_y && ws_cr && ws_cb;
  if ((ws_y || ws_cr || ws_cb) && !recs) return arg_error("workspaces: all three or none");
  if (recs && (max_len < 0 || max_len > 256)) return arg_error("max_len");
  if (seg && recs) {
    // records per strip segment: a narrow image has more of them than 64-block tiles
    // (hic_rle_rows_workspace_bytes)
    const int64_t ny = (out_rows / 8) * (W / 8), nc = (out_rows / 16) * (W / 16);
    const int64_t need_y = (int64_t)hic_rle_rows_workspace_bytes(ny, W / 8, 1);
    const int64_t need_c = (int64_t)hic_rle_rows_workspace_bytes(nc, W / 16, 2);
    if (wsb_y < need_y || wsb_c < need_c)
      return arg_error("hic_encode420_seg_u8: workspaces of %lld / %lld bytes, %lld / %lld needed", (long long)wsb_y,
                       (long long)wsb_c, (long long)need_y, (long long)need_c);
  }
  E = Enc420{};
  E.rgb = rgb_rows;
  E.in_row0 = (int)in_row0;
  E.in_rows = (int)in_rows;
  E.H = (int)H;
  E.W = (int)W;
  E.out_row0 = (int)out_row0;
  E.out_rows = (int)out_rows;
  E.coef[0] = coef_y;
  E.coef[1] = coef_cr;
  E.coef[2] = coef_cb;
  // ragged last strip: the records come from a tile pass after the launch, or (seg)
  // one per strip segment from the kernel itself
  aligned = W % 512 == 0 || seg;
  E.rec[0] = aligned ? static_cast<int64_t *>(ws_y) : nullptr;
  E.rec[1] = aligned ? static_cast<int64_t *>(ws_cr) : nullptr;
  E.rec[2] = aligned ? static_cast<int64_t *>(ws_cb) : nullptr;
  E.M = max_len;
  E.nstrips = (int)((W + 511) / 512);
  E.wlast = (int)(W - 512 * (int64_t)(E.nstrips - 1));
  E.nunits = E.nstrips * (int)(out_rows / 16);  // waves
  // one wave per unit (no persistent loop: units are the same size, and the
  // hardware's dispatch balances the tail better than a fixed split)
  // default 6: XCD-major workgroups, odd unit rows bottom-up (FETCH_SIZE 109.6 vs
  // 131.7 MB per 8K launch, kernel 58.0 vs 58.9 us, bench 0.0996 vs 0.1004 ms/step
  // median of 10 alternating pairs: profiles/r04/enc_order_xcd)
  const int order = knob(HIC_KNOB_ENCODE_ORDER);
  E.xcd = (order >> 1) & 1;
  E.alt = (order >> 2) & 1;
  return HIC_OK;
}

static int encode420(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H, int64_t W,
                     int64_t out_row0, int64_t out_rows, int16_t *coef_y, int16_t *coef_cr, int16_t *coef_cb,
                     void *ws_y, void *ws_cr, void *ws_cb, int max_len, void *stream, void *ev_start, void *ev_stop,
                     bool seg, int64_t wsb_y = 0, int64_t wsb_c = 0) {
  Enc420 E;
  bool recs = false, aligned = false;
  if (int e = prep420(rgb_rows, in_row0, in_rows, H, W, out_row0, out_rows, coef_y, coef_cr, coef_cb, ws_y, ws_cr,
                      ws_cb, max_len, seg, wsb_y, wsb_c, E, recs, aligned))
    return e;
  const dim3 grid((unsigned)((E.nunits + HIC_ENC_WPB - 1) / HIC_ENC_WPB)), block(64 * HIC_ENC_WPB);
  hipStream_t s = as_stream(stream);
  hipEvent_t e0 = static_cast<hipEvent_t>(ev_start), e1 = static_cast<hipEvent_t>(ev_stop);
  auto launch = [&](auto kern) {
    if (e0 || e1)
      hipExtLaunchKernelGGL(kern, grid, block, 0, s, e0, e1, 0, E);
    else
      hipLaunchKernelGGL(kern, grid, block, 0, s, E);
  };
  if (max_len == 15)
    launch(k_encode420<15>);
  else
    launch(k_encode420<0>);
  if (int e = check_launch("k_encode420")) return e;
  if (recs && !aligned) {  // one record per 64-block tile, all three planes (not seg)
    const int64_t ny = (out_rows / 8) * (W / 8), nc = (out_rows / 16) * (W / 16);
    if (int e = rle_tile16_launch(coef_y, ny, max_len, static_cast<int64_t *>(ws_y), s)) return e;
    if (int e = rle_tile16_launch(coef_cr, nc, max_len, static_cast<int64_t *>(ws_cr), s)) return e;
    if (int e = rle_tile16_launch(coef_cb, nc, max_len, static_cast<int64_t *>(ws_cb), s)) return e;
  }
  return HIC_OK;
}

extern "C" int hic_encode420_u8(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H, int64_t W,
                                int64_t out_row0, int64_t out_rows, int16_t *coef_y, int16_t *coef_cr,
                                int16_t *coef_cb, void *ws_y, void *ws_cr, void *ws_cb, int max_len, void *stream,
                                void *ev_start, void *ev_stop) {
  return encode420(rgb_rows, in_row0, in_rows, H, W, out_row0, out_rows, coef_y, coef_cr, coef_cb, ws_y, ws_cr, ws_cb,
                   max_len, stream, ev_start, ev_stop, false);
}

extern "C" int hic_encode420_batch_u8(int n, const hic_encode420_job *jobs, int max_len, void *stream,
                                     void *ev_start, void *ev_stop) {
  if (n < 1 || n > kEncBatchMax || !jobs) return arg_error("1 <= n <= %d jobs", kEncBatchMax);
  if (max_len != 15 && max_len != 0) return arg_error("max_len 15 or 0");
  Enc420Batch B{};
  B.n = n;
  B.unit0[0] = 0;
  for (int j = 0; j < n; ++j) {  // every job checked before the launch
    const hic_encode420_job &J = jobs[j];
    bool recs = false, aligned = false;
    if (int e = prep420(J.rgb_rows, J.in_row0, J.in_rows, J.H, J.W, J.out_row0, J.out_rows, J.coef_y, J.coef_cr,
                        J.coef_cb, J.ws_y, J.ws_cr, J.ws_cb, max_len, false, 0, 0, B.e[j], recs, aligned))
      return e;
    if (recs && !aligned) return arg_error("job %d: W %% 512 != 0 (the records need a tile pass: encode it alone)", j);
    if ((int64_t)B.unit0[j] + B.e[j].nunits > INT32_MAX / 64) return arg_error("too many units");
    B.unit0[j + 1] = B.unit0[j] + B.e[j].nunits;
  }
  B.xcd = B.e[0].xcd;
  const dim3 grid((unsigned)((B.unit0[n] + HIC_ENC_WPB - 1) / HIC_ENC_WPB)), block(64 * HIC_ENC_WPB);
  hipStream_t s = as_stream(stream);
  hipEvent_t e0 = static_cast<hipEvent_t>(ev_start), e1 = static_cast<hipEvent_t>(ev_stop);
  auto launch = [&](auto kern) {
    if (e0 || e1)
      hipExtLaunchKernelGGL(kern, grid, block, 0, s, e0, e1, 0, B);
    else
      hipLaunchKernelGGL(kern, grid, block, 0, s, B);
  };
  if (max_len == 15)
    launch(k_encode420_batch<15>);
  else
    launch(k_encode420_batch<0>);
  return check_launch("k_encode420_batch");
}

extern "C" int hic_encode420_seg_u8(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H, int64_t W,
                                    int64_t out_row0, int64_t out_rows, int16_t *coef_y, int16_t *coef_cr,
                                    int16_t *coef_cb, void *ws_y, void *ws_cr, void *ws_cb, int64_t ws_bytes_y,
                                    int64_t ws_bytes_c, int max_len, void *stream, void *ev_start, void *ev_stop) {
  return encode420(rgb_rows, in_row0, in_rows, H, W, out_row0, out_rows, coef_y, coef_cr, coef_cb, ws_y, ws_cr, ws_cb,
                   max_len, stream, ev_start, ev_stop, true, ws_bytes_y, ws_bytes_c);
}

extern "C" int hic_encode420_slots_u8(const uint8_t *rgb, int64_t H, int64_t W, const hic_slot_job *jobs,
                                      int max_len, void *stream, void *ev_start, void *ev_stop) {
  if (!rgb || !jobs) return arg_error("null pointer");
  if (max_len != kSlotM) return arg_error("the slot layout needs max_len 15");
  if (H < 16 || W < 512 || H % 16 || W % 512 || H >= (1 << 20) || W >= (1 << 20))
    return arg_error("hic_encode420_slots_u8 needs W %% 512 == 0 and H %% 16 == 0");
  if (H * W * 3 > INT32_MAX) return arg_error("image exceeds 2 GiB (32-bit buffer offsets)");
  if (reinterpret_cast<uintptr_t>(rgb) % 8) return arg_error("rgb must be 8-byte aligned");
  const int64_t nblk[3] = {(H / 8) * (W / 8), (H / 16) * (W / 16), (H / 16) * (W / 16)};
  const int rpt[3] = {1, 2, 2};
  // validate every job before anything is launched
  for (int k = 0; k < 3; ++k) {
    const hic_slot_job &J = jobs[k];
    if (!J.slot_len || !J.slot_val || !J.dc_diff || !J.workspace) return arg_error("job %d: null pointer", k);
    if (J.nblk != nblk[k] || J.records_per_tile != rpt[k])
      return arg_error("job %d: nblk %lld / records_per_tile %lld, expected %lld / %d", k, (long long)J.nblk,
                       (long long)J.records_per_tile, (long long)nblk[k], rpt[k]);
    if ((reinterpret_cast<uintptr_t>(J.slot_len) | reinterpret_cast<uintptr_t>(J.slot_val)) % 16)
      return arg_error("job %d: slot arrays must be 16-byte aligned", k);
    const int64_t need = (int64_t)hic_rle_slots_workspace_bytes(nblk[k], rpt[k]);
    if (J.workspace_bytes < need)
      return arg_error("job %d: workspace of %lld bytes, %lld needed", k, (long long)J.workspace_bytes,
                       (long long)need);
  }
  Enc420 E{};
  E.rgb = rgb;
  E.in_row0 = 0;
  E.in_rows = (int)H;
  E.H = (int)H;
  E.W = (int)W;
  E.out_row0 = 0;
  E.out_rows = (int)H;
  for (int k = 0; k < 3; ++k) {
    E.rec[k] = static_cast<int64_t *>(jobs[k].workspace);
    E.slen[k] = jobs[k].slot_len;
    E.sval[k] = jobs[k].slot_val;
    E.dc[k] = jobs[k].dc_diff;
    E.rdc[k] = reinterpret_cast<int32_t *>(E.rec[k] + slot_rdc_word(slot_nrec(nblk[k], rpt[k])));
  }
  E.M = kSlotM;
  E.nstrips = (int)(W / 512);
  E.wlast = 512;
  E.nunits = E.nstrips * (int)(H / 16);
  const int order = knob(HIC_KNOB_ENCODE_ORDER);
  E.xcd = (order >> 1) & 1;
  E.alt = (order >> 2) & 1;
  const dim3 grid((unsigned)((E.nunits + HIC_ENC_WPB - 1) / HIC_ENC_WPB)), block(64 * HIC_ENC_WPB);
  const hipStream_t s = as_stream(stream);
  const hipEvent_t e0 = static_cast<hipEvent_t>(ev_start), e1 = static_cast<hipEvent_t>(ev_stop);
  if (e0 || e1)
    hipExtLaunchKernelGGL((k_encode420<kSlotM, true>), grid, block, 0, s, e0, e1, 0, E);
  else
    hipLaunchKernelGGL((k_encode420<kSlotM, true>), grid, block, 0, s, E);
  return check_launch("k_encode420<slots>");
}

extern "C" int hic_probe_encode420(const uint8_t *rgb, int64_t H, int64_t W, int16_t *coef_y, int16_t *coef_cr,
                                   int16_t *coef_cb, int64_t *rec_y, int64_t *rec_c, void *stream, void *ev_start,
                                   void *ev_stop) {
  if (!rgb || !coef_y || !coef_cr || !coef_cb || !rec_y || !rec_c) return arg_error("null pointer");
  if (H < 16 || W < 512 || H % 16 || W % 512 || H >= (1 << 20) || W >= (1 << 20))
    return arg_error("hic_probe_encode420 needs W %% 512 == 0 and H %% 16 == 0");
  if (H * W * 3 > INT32_MAX) return arg_error("image exceeds 2 GiB");
  if (reinterpret_cast<uintptr_t>(rgb) % 8 ||
      (reinterpret_cast<uintptr_t>(coef_y) | reinterpret_cast<uintptr_t>(coef_cr) |
       reinterpret_cast<uintptr_t>(coef_cb)) % 16)
    return arg_error("alignment");
  Enc420 E{};
  E.rgb = rgb;
  E.in_row0 = 0;
  E.in_rows = (int)H;
  E.H = (int)H;
  E.W = (int)W;
  E.out_row0 = 0;
  E.out_rows = (int)H;
  E.coef[0] = coef_y;
  E.coef[1] = coef_cr;
  E.coef[2] = coef_cb;
  E.rec[0] = rec_y;
  E.rec[1] = rec_c;
  E.nstrips = (int)(W / 512);
  E.wlast = 512;
  E.nunits = E.nstrips * (int)(H / 16);
  const int order = knob(HIC_KNOB_ENCODE_ORDER);
  E.xcd = (order >> 1) & 1;
  E.alt = (order >> 2) & 1;
  const dim3 grid((unsigned)((E.nunits + HIC_ENC_WPB - 1) / HIC_ENC_WPB)), block(64 * HIC_ENC_WPB);
  const hipStream_t s = as_stream(stream);
  const hipEvent_t e0 = static_cast<hipEvent_t>(ev_start), e1 = static_cast<hipEvent_t>(ev_stop);
  if (e0 || e1)
    hipExtLaunchKernelGGL(k_probe_encode420<false>, grid, block, 0, s, e0, e1, 0, E);
  else
    hipLaunchKernelGGL(k_probe_encode420<false>, grid, block, 0, s, E);
  return check_launch("k_probe_encode420");
}

extern "C" int hic_probe_encode420_slots(const uint8_t *rgb, int64_t H, int64_t W, const hic_slot_job *jobs,
                                         void *stream, void *ev_start, void *ev_stop) {
  if (!rgb || !jobs) return arg_error("null pointer");
  if (H < 16 || W < 512 || H % 16 || W % 512 || H >= (1 << 20) || W >= (1 << 20))
    return arg_error("hic_probe_encode420_slots needs W %% 512 == 0 and H %% 16 == 0");
  if (H * W * 3 > INT32_MAX) return arg_error("image exceeds 2 GiB");
  if (reinterpret_cast<uintptr_t>(rgb) % 8) return arg_error("alignment");
  const int64_t nblk[3] = {(H / 8) * (W / 8), (H / 16) * (W / 16), (H / 16) * (W / 16)};
  const int rpt[3] = {1, 2, 2};
  Enc420 E{};
  for (int k = 0; k < 3; ++k) {
    const hic_slot_job &J = jobs[k];
    if (!J.slot_len || !J.slot_val || !J.dc_diff || !J.workspace || !J.d_index) return arg_error("job %d: null", k);
    if (J.nblk != nblk[k] || J.records_per_tile != rpt[k]) return arg_error("job %d: shape", k);
    if ((reinterpret_cast<uintptr_t>(J.slot_len) | reinterpret_cast<uintptr_t>(J.slot_val)) % 16)
      return arg_error("job %d: alignment", k);
    if (J.workspace_bytes < (int64_t)hic_rle_slots_workspace_bytes(nblk[k], rpt[k])) return arg_error("workspace");
    E.rec[k] = static_cast<int64_t *>(J.workspace);
    E.slen[k] = J.slot_len;
    E.sval[k] = J.slot_val;
    E.dc[k] = J.dc_diff;
    E.rdc[k] = reinterpret_cast<int32_t *>(E.rec[k] + slot_rdc_word(slot_nrec(nblk[k], rpt[k])));
    E.nsym[k] = J.d_index;
  }
  E.rgb = rgb;
  E.in_row0 = 0;
  E.in_rows = (int)H;
  E.H = (int)H;
  E.W = (int)W;
  E.out_row0 = 0;
  E.out_rows = (int)H;
  E.nstrips = (int)(W / 512);
  E.wlast = 512;
  E.nunits = E.nstrips * (int)(H / 16);
  const int order = knob(HIC_KNOB_ENCODE_ORDER);
  E.xcd = (order >> 1) & 1;
  E.alt = (order >> 2) & 1;
  const dim3 grid((unsigned)((E.nunits + HIC_ENC_WPB - 1) / HIC_ENC_WPB)), block(64 * HIC_ENC_WPB);
  const hipStream_t s = as_stream(stream);
  const hipEvent_t e0 = static_cast<hipEvent_t>(ev_start), e1 = static_cast<hipEvent_t>(ev_stop);
  if (e0 || e1)
    hipExtLaunchKernelGGL(k_probe_encode420<true>, grid, block, 0, s, e0, e1, 0, E);
  else
    hipLaunchKernelGGL(k_probe_encode420<true>, grid, block, 0, s, E);
  return check_launch("k_probe_encode420<slots>");
}
