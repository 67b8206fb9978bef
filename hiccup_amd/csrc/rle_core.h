// rle_core.h -- run-length building blocks shared by the RLE kernels (rle.hip)
// and the fused plane encoder (encode.hip).  Reference: codec.run_length_coding
// (codec.py:55-99); see rle.hip for the stream semantics.
#pragma once
#include "hic_common.h"

namespace hic {
namespace {

// ---- wave scan helpers -----------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(v, d, 64);
    if (lane >= d) v = v > o ? v : o;
  }
  return v;
}

// int32 wave64 inclusive scans on DPP (no LDS round trips): row_shr 1/2/4/8
// inside each 16-lane row, then row_bcast:15 / row_bcast:31 across rows (GFX9
// DPP).  Lanes whose DPP source is out of range read `ident`.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ int dpp_i32(int ident, int v) {
  return __builtin_amdgcn_update_dpp(ident, v, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ int wave_incl_sum_i32(int v) {
  v += dpp_i32<0x111>(0, v);
  v += dpp_i32<0x112>(0, v);
  v += dpp_i32<0x114>(0, v);
  v += dpp_i32<0x118>(0, v);
  v += dpp_i32<0x142, 0xA>(0, v);
  v += dpp_i32<0x143, 0xC>(0, v);
  return v;
}
__device__ __forceinline__ int wave_incl_max_i32(int v) {
  constexpr int I = -2147483647 - 1;
  v = max(v, dpp_i32<0x111>(I, v));
  v = max(v, dpp_i32<0x112>(I, v));
  v = max(v, dpp_i32<0x114>(I, v));
  v = max(v, dpp_i32<0x118>(I, v));
  v = max(v, dpp_i32<0x142, 0xA>(I, v));
  v = max(v, dpp_i32<0x143, 0xC>(I, v));
  return v;
}
// lane i <- lane i-1 (lane 0 <- ident)
__device__ __forceinline__ int wave_shr1_i32(int ident, int v) { return dpp_i32<0x138>(ident, v); }
__device__ __forceinline__ int wave_last_i32(int v) { return __builtin_amdgcn_readlane(v, 63); }

// run / M without a 64-bit division (a long software sequence on the GPU): runs
// are < 2^32 in practice; M = 15 (jpeg_encode's default) by multiply-shift.
__device__ __attribute__((noinline)) int64_t div_run_wide(int64_t run, int M) { return run / M; }
__device__ __forceinline__ int64_t div_run(int64_t run, int M) {
  if ((uint64_t)run < (1ull << 32)) {
    const uint32_t r = (uint32_t)run;
    if (M == 15) return (int64_t)(((uint64_t)r * 0x88888889ull) >> 35);  // exact for all uint32
    return (int64_t)(r / (uint32_t)M);
  }
  return div_run_wide(run, M);  // out of line: keeps every inlined caller small
}
__device__ __forceinline__ int syms_for_run(int64_t run, int M) { return 1 + (M > 0 ? (int)div_run(run, M) : 0); }

// AC element j (0..62) of a zig-zag int16 block held as 32 packed dwords.
__device__ __forceinline__ int zz_ac(const uint32_t (&w)[32], int j) {
  const int s = j + 1;
  return (int)(int16_t)((w[s >> 1] >> (16 * (s & 1))) & 0xFFFFu);
}

template <int MF>
__device__ __forceinline__ int div_m(int run, int M) {
  return MF == 15 ? (int)(((uint32_t)run * 0x8889u) >> 19) : run / M;  // exact for run < 2^16
}

// Interleave the low 16 bits of a with the low 16 bits of b: bit k of a -> bit
// 2k, bit k of b -> bit 2k+1.
__device__ __forceinline__ uint32_t zip16(uint32_t a, uint32_t b) {
  auto spread = [](uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
  };
  return spread(a) | (spread(b) << 1);
}

// v_pk_min_u16 (the compiler rewrites a vector min with 1 into compares)
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  const uint32_t lo = (a & 0xFFFFu) < (b & 0xFFFFu) ? (a & 0xFFFFu) : (b & 0xFFFFu);
  const uint32_t hi = (a >> 16) < (b >> 16) ? (a >> 16) : (b >> 16);
  return lo | hi << 16;
#endif
}
// Nonzero mask of a zig-zag int16 block held as 32 packed dwords: bit s set iff
// slot s != 0.  v_pk_min_u16(w, 1) turns each half into its 0/1 flag.
__device__ __forceinline__ uint64_t nz_mask16(const uint32_t (&w)[32]) {
  uint32_t lo[2] = {0, 0}, hi[2] = {0, 0};  // [half]: flags of even / odd slots
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      acc |= pk_min_u16(w[16 * h + k], 0x00010001u) << k;
    }
    lo[h] = acc & 0xFFFFu;  // even slots 32h + 2k
    hi[h] = acc >> 16;      // odd slots 32h + 2k + 1
  }
  return (uint64_t)zip16(lo[0], hi[0]) | ((uint64_t)zip16(lo[1], hi[1]) << 32);
}

// first / last nonzero AC index (-1 if none) and the symbols of every nonzero
// after the first (runs inside the block), from the block's AC nonzero mask
// (bit j = AC j, j = 0..62).
template <int MF>
__device__ __forceinline__ void summarize_ac(uint64_t ac, int M, int &first, int &last, int &nsym) {
  if (ac == 0) {
    first = last = -1;
    nsym = 0;
    return;
  }
  first = __builtin_ctzll(ac);
  last = 63 - __builtin_clzll(ac);
  const int cnt = __builtin_popcountll(ac);
  nsym = cnt - 1;
  if (M <= 0) return;
  // zeros strictly inside [first, last]; a run of >= M of them needs fillers
  const uint64_t span = (last >= 63 ? ~0ull : ((2ull << last) - 1)) & ~((1ull << first) - 1);
  uint64_t z = ~ac & span;
  bool long_gap;
  if (MF == 15) {
    const uint64_t z2 = z & (z >> 1), z4 = z2 & (z2 >> 2), z8 = z4 & (z4 >> 4);
    long_gap = (z8 & (z4 >> 8) & (z2 >> 12) & (z >> 14)) != 0;  // 15 consecutive zeros somewhere
  } else {
    long_gap = M <= 63;
  }
  if (long_gap) {
    uint64_t m = ac & (ac - 1);  // nonzeros after the first
    int pl = first;
    while (m) {
      const int j = __builtin_ctzll(m);
      m &= m - 1;
      nsym += div_m<MF>(j - pl - 1, M);
      pl = j;
    }
  }
}

// the same from a zig-zag int16 block held as 32 packed dwords
template <int MF>
__device__ __forceinline__ void summarize16(const uint32_t (&w)[32], int M, int &first, int &last, int &nsym,
                                            uint64_t *ac_out = nullptr) {
  const uint64_t ac = nz_mask16(w) >> 1;  // bit j = AC j (slot j + 1), j = 0..62
  if (ac_out) *ac_out = ac;
  summarize_ac<MF>(ac, M, first, last, nsym);
}

// ---------------------------------------------------------------------------
// Hot path geometry: int16 zig-zag blocks of 64 (the DCT kernels' ZIGZAG_I16
// output), AC = slots 1..63, one block per lane, one TILE = the 64 blocks of one
// wave.  Tile records (int64 x 3 per tile, in the RLE workspace):
//   [0] global stream position of the tile's first nonzero AC (-1: none)
//   [1] global position of its last nonzero (-1: none)
//   [2] symbols of every nonzero of the tile except the first one's
// (the first nonzero's symbols depend on the zeros carried in from earlier tiles).
constexpr int kWT = 64;  // blocks per hot-path tile

__device__ __forceinline__ void load_block16(const int16_t *__restrict__ blocks, int64_t b, uint32_t (&w)[32]) {
  const uint4 *q = reinterpret_cast<const uint4 *>(blocks + b * 64);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 t = q[k];
    w[4 * k] = t.x; w[4 * k + 1] = t.y; w[4 * k + 2] = t.z; w[4 * k + 3] = t.w;
  }
}

// Wave-level: the tile record's three values (wave-uniform) from each lane's block
// summary.  Every lane must call it.
__device__ __forceinline__ void tile_record_values(int first, int last, int nsym, int64_t b, int M, int64_t &r0,
                                                   int64_t &r1, int64_t &r2) {
  const int lane = threadIdx.x & 63;
  const int lastr = last >= 0 ? lane * 63 + last : -1;
  const int incl = wave_incl_max_i32(lastr);
  const int prev = wave_shr1_i32(-1, incl);
  int cnt = nsym;
  if (first >= 0 && prev >= 0) cnt += syms_for_run(lane * 63 + first - prev - 1, M);
  const int total = wave_last_i32(wave_incl_sum_i32(cnt));
  const int all_last = wave_last_i32(incl);
  const int64_t base = (b - lane) * 63;
  const uint64_t fm = __builtin_amdgcn_ballot_w64(first >= 0 && prev < 0);
  const int fl = fm ? __builtin_ctzll(fm) : 0;
  const int ff = __builtin_amdgcn_readlane(lane * 63 + first, fl);
  r0 = all_last < 0 ? -1 : base + ff;
  r1 = all_last >= 0 ? base + all_last : -1;
  r2 = total;
}

// Wave-level: the tile record from each lane's block summary (first / last nonzero
// AC, symbols after the first; first = last = -1, nsym = 0 for a missing block).
// Every lane must call it.
__device__ __forceinline__ void tile_record_fs(int first, int last, int nsym, int64_t b, int M,
                                               int64_t *__restrict__ rec) {
  const int lane = threadIdx.x & 63;
  // positions relative to the tile's first AC element (lane * 63 + j) fit int32
  const int lastr = last >= 0 ? lane * 63 + last : -1;
  const int incl = wave_incl_max_i32(lastr);
  const int prev = wave_shr1_i32(-1, incl);  // last nonzero of earlier lanes, -1: none
  int cnt = nsym;
  if (first >= 0 && prev >= 0) cnt += syms_for_run(lane * 63 + first - prev - 1, M);
  const int total = wave_last_i32(wave_incl_sum_i32(cnt));
  const int all_last = wave_last_i32(incl);
  const int64_t base = (b - lane) * 63;  // the tile's first AC element
  // rec[0]: the lane of the tile's first nonzero, or lane 0 (-1) in a tile without one
  if (all_last < 0 ? lane == 0 : (first >= 0 && prev < 0)) rec[0] = all_last < 0 ? -1 : base + lane * 63 + first;
  if (lane == 0) {
    rec[1] = all_last >= 0 ? base + all_last : -1;
    rec[2] = total;
  }
}

// Wave-level: the tile record of the 64 blocks held by this wave's lanes
// (valid = this lane's block exists).  Every lane must call it.
template <int MF>
__device__ __forceinline__ void tile_record16(const uint32_t (&w)[32], bool valid, int64_t b, int M,
                                              int64_t *__restrict__ rec) {
  int first = -1, last = -1, nsym = 0;
  if (valid) summarize16<MF>(w, M, first, last, nsym);
  tile_record_fs(first, last, nsym, b, M, rec);
}

// Copy n elements from LDS (element e at s[a + e]) to global g[o0 + e], where
// a == o0 mod (4 / sizeof(T)): aligned 4-byte stores by the 64 lanes of a wave,
// element stores at the edges.
template <typename T>
__device__ __forceinline__ void copy_out_wave(const T *s, int a, T *__restrict__ g, int64_t o0, int n, int64_t cap) {
  constexpr int E = 4 / (int)sizeof(T);  // elements per word
  const int lane = threadIdx.x & 63;
  const int64_t w0 = o0 / E, w1 = (o0 + n + E - 1) / E;
  // whole words inside [o0, o0 + n) and below the cap: aligned 4-byte copies,
  // four LDS reads in flight per lane
  const int64_t i0 = (o0 + E - 1) / E;
  int64_t i1 = (o0 + n) / E;
  if (i1 > cap / E) i1 = cap / E;
  if (i1 < i0) i1 = i0;
  auto src = [&](int64_t w) { return *reinterpret_cast<const uint32_t *>(s + (int)(w * E - o0) + a); };
  int64_t w = i0 + lane;
  for (; w + 192 < i1; w += 256) {
    const uint32_t v0 = src(w), v1 = src(w + 64), v2 = src(w + 128), v3 = src(w + 192);
    *reinterpret_cast<uint32_t *>(g + w * E) = v0;
    *reinterpret_cast<uint32_t *>(g + (w + 64) * E) = v1;
    *reinterpret_cast<uint32_t *>(g + (w + 128) * E) = v2;
    *reinterpret_cast<uint32_t *>(g + (w + 192) * E) = v3;
  }
  for (; w < i1; w += 64) *reinterpret_cast<uint32_t *>(g + w * E) = src(w);
  // partial words at either end (and any words cut by the cap): element stores
  auto edge = [&](int64_t ew) {
    for (int k = 0; k < E; ++k) {
      const int64_t e = ew * E + k;
      if (e >= o0 && e < o0 + n && e < cap) g[e] = s[(int)(e - o0) + a];
    }
  };
  if (lane == 0 && w0 < i0) edge(w0);
  for (int64_t ew = (i1 > w0 ? i1 : w0 + (w0 < i0 ? 1 : 0)) + lane; ew < w1; ew += 64) edge(ew);
}

// 32-lane segmented int32 inclusive scans (lanes 0-31 and 32-63 independent): the
// wave scans without their last step (row_bcast:31 joins the two halves).
__device__ __forceinline__ int seg32_incl_sum_i32(int v) {
  v += dpp_i32<0x111>(0, v);
  v += dpp_i32<0x112>(0, v);
  v += dpp_i32<0x114>(0, v);
  v += dpp_i32<0x118>(0, v);
  v += dpp_i32<0x142, 0xA>(0, v);
  return v;
}
__device__ __forceinline__ int seg32_incl_max_i32(int v) {
  constexpr int I = -2147483647 - 1;
  v = max(v, dpp_i32<0x111>(I, v));
  v = max(v, dpp_i32<0x112>(I, v));
  v = max(v, dpp_i32<0x114>(I, v));
  v = max(v, dpp_i32<0x118>(I, v));
  v = max(v, dpp_i32<0x142, 0xA>(I, v));
  return v;
}

// Two half-tile records at once: lanes 0-31 hold blocks b0 .. b0 + 31 of one stream
// (record -> rec_lo), lanes 32-63 the same block indices of another stream (->
// rec_hi); each record covers 32 blocks (a 64-block tile's two halves combine as
// the scan's agg_combine does), or the first nvalid of them (a ragged row segment).
// Same fields as tile_record16.
template <int MF>
__device__ __forceinline__ void tile_record16_half(const uint32_t (&w)[32], int64_t b0, int M,
                                                   int64_t *__restrict__ rec_lo, int64_t *__restrict__ rec_hi,
                                                   int nvalid = 32) {
  const int lane = threadIdx.x & 63, sl = lane & 31;
  int first = -1, last = -1, nsym = 0;
  if (sl < nvalid) summarize16<MF>(w, M, first, last, nsym);  // nvalid: blocks of each half that exist
  const int lastr = last >= 0 ? sl * 63 + last : -1;
  const int incl = seg32_incl_max_i32(lastr);
  int prev = wave_shr1_i32(-1, incl);
  if (sl == 0) prev = -1;
  int cnt = nsym;
  if (first >= 0 && prev >= 0) cnt += syms_for_run(sl * 63 + first - prev - 1, M);
  const int icnt = seg32_incl_sum_i32(cnt);
  const int tot_lo = __builtin_amdgcn_readlane(icnt, 31), tot_hi = __builtin_amdgcn_readlane(icnt, 63);
  const int all_lo = __builtin_amdgcn_readlane(incl, 31), all_hi = __builtin_amdgcn_readlane(incl, 63);
  const int all_last = lane < 32 ? all_lo : all_hi, total = lane < 32 ? tot_lo : tot_hi;
  int64_t *rec = lane < 32 ? rec_lo : rec_hi;
  const int64_t base = b0 * 63;
  if (all_last < 0 ? sl == 0 : (first >= 0 && prev < 0)) rec[0] = all_last < 0 ? -1 : base + sl * 63 + first;
  if (sl == 0) {
    rec[1] = all_last >= 0 ? base + all_last : -1;
    rec[2] = total;
  }
}

// Copy n elements from LDS (element e at s[a + e], s 16-byte aligned) to global
// g[o0 + e] (g 16-byte aligned), where a == o0 mod (16 / sizeof(T)): one
// ds_read_b128 + global_store_dwordx4 per 16-byte chunk, element stores for the
// partial chunks at either end and anything cut by the cap.
template <typename T, bool NT = false>
__device__ __forceinline__ void copy_out_wave16(const T *s, int a, T *__restrict__ g, int64_t o0, int n, int64_t cap) {
  constexpr int C = 16 / (int)sizeof(T);  // elements per chunk
  const int lane = threadIdx.x & 63;
  const int64_t c0 = (o0 + C - 1) / C;
  int64_t c1 = (o0 + n) / C;
  if (c1 > cap / C) c1 = cap / C;
  if (c1 < c0) c1 = c0;
  const int64_t sb = o0 - a;  // global element at s[0]
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  for (int64_t c = c0 + lane; c < c1; c += 64) {
    const u32x4 v = *reinterpret_cast<const u32x4 *>(s + (int)(c * C - sb));
    if (NT)  // nontemporal (nt): streaming output, no reuse in this launch
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(g + c * C));
    else
      *reinterpret_cast<u32x4 *>(g + c * C) = v;
  }
  // head: [o0, c0*C); tail: [c1*C, o0+n) -- each at most C - 1 elements unless the cap cut
  const int64_t hend = c0 * C < o0 + n ? c0 * C : o0 + n;
  for (int64_t e = o0 + lane; e < hend; e += 64)
    if (e < cap) g[e] = s[(int)(e - sb)];
  const int64_t tbeg = c1 * C > hend ? c1 * C : hend;
  for (int64_t e = tbeg + lane; e < o0 + n; e += 64)
    if (e < cap) g[e] = s[(int)(e - sb)];
}

// ---- indexed tile gather -----------------------------------------------------
// One wave expands the symbols [o0, o1) of one 64-block tile into its zeroed LDS
// tile: AC position j of block b goes to win[b * ROW + 1 + j] (slot 0 is the DC,
// slots 64 .. ROW-1 padding).  codec.decode_run_length's expansion (codec.py:102-113)
// for the blocks of one tile, from the encoder-side index (k_rld_indexed16,
// k_rld_idct_indexed).  P: the position after the previous tile's last symbol,
// relative to this tile (<= 0: a run carried in starts before it); returns P after
// this tile's last symbol.
//
// A wave step takes 64 G symbols, G consecutive ones per lane, loaded as whole
// vectors.  The symbols of the step's first and last group that belong to other
// tiles are not masked one by one: the lane holding o0 starts its positions
// Σ(len+1) of its leading foreign symbols early, so they land before the tile
// (negative positions), and every lane stops at `lim`, the position after its last
// own symbol, so the trailing foreign ones land after it.  Each symbol is then
// q += len + 1, one compare, q / 63 = (q * 2081) >> 17 on [0, 4032), and one
// ds_write_b16 to its slot or to the lane's trash slot (never read) -- no branch.
#ifndef HIC_DEC_G
#define HIC_DEC_G 16  // the decoders' G
#endif
#ifndef HIC_DEC_PF
#define HIC_DEC_PF 2  // and D (2 = one step ahead; 1-6 measured equal)
#endif
template <int G>
struct SymGroup {
  uint32_t l[G / 4];  // G lengths (bytes)
  uint32_t v[G / 2];  // G values (int16 pairs)
};
template <int G>
__device__ __forceinline__ void load_group(const uint8_t *__restrict__ sym_len, const int16_t *__restrict__ sym_val,
                                           int64_t s0, int64_t nsym, SymGroup<G> &x) {
  typedef uint32_t vl_t __attribute__((ext_vector_type(G / 4)));
  typedef uint32_t vv_t __attribute__((ext_vector_type(G / 2)));
  if (s0 + G <= nsym) {  // s0 is a multiple of G: aligned vector loads
    const vl_t l = *reinterpret_cast<const vl_t *>(sym_len + s0);
    const vv_t v = *reinterpret_cast<const vv_t *>(sym_val + s0);
#pragma unroll
    for (int j = 0; j < G / 4; ++j) x.l[j] = l[j];
#pragma unroll
    for (int j = 0; j < G / 2; ++j) x.v[j] = v[j];
  } else {  // the stream's last group: nothing past nsym is read
#pragma unroll
    for (int j = 0; j < G / 4; ++j) x.l[j] = 0;
#pragma unroll
    for (int j = 0; j < G / 2; ++j) x.v[j] = 0;
#pragma unroll
    for (int k = 0; k < G; ++k)
      if (s0 + k < nsym) {
        x.l[k >> 2] |= (uint32_t)sym_len[s0 + k] << (8 * (k & 3));
        x.v[k >> 1] |= (uint32_t)(uint16_t)sym_val[s0 + k] << (16 * (k & 1));
      }
  }
}
// n + the sum of the first n lengths (0 <= n <= G)
template <int G>
__device__ __forceinline__ int len_prefix(const SymGroup<G> &x, int n) {
  int a = n;
#pragma unroll
  for (int j = 0; j < G / 4; ++j) {
    const int m = n - 4 * j;
    const uint32_t mask = m >= 4 ? 0xFFFFFFFFu : (m <= 0 ? 0u : (1u << (8 * m)) - 1u);
    a = (int)__builtin_amdgcn_udot4(x.l[j] & mask, 0x01010101u, (uint32_t)a, false);
  }
  return a;
}
template <int ROW, int G, int D>
__device__ __forceinline__ int gather_tile(const uint8_t *__restrict__ sym_len, const int16_t *__restrict__ sym_val,
                                           int64_t o0, int64_t o1, int64_t nsym, int P, int span, int16_t *win,
                                           int trash, int lane) {
  static_assert(G == 4 || G == 8 || G == 16, "group size");
  constexpr int S = 64 * G;  // symbols per wave step
  const int64_t c0 = o0 & ~(int64_t)(G - 1);
  // loads run D - 1 steps ahead of their use (a 64-block tile of dense blocks is ~4
  // steps at G = 16).  D = 1 .. 6 measured the same (profiles/r05/decode_gather/):
  // the gather is not waiting on memory latency
  SymGroup<G> ring[D];
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (c0 + i * S < o1) load_group<G>(sym_len, sym_val, c0 + i * S + (int64_t)G * lane, nsym, ring[i]);
  for (int64_t cb = c0; cb < o1; cb += D * S) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int64_t c = cb + i * S;
      if (c >= o1) break;  // wave-uniform
      const SymGroup<G> &cur = ring[i];
      int pre = 0, own;  // Σ(len+1) of the lane's leading foreign symbols / of its own
      if (c >= o0 && c + S <= o1) {  // wave-uniform: every symbol of the step is the tile's
        own = len_prefix<G>(cur, G);
      } else {
        const int64_t s0 = c + (int64_t)G * lane;
        const int64_t a = o0 - s0, e = o1 - s0;
        const int skip = a <= 0 ? 0 : (a >= G ? G : (int)a);
        const int nv = e <= skip ? skip : (e >= G ? G : (int)e);
        pre = len_prefix<G>(cur, skip);
        own = len_prefix<G>(cur, nv) - pre;
      }
      const int incl = wave_incl_sum_i32(own);
      const int end = P + incl;
      uint32_t lim = (uint32_t)(end <= 0 ? 0 : (end < span ? end : span));
      // opaque to the optimiser: it would otherwise split the one unsigned compare
      // below in two and sink the slot arithmetic into a branch per symbol
      asm volatile("" : "+v"(lim));
      int r = end - own - pre;  // r = q + 1 (q: the symbol's position)
#pragma unroll
      for (int k = 0; k < G; ++k) {
        r += (int)((cur.l[k >> 2] >> (8 * (k & 3))) & 255u) + 1;
        // slot + 1 = q + 1 + (ROW - 63) (q / 63), q / 63 = (r * 2081 - 2081) >> 17
        int slot1 = r + __mul24((__mul24(r, 2081) - 2081) >> 17, ROW - 63);
        asm volatile("" : "+v"(slot1));
        slot1 = (uint32_t)(r - 1) < lim ? slot1 : trash;
        win[slot1] = (int16_t)(cur.v[k >> 1] >> (16 * (k & 1)));
      }
      P += wave_last_i32(incl);
      // refill the slot just consumed, D steps ahead
      if (c + D * S < o1) load_group<G>(sym_len, sym_val, c + D * S + (int64_t)G * lane, nsym, ring[i]);
    }
  }
  return P;
}

// The slot-layout form (slots.h): a 64-block tile holds 1 << rsh records, record r's
// n symbols at [r * cap, r * cap + n) of the slot arrays (cap = 63 x 64 >> rsh), its
// first symbol's zeros starting after record-relative position P.  SlotTileIx holds
// the tile's records' {n, P, pdc, nfill} (the close's index), read by scalar loads
// at the top of the decoder so that their latency overlaps its LDS zero-fill.
struct SlotTileIx {
  int4 r[2];
};
__device__ __forceinline__ SlotTileIx slot_tile_ix(const int32_t *sidx, int64_t t, int rsh, int64_t nblk) {
  typedef const __attribute__((address_space(4))) int32_t cint;  // uniform address: s_load
  const int64_t nrec = (nblk + (64 >> rsh) - 1) >> (6 - rsh), r0 = t << rsh;  // records of the plane
  SlotTileIx x;
  cint *a = (cint *)(uintptr_t)(sidx + 4 * r0);
  x.r[0] = make_int4(a[0], a[1], a[2], a[3]);
  x.r[1] = make_int4(0, 0, 0, 0);
  if (rsh && r0 + 1 < nrec) x.r[1] = make_int4(a[4], a[5], a[6], a[7]);
  return x;
}
// Returns the last record's end position (as gather_tile; 0 for a tile without symbols).
template <int ROW>
__device__ __forceinline__ int slots_gather_tile(const uint8_t *__restrict__ slot_len,
                                                 const int16_t *__restrict__ slot_val, const SlotTileIx &ix,
                                                 int64_t t, int rsh, int span, int16_t *win, int trash, int lane) {
  const int capr = 63 * (64 >> rsh);
  int P = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (k > 0 && !rsh) break;
    const int n = __builtin_amdgcn_readfirstlane(ix.r[k].x);
    if (n > 0) {
      const int64_t o0 = ((t << rsh) + k) * capr;
      P = gather_tile<ROW, HIC_DEC_G, HIC_DEC_PF>(slot_len, slot_val, o0, o0 + n, o0 + capr,
                                                 __builtin_amdgcn_readfirstlane(ix.r[k].y) + k * capr, span, win,
                                                 trash, lane);
    }
  }
  return P;
}

}  // namespace
}  // namespace hic
