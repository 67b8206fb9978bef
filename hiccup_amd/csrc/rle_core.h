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

// Symbols produced by a nonzero preceded by `run` zeros: run / M fillers
// (M-1, 0) then (run % M, value).
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

// Nonzero mask of a zig-zag int16 block held as 32 packed dwords: bit s set iff
// slot s != 0.  v_pk_min_u16(w, 1) turns each half into its 0/1 flag.
__device__ __forceinline__ uint64_t nz_mask16(const uint32_t (&w)[32]) {
  uint32_t lo[2] = {0, 0}, hi[2] = {0, 0};  // [half]: flags of even / odd slots
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t x = w[16 * h + k];
      const uint32_t f = ((x & 0xFFFFu) != 0 ? 1u : 0u) | ((x >> 16) != 0 ? 0x10000u : 0u);
      acc |= f << k;
    }
    lo[h] = acc & 0xFFFFu;  // even slots 32h + 2k
    hi[h] = acc >> 16;      // odd slots 32h + 2k + 1
  }
  return (uint64_t)zip16(lo[0], hi[0]) | ((uint64_t)zip16(lo[1], hi[1]) << 32);
}

// first / last nonzero AC index (-1 if none) and the symbols of every nonzero
// after the first (runs inside the block), from the block's nonzero mask.
template <int MF>
__device__ __forceinline__ void summarize16(const uint32_t (&w)[32], int M, int &first, int &last, int &nsym) {
  const uint64_t ac = nz_mask16(w) >> 1;  // bit j = AC j (slot j + 1), j = 0..62
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

// Wave-level: the tile record of the 64 blocks held by this wave's lanes
// (valid = this lane's block exists).  Every lane must call it.
template <int MF>
__device__ __forceinline__ void tile_record16(const uint32_t (&w)[32], bool valid, int64_t b, int M,
                                              int64_t *__restrict__ rec) {
  const int lane = threadIdx.x & 63;
  int first = -1, last = -1, nsym = 0;
  if (valid) summarize16<MF>(w, M, first, last, nsym);
  const int64_t base = b * 63;
  const int64_t lastg = last >= 0 ? base + last : -1;
  const int64_t incl = wave_incl_max(lastg);
  int64_t prev = __shfl_up(incl, 1, 64);
  if (lane == 0) prev = -1;
  int64_t cnt = nsym;
  if (first >= 0 && prev >= 0) cnt += syms_for_run(base + first - prev - 1, M);
  const int64_t total = __shfl(wave_incl_sum(cnt), 63, 64);
  const int64_t all_last = __shfl(incl, 63, 64);
  if (first >= 0 && prev < 0) rec[0] = base + first;
  if (lane == 0) {
    rec[1] = all_last;
    rec[2] = total;
    if (all_last < 0) rec[0] = -1;
  }
}

// Copy n elements from LDS (element e at s[a + e]) to global g[o0 + e], where
// a == o0 mod (4 / sizeof(T)): aligned 4-byte stores by the 64 lanes of a wave,
// element stores at the edges.
template <typename T>
__device__ __forceinline__ void copy_out_wave(const T *s, int a, T *__restrict__ g, int64_t o0, int n, int64_t cap) {
  constexpr int E = 4 / (int)sizeof(T);  // elements per word
  const int lane = threadIdx.x & 63;
  const int64_t w0 = o0 / E, w1 = (o0 + n + E - 1) / E;
  for (int64_t w = w0 + lane; w < w1; w += 64) {
    const int64_t e0 = w * E;
    if (e0 >= o0 && e0 + E <= o0 + n && e0 + E <= cap) {
      const int li = (int)(e0 - o0) + a;  // multiple of E
      *reinterpret_cast<uint32_t *>(g + e0) = *reinterpret_cast<const uint32_t *>(s + li);
    } else {
      for (int k = 0; k < E; ++k) {
        const int64_t e = e0 + k;
        if (e >= o0 && e < o0 + n && e < cap) g[e] = s[(int)(e - o0) + a];
      }
    }
  }
}

}  // namespace
}  // namespace hic
