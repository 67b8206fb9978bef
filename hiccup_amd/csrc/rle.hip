// rle.hip -- zig-zag / DC-DPCM / AC run-length front end of hiccup's JPEG codec
// and its inverse, on MI355X.
//
// Reference: codec.run_length_coding (codec.py:55-99), codec.decode_run_length
// (codec.py:102-113), codec.differential_coding (codec.py:47-52),
// utils.differences / invert_differences (utils.py:51-73), the AC-stream
// assembly of codec.jpeg_encode (codec.py:292-301: for every block in raster
// order, zigzag(block)[1:], concatenated over the whole channel) and its
// inverse in codec.jpeg_decode (codec.py:397-425).
//
// The reference RLE is ONE sequential scan over a channel's entire AC stream:
// runs cross block boundaries, a trailing zero run becomes the single EOB (0,0),
// and a run l >= max_len becomes l/max_len fillers (max_len-1, 0) + (l%max_len, v).
// Here it is a three-pass decoupled scan:
//   K1 (per tile of 256 blocks, one block per lane): first/last nonzero and the
//       symbol count of every nonzero whose predecessor is inside the tile;
//   K2 (one workgroup): exclusive max-scan of "last nonzero" and exclusive
//       sum-scan of per-tile symbol counts -> tile offsets; EOB; total count;
//   K3 (per tile): recompute, scan inside the tile, write symbols (SoA) and the
//       DC differences.  Long filler runs (a nonzero after many all-zero blocks)
//       are written cooperatively by the whole workgroup.
// Sharding: the same kernels take a carry (zeros preceding the shard since the
// last nonzero of earlier shards), the previous shard's last DC, and whether this
// shard closes the stream (EOB) -- see hic_rle_stitch.
#include <atomic>
#include <climits>

#include "rle_core.h"

namespace hic {
namespace {

constexpr int kTB = 256;  // blocks (= lanes) per tile

// Exclusive sum over the workgroup; returns the exclusive prefix, sets total.
template <typename T, int NT>
__device__ __forceinline__ T block_excl_sum(T v, T *s_buf, T &total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const T incl = wave_incl_sum(v);
  if (lane == 63) s_buf[wave] = incl;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wave) pre += s_buf[w];
    tot += s_buf[w];
  }
  __syncthreads();
  total = tot;
  return pre + incl - v;
}
// Exclusive max over the workgroup (identity `ident`); sets the overall max.
template <typename T, int NT>
__device__ __forceinline__ T block_excl_max(T v, T ident, T *s_buf, T &all) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const T incl = wave_incl_max(v);
  T excl = __shfl_up(incl, 1, 64);
  if (lane == 0) excl = ident;
  if (lane == 63) s_buf[wave] = incl;
  __syncthreads();
  T pre = ident, a = ident;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wave) pre = pre > s_buf[w] ? pre : s_buf[w];
    a = a > s_buf[w] ? a : s_buf[w];
  }
  __syncthreads();
  all = a;
  return excl > pre ? excl : pre;
}

// Element j (0 <= j < A) of block b lives at blocks[b*L + off + j]; its global
// stream position is b*A + j and only positions < n_ac exist.
struct StreamGeo {
  int L, off, A;
  int64_t n_ac;
};

template <typename T>
__device__ __forceinline__ void summarize(const T *__restrict__ blocks, int64_t b, const StreamGeo &g, int M,
                                          int &first, int &last, int &nsym_in) {
  first = -1;
  last = -1;
  nsym_in = 0;
  const T *blk = blocks + b * g.L + g.off;
  if (sizeof(T) == 2 && g.L == 64 && g.off == 1 && (b + 1) * g.A <= g.n_ac) {
    // hot path: one 128-byte zig-zag block held in registers
    const uint4 *q = reinterpret_cast<const uint4 *>(blocks + b * 64);
    uint32_t w[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 t = q[k];
      w[4 * k] = t.x; w[4 * k + 1] = t.y; w[4 * k + 2] = t.z; w[4 * k + 3] = t.w;
    }
#pragma unroll
    for (int j = 0; j < 63; ++j) {
      const int s = j + 1;
      const bool nz = ((w[s >> 1] >> (16 * (s & 1))) & 0xFFFFu) != 0;
      if (nz) {
        if (first < 0)
          first = j;
        else
          nsym_in += syms_for_run(j - last - 1, M);
        last = j;
      }
    }
  } else {
    const int64_t lim = g.n_ac - b * g.A;
    const int A = lim < g.A ? (int)(lim > 0 ? lim : 0) : g.A;
    for (int j = 0; j < A; ++j) {
      if (blk[j] != 0) {
        if (first < 0)
          first = j;
        else
          nsym_in += syms_for_run(j - last - 1, M);
        last = j;
      }
    }
  }
}

// K1: per-tile aggregates.  ws layout per tile: [0] first (global), [1] last
// (global), [2] symbols except the tile's first nonzero's.
template <typename T>
__global__ __launch_bounds__(kTB) void k_rle_tile(const T *__restrict__ blocks, int64_t nblk, StreamGeo g, int M,
                                                  int64_t *__restrict__ tiles) {
  __shared__ int64_t s_buf[8];
  const int64_t b = (int64_t)blockIdx.x * kTB + threadIdx.x;
  int first = -1, last = -1, nsym = 0;
  if (b < nblk) summarize(blocks, b, g, M, first, last, nsym);
  const int64_t base = b * g.A;
  const int64_t lastg = last >= 0 ? base + last : -1;
  int64_t all_last;
  const int64_t prev = block_excl_max<int64_t, kTB>(lastg, (int64_t)-1, s_buf, all_last);
  int64_t cnt = nsym;
  if (first >= 0 && prev >= 0) cnt += syms_for_run(base + first - prev - 1, M);
  int64_t total;
  block_excl_sum<int64_t, kTB>(cnt, s_buf, total);
  // the tile's first nonzero: the only lane with a nonzero and no predecessor
  if (first >= 0 && prev < 0) tiles[blockIdx.x * 3 + 0] = base + first;
  if (threadIdx.x == 0) {
    tiles[blockIdx.x * 3 + 1] = all_last;
    tiles[blockIdx.x * 3 + 2] = total;
    if (all_last < 0) tiles[blockIdx.x * 3 + 0] = -1;
  }
}

// K2: single workgroup of 1024 threads.  Produces per tile: [0] symbol offset,
// [1] global position of the last nonzero before the tile (virtual -1-carry if
// none).  Writes the EOB symbol and the count.
// Each thread folds kScanK consecutive tile records in registers, one
// workgroup-wide exclusive scan combines the per-thread aggregates, and each
// thread walks its tiles again to write their offsets.  The aggregate of a run
// of tiles is itself a tile record {first, last, count except the first
// nonzero's symbols}; combining A then B adds B's first-nonzero symbols, whose
// run starts after A's last nonzero.
constexpr int kScanT = 1024;
constexpr int kScanK = 8;  // tiles per thread per pass


struct Agg {
  int64_t first, last, cnt;
};
__device__ __forceinline__ Agg agg_combine(const Agg &A, const Agg &B, int M) {
  if (B.last < 0) return A;
  if (A.last < 0) return B;
  return Agg{A.first, B.last, A.cnt + B.cnt + syms_for_run(B.first - A.last - 1, M)};
}
__device__ __forceinline__ Agg agg_shfl_up(const Agg &a, int d) {
  return Agg{__shfl_up(a.first, d, 64), __shfl_up(a.last, d, 64), __shfl_up(a.cnt, d, 64)};
}

template <typename L_T, typename V_T>
__device__ __forceinline__ void scan_tiles(const int64_t *__restrict__ tiles, int64_t *__restrict__ offs,
                                                     int64_t ntiles, int64_t n_ac, int M,
                                                     const int64_t *__restrict__ stitch, L_T *__restrict__ sym_len,
                                                     V_T *__restrict__ sym_val, int64_t cap,
                                                     int64_t *__restrict__ d_count, Agg *s_wave_buf) {
  Agg *s_wave = s_wave_buf;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t carry = stitch ? stitch[0] : 0;
  const bool emit_eob = stitch ? stitch[1] != 0 : true;
  const int64_t p0 = -1 - carry;  // virtual last nonzero before the stream
  Agg run{-1, -1, 0};             // aggregate of all tiles of earlier passes
  for (int64_t c0 = 0; c0 < ntiles; c0 += (int64_t)kScanT * kScanK) {
    const int64_t t0 = c0 + (int64_t)threadIdx.x * kScanK;
    Agg rec[kScanK];
#pragma unroll
    for (int k = 0; k < kScanK; ++k) {
      const int64_t t = t0 + k;
      rec[k] = t < ntiles ? Agg{tiles[t * 3 + 0], tiles[t * 3 + 1], tiles[t * 3 + 2]} : Agg{-1, -1, 0};
    }
    Agg mine = rec[0];
#pragma unroll
    for (int k = 1; k < kScanK; ++k) mine = agg_combine(mine, rec[k], M);
    // workgroup-wide inclusive scan of the per-thread aggregates
    Agg incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const Agg o = agg_shfl_up(incl, d);
      if (lane >= d) incl = agg_combine(o, incl, M);
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    // wave 0 scans the 16 wave totals (exclusive) in place; lane 15 also forms the
    // aggregate of everything so far
    if (wave == 0) {
      constexpr int NW = kScanT / 64;
      Agg t = lane < NW ? s_wave[lane] : Agg{-1, -1, 0};
      Agg it = t;
#pragma unroll
      for (int d = 1; d < NW; d <<= 1) {
        const Agg o = agg_shfl_up(it, d);
        if (lane >= d) it = agg_combine(o, it, M);
      }
      Agg ex = agg_shfl_up(it, 1);
      if (lane == 0) ex = Agg{-1, -1, 0};
      if (lane < NW) s_wave[lane] = agg_combine(run, ex, M);
      if (lane == NW - 1) s_wave[NW] = agg_combine(run, it, M);
    }
    __syncthreads();
    Agg excl = agg_shfl_up(incl, 1);
    if (lane == 0) excl = Agg{-1, -1, 0};
    excl = agg_combine(s_wave[wave], excl, M);
    const Agg all = s_wave[kScanT / 64];
    __syncthreads();
    // state entering this thread's first tile
    int64_t prev = excl.last >= 0 ? excl.last : p0;
    int64_t off = excl.last >= 0 ? excl.cnt + syms_for_run(excl.first - p0 - 1, M) : 0;
#pragma unroll
    for (int k = 0; k < kScanK; ++k) {
      const int64_t t = t0 + k;
      if (t < ntiles) {
        offs[t * 2 + 0] = off;
        offs[t * 2 + 1] = prev;
        if (rec[k].last >= 0) {
          off += rec[k].cnt + syms_for_run(rec[k].first - prev - 1, M);
          prev = rec[k].last;
        }
      }
    }
    run = all;
  }
  if (threadIdx.x == 0) {
    const int64_t last = run.last >= 0 ? run.last : p0;
    const bool ends_nonzero = n_ac > 0 && last == n_ac - 1;
    int64_t total = run.last >= 0 ? run.cnt + syms_for_run(run.first - p0 - 1, M) : 0;
    if (emit_eob && !ends_nonzero) {
      if (total < cap) {
        sym_len[total] = 0;
        sym_val[total] = 0;
      }
      ++total;
    }
    *d_count = total <= cap ? total : -total;
  }
}

template <typename L_T, typename V_T>
__global__ __launch_bounds__(kScanT) void k_rle_scan(const int64_t *__restrict__ tiles, int64_t *__restrict__ offs,
                                                     int64_t ntiles, int64_t n_ac, int M,
                                                     const int64_t *__restrict__ stitch, L_T *__restrict__ sym_len,
                                                     V_T *__restrict__ sym_val, int64_t cap,
                                                     int64_t *__restrict__ d_count) {
  __shared__ Agg s_wave[kScanT / 64 + 1];
  scan_tiles<L_T, V_T>(tiles, offs, ntiles, n_ac, M, stitch, sym_len, sym_val, cap, d_count, s_wave);
}

// K3: emit symbols (+ DC differences when dc_diff != nullptr).
// Each lane writes its block's symbols into an LDS stage at the tile-relative
// offset, then the workgroup copies the tile's contiguous symbol range out with
// aligned 4-byte stores (partial edge words by element stores).  A tile whose
// symbols exceed the stage (a nonzero after >~1300 carried-in zeros) takes the
// direct path, with long filler runs written cooperatively.
constexpr int kStageSyms = kTB * 68;

template <typename L_T, typename V_T>
__device__ __forceinline__ void put_sym(bool staged, int64_t o, int64_t o_tile, int lo, int vo, uint8_t *s_len,
                                        V_T *s_val, L_T *__restrict__ sym_len, V_T *__restrict__ sym_val, int64_t cap,
                                        int len, int val) {
  if (staged) {
    const int r = (int)(o - o_tile);
    s_len[lo + r] = (uint8_t)len;
    s_val[vo + r] = (V_T)val;
  } else if (o < cap) {
    sym_len[o] = (L_T)len;
    sym_val[o] = (V_T)val;
  }
}

// Copy n elements from LDS (element e at s[a + e]) to global g[o0 + e], where
// a == o0 mod (4 / sizeof(T)): aligned 4-byte stores, element stores at the edges.
template <typename T>
__device__ __forceinline__ void copy_out(const T *s, int a, T *__restrict__ g, int64_t o0, int n, int64_t cap) {
  constexpr int E = 4 / (int)sizeof(T);  // elements per word
  const int64_t w0 = o0 / E, w1 = (o0 + n + E - 1) / E;
  for (int64_t w = w0 + threadIdx.x; w < w1; w += kTB) {
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

template <typename T, typename L_T, typename V_T>
__global__ __launch_bounds__(kTB) void k_rle_emit(const T *__restrict__ blocks, int64_t nblk, StreamGeo g, int M,
                                                  const int64_t *__restrict__ offs, const int64_t *__restrict__ stitch,
                                                  int32_t *__restrict__ dc_diff, L_T *__restrict__ sym_len,
                                                  V_T *__restrict__ sym_val, int64_t cap) {
  __shared__ int64_t s_buf[8];
  __shared__ int64_t s_fill_start[kTB];
  __shared__ int64_t s_fill_count[kTB];
  __shared__ int s_nfill;
  __shared__ uint8_t s_len[kStageSyms + 4];
  __shared__ V_T s_val[kStageSyms + 4];
  if (threadIdx.x == 0) s_nfill = 0;
  const int64_t b = (int64_t)blockIdx.x * kTB + threadIdx.x;
  int first = -1, last = -1, nsym = 0;
  if (b < nblk) summarize(blocks, b, g, M, first, last, nsym);
  const int64_t base = b * g.A;
  const int64_t lastg = last >= 0 ? base + last : -1;
  int64_t all_last;
  int64_t prev = block_excl_max<int64_t, kTB>(lastg, (int64_t)-1, s_buf, all_last);
  if (prev < 0) prev = offs[blockIdx.x * 2 + 1];
  const int64_t cnt = nsym + (first >= 0 ? syms_for_run(base + first - prev - 1, M) : 0);
  int64_t total;
  const int64_t o_tile = offs[blockIdx.x * 2 + 0];
  int64_t o = o_tile + block_excl_sum<int64_t, kTB>(cnt, s_buf, total);
  const bool staged = total <= kStageSyms;  // uniform across the workgroup
  const int lo = (int)(o_tile & 3), vo = (int)(o_tile & ((4 / (int)sizeof(V_T)) - 1));

  if (b < nblk) {
    if (dc_diff) {  // codec.differential_coding over raster-ordered blocks
      const int dc = (int)blocks[b * g.L];
      if (b > 0)
        dc_diff[b] = dc - (int)blocks[(b - 1) * g.L];
      else
        dc_diff[b] = (stitch && stitch[2]) ? dc - (int)stitch[3] : dc;
    }
    if (first >= 0) {
      const T *blk = blocks + b * g.L + g.off;
      int64_t p = prev;
      for (int j = first; j <= last; ++j) {
        const int v = (int)blk[j];
        if (v == 0) continue;
        int64_t run = base + j - p - 1;
        if (M > 0) {
          const int64_t nf = div_run(run, M);
          if (!staged && nf > 32) {
            // long carried-in run: the whole workgroup writes the fillers
            const int slot = atomicAdd(&s_nfill, 1);
            s_fill_start[slot] = o;
            s_fill_count[slot] = nf;
            o += nf;
          } else {
            for (int64_t k = 0; k < nf; ++k, ++o)
              put_sym<L_T, V_T>(staged, o, o_tile, lo, vo, s_len, s_val, sym_len, sym_val, cap, M - 1, 0);
          }
          run -= nf * M;
        }
        put_sym<L_T, V_T>(staged, o, o_tile, lo, vo, s_len, s_val, sym_len, sym_val, cap, (int)run, v);
        ++o;
        p = base + j;
      }
    }
  }
  __syncthreads();
  if (staged) {
    if (sizeof(L_T) == 1) {
      copy_out<uint8_t>(s_len, lo, reinterpret_cast<uint8_t *>(sym_len), o_tile, (int)total, cap);
    } else {
      for (int k = threadIdx.x; k < (int)total; k += kTB)
        if (o_tile + k < cap) sym_len[o_tile + k] = (L_T)s_len[lo + k];
    }
    copy_out<V_T>(s_val, vo, sym_val, o_tile, (int)total, cap);
  } else {
    const int nfill = s_nfill;
    for (int f = 0; f < nfill; ++f) {
      const int64_t s0 = s_fill_start[f], nf = s_fill_count[f];
      for (int64_t k = threadIdx.x; k < nf; k += kTB)
        if (s0 + k < cap) {
          sym_len[s0 + k] = (L_T)(M - 1);
          sym_val[s0 + k] = 0;
        }
    }
  }
}

// ---------------------------------------------------------------------------
// Hot path (rle_core.h geometry): one tile per wave, no workgroup barriers.
template <int MF>
__global__ __launch_bounds__(256) void k_rle_tile16(const int16_t *__restrict__ blocks, int64_t nblk, int M,
                                                    int64_t *__restrict__ tiles) {
  const int64_t tw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = tw * kWT + (threadIdx.x & 63);
  uint32_t w[32];
  if (b < nblk) load_block16(blocks, b, w);
  tile_record16<MF>(w, b < nblk, b, M, tiles + tw * 3);
}

// Symbols of one tile.  Each lane writes its block's symbols into the wave's LDS
// stage at their tile-relative positions, then the wave copies the contiguous
// range out with aligned 4-byte stores.  A tile with more symbols than the stage
// (a nonzero after >~960 carried-in zeros) writes directly, its long filler runs
// by the whole wave.
constexpr int kWSyms = 4096;  // staged symbols per wave (a dense tile has <= 64 * 63)

template <int MF, bool NT>
// w: this lane's block in registers; blk: the same block in global memory, read
// for lane-varying coefficient indices (keeps w out of scratch).
__device__ __forceinline__ void emit_tile16(const uint32_t (&w)[32], const int16_t *__restrict__ blk, bool valid,
                                            int64_t b, int64_t nblk, int M, int64_t o_tile, int64_t prev_tile,
                                            uint8_t *s_len, int16_t *s_val, uint8_t *__restrict__ sym_len,
                                            int16_t *__restrict__ sym_val, int64_t cap) {
  const int lane = threadIdx.x & 63;
  int first = -1, last = -1, nsym = 0;
  uint64_t ac = 0;
  if (valid) summarize16<MF>(w, M, first, last, nsym, &ac);
  const int64_t base = b * 63;
  // in-tile positions (lane * 63 + j) and counts fit int32: DPP scans
  const int incl = wave_incl_max_i32(last >= 0 ? lane * 63 + last : -1);
  const int prevr = wave_shr1_i32(-1, incl);
  // no nonzero before it inside the tile: the tile's carried-in predecessor
  const int64_t prev = prevr >= 0 ? (b - lane) * 63 + prevr : prev_tile;
  const int64_t run0 = base + first - prev - 1;  // carried run before the first nonzero
  const int cnt = nsym + (first >= 0 ? syms_for_run(run0, M) : 0);
  const int incl_cnt = wave_incl_sum_i32(cnt);
  const int total = wave_last_i32(incl_cnt);
  const int64_t o_thr = o_tile + incl_cnt - cnt;
  const bool staged = total <= kWSyms;  // uniform across the wave
  // stage offsets congruent to the output position mod 16 bytes (16-byte copy-out)
  const int lo = (int)(o_tile & 15), vo = (int)(o_tile & 7);
  int64_t nf0 = 0;  // fillers of a long carried run written by the whole wave (unstaged)
  const bool dense = nsym == __builtin_popcountll(ac) - 1;  // no run >= max_len inside the block
  if (first >= 0) {
    int64_t o = o_thr;
    const int64_t nf = div_run(run0, M);
    const int rem = (int)(run0 - nf * M);
    if (staged) {
      // the carried run's fillers, then (dense case) every nonzero from the first on
      // in one branch-free pass over the block's registers -- no reload of the
      // first value from memory, so nothing here waits on the next tile's prefetch
      int r = (int)(o - o_tile);
      for (int64_t k = 0; k < nf; ++k, ++r) {
        s_len[lo + r] = (uint8_t)(M - 1);
        s_val[vo + r] = 0;
      }
      o += nf;
      if (!dense) {
        s_len[lo + r] = (uint8_t)rem;
        s_val[vo + r] = blk[1 + first];
        ++o;
      }
    } else {
      nf0 = nf;
      if (o + nf < cap) {
        sym_len[o + nf] = (uint8_t)rem;
        sym_val[o + nf] = blk[1 + first];
      }
      o += nf + 1;
    }
    if (staged && dense) {
      // one symbol per nonzero from the first, branch-free: a zero coefficient
      // writes to the stage's dummy slot and does not advance r.  The first
      // nonzero needs no case of its own: with pl = first - 1 - rem its run
      // j - pl - 1 is the carried run's remainder, and no coefficient before it
      // is nonzero.  One index serves both arrays (val index = len index + dv), so
      // a coefficient costs a compare, a subtract, two selects, an address and a
      // carry-add.
      typedef __attribute__((address_space(3))) uint8_t lds_u8;
      typedef __attribute__((address_space(3))) int16_t lds_i16;
      // LDS byte addresses: len slot = la, val slot = 2 la + vshift
      const uint32_t lbase = (uint32_t)(uintptr_t)(lds_u8 *)s_len;
      const uint32_t vshift = (uint32_t)(uintptr_t)(lds_i16 *)s_val + 2u * (uint32_t)(vo - lo) - 2u * lbase;
      // dummy slot past every real one: len kWSyms + 16 > lo + kWSyms - 1, val
      // kWSyms + 16 + vo - lo > vo + kWSyms - 1 (lo, vo < 16), both inside the stage
      const uint32_t ldummy = lbase + kWSyms + 16;
      uint32_t la = lbase + (uint32_t)((int)(o - o_tile) + lo);  // next symbol's len slot
      int pl = first - 1 - rem;
#pragma unroll
      for (int j = 0; j < 63; ++j) {
        const int v = zz_ac(w, j);
        const bool nz = v != 0;
        const uint32_t a = nz ? la : ldummy;
        *(lds_u8 *)(uintptr_t)a = (uint8_t)(j - pl - 1);
        uint32_t va;  // 2 a + vshift in one instruction (the compiler splits it in two)
        asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(va) : "v"(a), "v"(vshift));
        *(lds_i16 *)(uintptr_t)va = (int16_t)v;
        la += nz ? 1u : 0u;
        pl = nz ? j : pl;
      }
    } else if (staged) {
      int r = (int)(o - o_tile);  // tile-relative output position
      int pl = first;
      for (uint64_t m = ac & (ac - 1); m; m &= m - 1) {  // nonzeros after the first
        const int j = __builtin_ctzll(m);
        const int v = blk[1 + j];
        int run = j - pl - 1;
        const int nf = div_m<MF>(run, M);
        for (int f = 0; f < nf; ++f, ++r) {
          s_len[lo + r] = (uint8_t)(M - 1);
          s_val[vo + r] = 0;
        }
        run -= nf * M;
        s_len[lo + r] = (uint8_t)run;
        s_val[vo + r] = (int16_t)v;
        ++r;
        pl = j;
      }
    } else {
      int pl = first;
      for (uint64_t m = ac & (ac - 1); m; m &= m - 1) {
        const int j = __builtin_ctzll(m);
        const int v = blk[1 + j];
        int run = j - pl - 1;
        const int nf = run / M;
        for (int k = 0; k < nf; ++k, ++o)
          if (o < cap) {
            sym_len[o] = (uint8_t)(M - 1);
            sym_val[o] = 0;
          }
        run -= nf * M;
        if (o < cap) {
          sym_len[o] = (uint8_t)run;
          sym_val[o] = (int16_t)v;
        }
        ++o;
        pl = j;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  // (no vmcnt drain here: the copy-out reads only this wave's LDS stage, so the
  // next tile's prefetch stays in flight across it)
  if (staged) {
    copy_out_wave16<uint8_t, NT>(s_len, lo, sym_len, o_tile, (int)total, cap);
    copy_out_wave16<int16_t, NT>(s_val, vo, sym_val, o_tile, (int)total, cap);
  } else {
    // long carried runs: the whole wave writes each lane's fillers
    uint64_t m = __ballot(nf0 > 0);
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      const int64_t s0 = __shfl(o_thr, l, 64), nf = __shfl(nf0, l, 64);
      for (int64_t k = lane; k < nf; k += 64)
        if (s0 + k < cap) {
          sym_len[s0 + k] = (uint8_t)(M - 1);
          sym_val[s0 + k] = 0;
        }
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// Batched hot path: the scan and the emit of up to kMaxJobs channels (e.g. Y, Cr,
// Cb of one image) in one launch each.  The scan runs one workgroup per channel;
// the emit's persistent waves walk the concatenated tile space of all channels.
constexpr int kMaxJobs = 4;
struct RleJob16 {
  const int16_t *blocks;
  int64_t nblk;
  const int64_t *stitch;
  int32_t *dc_diff;
  uint8_t *sym_len;
  int16_t *sym_val;
  int64_t cap;
  int64_t *d_count;
  int64_t *ws;     // tile records [3 * nrec] then offsets [2 * nrec]
  int64_t ntiles;
  int64_t tile0;   // first global tile index of this job
  int64_t nrec;    // records: one per 64-block tile, or one per 32-block half tile (rshift 1)
  int rshift;      // log2(records per 64-block tile)
  // row segments (hic_rle_encode_i16_rows_batch): rows of rowb blocks, each cut into
  // tiles of 64 blocks from the row's start, the last one shorter; 0 = plain tiles
  int64_t rowb;
  int64_t tpr, rpr;  // tiles and records per row
  int64_t wsb;       // workspace bytes (0: not checked; a rows job must give it)
  int64_t *index;    // optional tile index the emit writes (hic_rle_tile_index_i16's)
  // slot layout (slots.h; the close k_rle_scan16b<true> and the compaction)
  uint8_t *slot_len;
  int16_t *slot_val;
  int32_t *sidx;     // 4 int32 per record {n, P, pdc, nfill}
  int32_t *rdc;      // the records' last DCs (in the workspace)
  int64_t bpr;       // blocks per record (64 or 32); capacity 63 * bpr
};
struct RleJobs16 {
  RleJob16 j[kMaxJobs];
  int n;
  int M;
  int64_t total_tiles;
  uint32_t epoch;  // the scan launch's hand-off epoch (its failure granule's tag)
};

// Multi-workgroup scan for the batched hot path: each channel's tiles are cut
// into partitions of kScan16T tiles, one workgroup per partition (all resident at
// once: ~100 workgroups at 8K).  Partitions of 256 (4-wave workgroups): beside the
// other stream's encoder (2 waves per SIMD of 234 VGPRs) a 1024-thread workgroup
// waits for a whole CU's 16 wave slots to drain.  A partition reduces its tiles, publishes the
// aggregate as three tagged 8-byte granules {value, epoch tag} (sc1 stores:
// MI355X_MICROARCH.md, granule hand-off; no fences), polls the granules of every
// earlier partition of its channel (sc1 loads) and folds them, then scans its
// own tiles (one tile per thread, coalesced record loads and offset stores).
// The epoch is unique per launch, so stale granules never match; a bounded spin
// reports failure through d_count instead of hanging.
__device__ __forceinline__ void put_granule(uint64_t *g, int64_t v, uint32_t tag) {
  __hip_atomic_store(g, (uint64_t)(uint32_t)(int32_t)v | ((uint64_t)tag << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool get_granule(const uint64_t *g, uint32_t tag, int64_t &v) {
  const uint64_t x = __hip_atomic_load(const_cast<uint64_t *>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v = (int64_t)(int32_t)(uint32_t)x;
  return (uint32_t)(x >> 32) == tag;
}

#ifndef HIC_SCAN16_T
#define HIC_SCAN16_T 256
#endif
constexpr int kScan16T = HIC_SCAN16_T;
static_assert(kScan16T % 64 == 0 && kScan16T <= 1024, "scan partition: whole waves");
// workspace words of a job with nrec records: the records (3) and their offsets (2),
// 3 hand-off granules per scan partition and the failure granule, + slack
inline int64_t rle_ws_words(int64_t nrec) {
  const int64_t n = nrec > 0 ? nrec : 1;
  return 5 * n + 3 * ((n + kScan16T - 1) / kScan16T) + 8;
}
// SLOTS (the slot layout's close, slots.h): each record's first symbol length, its
// first block's DC difference, and its index entry, from the same exclusive scan.
template <bool SLOTS>
__global__ __launch_bounds__(kScan16T) void k_rle_scan16b(RleJobs16 jobs, uint32_t epoch) {
  __shared__ Agg s_wave[kScan16T / 64 + 1];
  __shared__ Agg s_pre;
  __shared__ int s_fail;
  // workgroup -> (job, partition)
  int jb = 0;
  int64_t p = blockIdx.x;
  while (jb + 1 < jobs.n && p >= (jobs.j[jb].nrec + kScan16T - 1) / kScan16T) {
    p -= (jobs.j[jb].nrec + kScan16T - 1) / kScan16T;
    ++jb;
  }
  const RleJob16 &J = jobs.j[jb];
  const int M = jobs.M;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nt = J.nrec, np = (nt + kScan16T - 1) / kScan16T;
  const int64_t *tiles = J.ws;
  int64_t *offs = J.ws + 3 * nt;
  uint64_t *gran = reinterpret_cast<uint64_t *>(J.ws + 5 * nt);  // 3 per partition
  const uint32_t tag = (epoch << 2) | 1u;
  const int64_t t = p * kScan16T + threadIdx.x;
  const Agg rec = t < nt ? Agg{tiles[t * 3 + 0], tiles[t * 3 + 1], tiles[t * 3 + 2]} : Agg{-1, -1, 0};
  // workgroup inclusive scan of the partition's tile records
  Agg incl = rec;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const Agg o = agg_shfl_up(incl, d);
    if (lane >= d) incl = agg_combine(o, incl, M);
  }
  if (lane == 63) s_wave[wave] = incl;
  if (threadIdx.x == 0) s_fail = 0;
  __syncthreads();
  if (wave == 0) {
    constexpr int NW = kScan16T / 64;
    Agg it = lane < NW ? s_wave[lane] : Agg{-1, -1, 0};
#pragma unroll
    for (int d = 1; d < NW; d <<= 1) {
      const Agg o = agg_shfl_up(it, d);
      if (lane >= d) it = agg_combine(o, it, M);
    }
    Agg ex = agg_shfl_up(it, 1);
    if (lane == 0) ex = Agg{-1, -1, 0};
    if (lane < NW) s_wave[lane] = ex;
    if (lane == NW - 1) {
      s_wave[NW] = it;  // the partition's aggregate: publish it
      put_granule(gran + 3 * p + 0, it.first, tag);
      put_granule(gran + 3 * p + 1, it.last, tag);
      put_granule(gran + 3 * p + 2, it.cnt, tag);
    }
    // fold the aggregates of the earlier partitions (lane q < p polls partition q)
    Agg pre{-1, -1, 0};
    for (int64_t q0 = 0; q0 < p; q0 += 64) {
      const int64_t q = q0 + lane;
      Agg a{-1, -1, 0};
      if (q < p) {
        bool ok = false;
        for (int spin = 0; spin < (1 << 22) && !ok; ++spin) {
          int64_t f, l, c;
          ok = (int)get_granule(gran + 3 * q + 0, tag, f) & (int)get_granule(gran + 3 * q + 1, tag, l) &
               get_granule(gran + 3 * q + 2, tag, c);
          if (ok) a = Agg{f, l, c};
          else __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) s_fail = 1;
      }
      // the window's ordered total by a wave scan (agg_combine is associative):
      // log2(64) steps instead of one serial combine per earlier partition (the
      // 16K image has 512 partitions per channel, and its last ones folded them all)
      Agg wi = a;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const Agg o = agg_shfl_up(wi, d);
        if (lane >= d) wi = agg_combine(o, wi, M);
      }
      const int lastl = (int)(p - q0 < 64 ? p - q0 - 1 : 63);
      pre = agg_combine(pre, Agg{__shfl(wi.first, lastl, 64), __shfl(wi.last, lastl, 64), __shfl(wi.cnt, lastl, 64)}, M);
    }
    if (lane == 0) s_pre = pre;
  }
  __syncthreads();
  const int64_t carry = J.stitch ? J.stitch[0] : 0;
  const int64_t p0 = -1 - carry;  // virtual last nonzero before the stream
  Agg excl = agg_shfl_up(incl, 1);
  if (lane == 0) excl = Agg{-1, -1, 0};
  excl = agg_combine(agg_combine(s_pre, s_wave[wave], M), excl, M);
  if (t < nt) {
    offs[t * 2 + 0] = excl.last >= 0 ? excl.cnt + syms_for_run(excl.first - p0 - 1, M) : 0;
    offs[t * 2 + 1] = excl.last >= 0 ? excl.last : p0;
  }
  if (SLOTS && t < nt) {
    // the record's first nonzero continues the zero run since the previous record's
    // last nonzero: its fillers and its first symbol's length (written as 0 by the
    // fused kernel); P: the record-relative position the run's remainder starts after
    const int64_t prv = excl.last >= 0 ? excl.last : p0, capr = 63 * J.bpr;
    int n = 0, P = 0, nf = 0;
    if (rec.first >= 0) {
      const int64_t run = rec.first - prv - 1, f = div_run(run, M);
      const int len0 = (int)(run - f * M);
      nf = (int)f;
      n = (int)rec.cnt + 1;
      P = (int)(rec.first - t * capr) - len0;
      J.slot_len[t * capr] = (uint8_t)len0;
    }
    // codec.differential_coding across the record boundary
    const int pdc = t > 0 ? J.rdc[t - 1] : 0;
    if (t > 0) J.dc_diff[t * J.bpr] -= pdc;
    *reinterpret_cast<int4 *>(J.sidx + 4 * t) = make_int4(n, P, pdc, nf);
  }
  if (p == np - 1 && threadIdx.x == 0) {  // the channel's last partition closes the stream
    const Agg all = agg_combine(s_pre, s_wave[kScan16T / 64], M);
    const int64_t last = all.last >= 0 ? all.last : p0;
    const int64_t n_ac = J.nblk * 63;
    const bool emit_eob = J.stitch ? J.stitch[1] != 0 : true;
    int64_t total = all.last >= 0 ? all.cnt + syms_for_run(all.first - p0 - 1, M) : 0;
    if (emit_eob && !(n_ac > 0 && last == n_ac - 1)) {
      if (total < J.cap) {
        J.sym_len[total] = 0;
        J.sym_val[total] = 0;
      }
      ++total;
    }
    *J.d_count = total <= J.cap ? total : -total;
  }
  // a hand-off that timed out is reported, not waited for: a tagged failure granule
  // after the partitions' ones, folded into *d_count by the emit (which runs after
  // every partition's write, so the report cannot be overwritten by a total)
  if (s_fail && threadIdx.x == 0) put_granule(gran + 3 * np, 1, tag);
}

template <int MF, bool NT>
__global__ __launch_bounds__(256) void k_rle_emit16b(RleJobs16 jobs) {
  // per wave: kWSyms symbols + 16-byte alignment slack + the dummy slot
  __shared__ __attribute__((aligned(16))) uint8_t s_len_all[4][kWSyms + 32];
  __shared__ __attribute__((aligned(16))) int16_t s_val_all[4][kWSyms + 32];
  // wv (and the tile / job indices derived from it) wave-uniform in SGPRs: the jobs'
  // fields are then scalar loads from the kernel arguments, not per-lane loads of a
  // dynamically indexed argument copy, each followed by a vmcnt(0) that also drained
  // the next tile's prefetch and this tile's symbol stores
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int M = jobs.M;
  if (blockIdx.x == 0 && threadIdx.x < jobs.n) {  // the scan's failure report (sticky)
    const RleJob16 &J = jobs.j[threadIdx.x];
    const int64_t np = (J.nrec + kScan16T - 1) / kScan16T;
    int64_t f;
    if (get_granule(reinterpret_cast<const uint64_t *>(J.ws + 5 * J.nrec) + 3 * np, (jobs.epoch << 2) | 1u, f))
      *J.d_count = HIC_COUNT_SCAN_TIMEOUT;
  }
  int64_t g = (int64_t)blockIdx.x * 4 + wv;
  if (g >= jobs.total_tiles) return;  // wave-uniform
  struct Next {
    uint32_t w[32];
    int64_t off, prev;
    int pdc;
  };
  auto job_of = [&](int64_t gt) {
    int k = 0;
    while (k + 1 < jobs.n && gt >= jobs.j[k + 1].tile0) ++k;
    return __builtin_amdgcn_readfirstlane(k);
  };
  // tile t's first block, its block count and its first record
  auto geo = [&](const RleJob16 &J, int64_t t, int64_t &b0, int64_t &bend, int64_t &r0) {
    if (J.rowb > 0) {
      const int64_t row = (int)t / (int)J.tpr, j = t - row * J.tpr;  // tile counts < 2^31
      b0 = row * J.rowb + j * kWT;
      bend = row * J.rowb + (j * kWT + kWT < J.rowb ? j * kWT + kWT : J.rowb);
      r0 = row * J.rpr + (j << J.rshift);
    } else {
      b0 = t * kWT;
      bend = b0 + kWT < J.nblk ? b0 + kWT : J.nblk;
      r0 = t << J.rshift;
    }
  };
  auto fetch = [&](int64_t gt, Next &n) {
    const RleJob16 &J = jobs.j[job_of(gt)];
    const int64_t t = gt - J.tile0;
    int64_t b0, bend, r0;
    geo(J, t, b0, bend, r0);
    const int64_t b = b0 + lane;
    // coalesced: 16-B chunk c = 64 k + lane of the tile (block c / 8, part c % 8)
    // into w[4k .. 4k + 3]; transposed to one block per lane through LDS (to_lanes)
    {
      const uint4 *q = reinterpret_cast<const uint4 *>(J.blocks + b0 * 64);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool ok = b0 + 8 * k + (lane >> 3) < bend;
        const uint4 v = ok ? q[64 * k + lane] : make_uint4(0, 0, 0, 0);
        n.w[4 * k] = v.x; n.w[4 * k + 1] = v.y; n.w[4 * k + 2] = v.z; n.w[4 * k + 3] = v.w;
      }
    }
    // the tile's first record (a 64-block tile may carry two 32-block records)
    const int64_t *offs = J.ws + 3 * J.nrec;
    n.off = offs[r0 * 2 + 0];
    n.prev = offs[r0 * 2 + 1];
    n.pdc = (lane == 0 && b > 0 && b <= J.nblk) ? (int)J.blocks[(b - 1) * 64] : 0;
  };
  Next cur;
  fetch(g, cur);
  for (;;) {
    const int64_t gn = g + nwaves;
    Next nxt;
    if (gn < jobs.total_tiles) fetch(gn, nxt);
    const RleJob16 &J = jobs.j[job_of(g)];
    int64_t b0, bend, r0;
    geo(J, g - J.tile0, b0, bend, r0);
    // the tile index (hic_rle_tile_index_i16's words, from the values fetched for
    // this tile: its first record's offsets, the DC of the block before it)
    if (J.index && lane == 0) {
      int64_t *ix = J.index + 3 * (g - J.tile0);
      ix[0] = cur.off;
      ix[1] = cur.prev;
      ix[2] = cur.pdc;
    }
    const int64_t b = b0 + lane;
    const bool valid = b < bend;
    {
      // transpose through the wave's symbol-value stage (free until this tile's
      // emit): chunk (block bb, part p) at 16-B slot 8 bb + (p ^ (bb & 7)) -- the
      // stores are 1 KiB contiguous, the loads (block = lane) hit 8 distinct
      // 16-B bank groups per 8 lanes
      uint4 *sx = reinterpret_cast<uint4 *>(s_val_all[wv]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = 64 * k + lane, bb = c >> 3, pp = c & 7;
        sx[8 * bb + (pp ^ (bb & 7))] = make_uint4(cur.w[4 * k], cur.w[4 * k + 1], cur.w[4 * k + 2], cur.w[4 * k + 3]);
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint4 v = sx[8 * lane + (k ^ (lane & 7))];
        cur.w[4 * k] = v.x; cur.w[4 * k + 1] = v.y; cur.w[4 * k + 2] = v.z; cur.w[4 * k + 3] = v.w;
      }
      __builtin_amdgcn_wave_barrier();
    }
    // DC differences: the previous block's DC comes from the neighbouring lane
    const int dc = (int)(int16_t)(cur.w[0] & 0xFFFFu);
    int pdc = __shfl_up(dc, 1, 64);
    if (lane == 0) pdc = cur.pdc;
    if (valid) {
      if (b > 0)
        J.dc_diff[b] = dc - pdc;
      else
        J.dc_diff[b] = (J.stitch && J.stitch[2]) ? dc - (int)J.stitch[3] : dc;
    }
    emit_tile16<MF, NT>(cur.w, J.blocks + (valid ? b : 0) * 64, valid, b, J.nblk, M, cur.off, cur.prev,
                    s_len_all[wv], s_val_all[wv], J.sym_len, J.sym_val, J.cap);
    if (gn >= jobs.total_tiles) break;
    g = gn;
    cur = nxt;
  }
}

// The slot layout's closing step has no emit to fold a timed-out scan hand-off
// into the count (k_rle_emit16b's prologue): one small launch after the close does.
__global__ void k_rle_scan_fold(RleJobs16 jobs) {
  if (threadIdx.x < jobs.n) {
    const RleJob16 &J = jobs.j[threadIdx.x];
    const int64_t np = (J.nrec + kScan16T - 1) / kScan16T;
    int64_t f;
    if (get_granule(reinterpret_cast<const uint64_t *>(J.ws + 5 * J.nrec) + 3 * np, (jobs.epoch << 2) | 1u, f))
      *J.d_count = HIC_COUNT_SCAN_TIMEOUT;
  }
}

// The contiguous stream of slot-layout channels (hic_rle_slots_compact): one wave per
// record writes its nfill fillers and copies its slot's n symbols to the record's
// stream offset (the scan's offs).  Records of all jobs in one grid (tile0: a job's
// first global record).
__global__ __launch_bounds__(256) void k_rle_slots_compact(RleJobs16 jobs) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t g = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); g < jobs.total_tiles;
       g += nw) {
    int k = 0;
    while (k + 1 < jobs.n && g >= jobs.j[k + 1].tile0) ++k;
    const RleJob16 &J = jobs.j[k];
    const int64_t r = g - J.tile0, capr = 63 * J.bpr;
    const int64_t off = J.ws[3 * J.nrec + 2 * r];
    const int4 ix = *reinterpret_cast<const int4 *>(J.sidx + 4 * r);
    const int n = ix.x, nf = ix.w;
    for (int64_t i = lane; i < nf; i += 64)
      if (off + i < J.cap) {
        J.sym_len[off + i] = (uint8_t)(jobs.M - 1);
        J.sym_val[off + i] = 0;
      }
    const int64_t o = off + nf;
    for (int i = lane; i < n; i += 64)
      if (o + i < J.cap) {
        J.sym_len[o + i] = J.slot_len[r * capr + i];
        J.sym_val[o + i] = J.slot_val[r * capr + i];
      }
  }
}

// Shard summary: {trailing_zeros, has_nonzero, first_dc, last_dc}
template <typename T>
__global__ void k_rle_summary(const T *__restrict__ blocks, int64_t nblk, StreamGeo g,
                              const int64_t *__restrict__ tiles, int64_t ntiles, int64_t *__restrict__ out) {
  __shared__ int64_t s_buf[8];
  int64_t m = -1;
  for (int64_t t = threadIdx.x; t < ntiles; t += kTB) {
    const int64_t v = tiles[t * 3 + 1];
    m = v > m ? v : m;
  }
  int64_t all;
  block_excl_max<int64_t, kTB>(m, (int64_t)-1, s_buf, all);
  if (threadIdx.x == 0) {
    out[0] = g.n_ac - 1 - all;  // == n_ac when there is no nonzero
    out[1] = all >= 0 ? 1 : 0;
    out[2] = nblk > 0 ? (int64_t)blocks[0] : 0;
    out[3] = nblk > 0 ? (int64_t)blocks[(nblk - 1) * g.L] : 0;
  }
}

__global__ void k_rle_stitch(const int64_t *__restrict__ all, int world, int rank, int stride,
                             int64_t *__restrict__ st) {
  if (threadIdx.x != 0) return;
  int64_t carry = 0;
  for (int r = rank - 1; r >= 0; --r) {
    carry += all[(int64_t)r * stride + 0];
    if (all[(int64_t)r * stride + 1]) break;
  }
  st[0] = carry;
  st[1] = rank == world - 1 ? 1 : 0;
  st[2] = rank > 0 ? 1 : 0;
  st[3] = rank > 0 ? all[(int64_t)(rank - 1) * stride + 3] : 0;
}

// ---------------------------------------------------------------------------
// Decode: symbols -> zig-zag blocks
constexpr int kSPT = 8;                // symbols per thread
constexpr int kTS = kTB * kSPT;        // symbols per tile

template <typename L_T>
__global__ __launch_bounds__(kTB) void k_rld_tile(const L_T *__restrict__ sym_len, int64_t nsym,
                                                  int64_t *__restrict__ tile_sum) {
  __shared__ int64_t s_buf[8];
  const int64_t s0 = (int64_t)blockIdx.x * kTS + (int64_t)threadIdx.x * kSPT;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < kSPT; ++k)
    if (s0 + k < nsym) acc += (int64_t)sym_len[s0 + k] + 1;
  int64_t total;
  block_excl_sum<int64_t, kTB>(acc, s_buf, total);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// In-place exclusive scan of n int64 values by one workgroup; returns total in *out_total.
__global__ __launch_bounds__(kScanT) void k_scan_inplace(int64_t *__restrict__ v, int64_t n,
                                                         int64_t *__restrict__ out_total) {
  // kScanK consecutive values per thread per pass: one workgroup-wide scan per
  // kScanT * kScanK values
  __shared__ int64_t s_buf[32];
  int64_t run = 0;
  for (int64_t c0 = 0; c0 < n; c0 += (int64_t)kScanT * kScanK) {
    const int64_t i0 = c0 + (int64_t)threadIdx.x * kScanK;
    int64_t x[kScanK], sum = 0;
#pragma unroll
    for (int k = 0; k < kScanK; ++k) {
      x[k] = i0 + k < n ? v[i0 + k] : 0;
      sum += x[k];
    }
    int64_t tot;
    int64_t e = run + block_excl_sum<int64_t, kScanT>(sum, s_buf, tot);
#pragma unroll
    for (int k = 0; k < kScanK; ++k) {
      if (i0 + k < n) v[i0 + k] = e;
      e += x[k];
    }
    run += tot;
  }
  if (threadIdx.x == 0) *out_total = run;
}

// Multi-workgroup form of k_scan_inplace for long sequences (a 16K luma plane has
// ~65k symbol tiles, 8 serial passes of the one-workgroup scan, ~56 us): one
// workgroup per kScanT * kScanK chunk sums its chunk into part[chunk]; part is
// scanned by k_scan_inplace; each chunk is then scanned from its offset.
__global__ __launch_bounds__(kScanT) void k_scan_chunk_sum(const int64_t *__restrict__ v, int64_t n,
                                                           int64_t *__restrict__ part) {
  __shared__ int64_t s_buf[32];
  const int64_t i0 = (int64_t)blockIdx.x * kScanT * kScanK + (int64_t)threadIdx.x * kScanK;
  int64_t sum = 0;
#pragma unroll
  for (int k = 0; k < kScanK; ++k) sum += i0 + k < n ? v[i0 + k] : 0;
  int64_t tot;
  block_excl_sum<int64_t, kScanT>(sum, s_buf, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanT) void k_scan_chunk_apply(int64_t *__restrict__ v, int64_t n,
                                                             const int64_t *__restrict__ part) {
  __shared__ int64_t s_buf[32];
  const int64_t i0 = (int64_t)blockIdx.x * kScanT * kScanK + (int64_t)threadIdx.x * kScanK;
  int64_t x[kScanK], sum = 0;
#pragma unroll
  for (int k = 0; k < kScanK; ++k) {
    x[k] = i0 + k < n ? v[i0 + k] : 0;
    sum += x[k];
  }
  int64_t tot;
  int64_t e = part[blockIdx.x] + block_excl_sum<int64_t, kScanT>(sum, s_buf, tot);
#pragma unroll
  for (int k = 0; k < kScanK; ++k) {
    if (i0 + k < n) v[i0 + k] = e;
    e += x[k];
  }
}

// Exclusive scan of v[0, n) in place, total to *out_total.  `part` needs
// ceil(n / (kScanT * kScanK)) int64 slots when n exceeds one chunk (else unused).
int scan_inplace(int64_t *v, int64_t n, int64_t *out_total, int64_t *part, hipStream_t s) {
  constexpr int64_t kChunk = (int64_t)kScanT * kScanK;
  if (n <= kChunk || !part) {
    hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(kScanT), 0, s, v, n, out_total);
    return check_launch("k_scan_inplace");
  }
  const int64_t g = (n + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(k_scan_chunk_sum, dim3((unsigned)g), dim3(kScanT), 0, s, v, n, part);
  hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(kScanT), 0, s, part, g, out_total);
  hipLaunchKernelGGL(k_scan_chunk_apply, dim3((unsigned)g), dim3(kScanT), 0, s, v, n, part);
  return check_launch("k_scan_chunk_apply");
}

template <typename L_T, typename V_T, typename T>
__global__ __launch_bounds__(kTB) void k_rld_scatter(const L_T *__restrict__ sym_len, const V_T *__restrict__ sym_val,
                                                     int64_t nsym, const int64_t *__restrict__ tile_off, StreamGeo g,
                                                     T *__restrict__ blocks) {
  __shared__ int64_t s_buf[8];
  const int64_t s0 = (int64_t)blockIdx.x * kTS + (int64_t)threadIdx.x * kSPT;
  int64_t acc = 0;
  int lens[kSPT];
#pragma unroll
  for (int k = 0; k < kSPT; ++k) {
    lens[k] = s0 + k < nsym ? (int)sym_len[s0 + k] : 0;
    if (s0 + k < nsym) acc += (int64_t)lens[k] + 1;
  }
  int64_t total;
  int64_t pos = tile_off[blockIdx.x] + block_excl_sum<int64_t, kTB>(acc, s_buf, total);
#pragma unroll
  for (int k = 0; k < kSPT; ++k) {
    if (s0 + k < nsym) {
      pos += lens[k];
      if (pos < g.n_ac) {
        const int64_t bb = pos / g.A, j = pos - bb * g.A;
        blocks[bb * g.L + g.off + j] = (T)sym_val[s0 + k];
      }
      ++pos;
    }
  }
}

// DC: per-tile sums, scan, then write prefix sums into slot 0 of every block.
__global__ __launch_bounds__(kTB) void k_dc_tile(const int32_t *__restrict__ diff, int64_t nblk,
                                                 int64_t *__restrict__ tile_sum) {
  __shared__ int64_t s_buf[8];
  const int64_t s0 = (int64_t)blockIdx.x * kTS + (int64_t)threadIdx.x * kSPT;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < kSPT; ++k)
    if (s0 + k < nblk) acc += diff[s0 + k];
  int64_t total;
  block_excl_sum<int64_t, kTB>(acc, s_buf, total);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

template <typename T>
__global__ __launch_bounds__(kTB) void k_dc_apply(const int32_t *__restrict__ diff, int64_t nblk,
                                                  const int64_t *__restrict__ tile_off, int L, T *__restrict__ blocks) {
  __shared__ int64_t s_buf[8];
  const int64_t s0 = (int64_t)blockIdx.x * kTS + (int64_t)threadIdx.x * kSPT;
  int64_t acc = 0;
  int d[kSPT];
#pragma unroll
  for (int k = 0; k < kSPT; ++k) {
    d[k] = s0 + k < nblk ? diff[s0 + k] : 0;
    acc += d[k];
  }
  int64_t total;
  int64_t run = tile_off[blockIdx.x] + block_excl_sum<int64_t, kTB>(acc, s_buf, total);
#pragma unroll
  for (int k = 0; k < kSPT; ++k)
    if (s0 + k < nblk) {
      run += d[k];
      blocks[(s0 + k) * L] = (T)run;
    }
}

__global__ void k_rld_status(const int64_t *__restrict__ total, const int64_t *__restrict__ last_sym, int64_t n_ac,
                             const int64_t *__restrict__ stitch, int64_t *__restrict__ status) {
  // codec.decode_run_length: EOB (last symbol (0,0)) zero-fills up to `length`.  A
  // shard that does not close the stream (stitch[1] == 0) ends in the zero run the
  // next shard carries on, so it zero-fills too; its positions start `carry` early.
  const int64_t t = *total - (stitch ? stitch[0] : 0);
  const bool eob = last_sym[0] == 0 && last_sym[1] == 0;
  const bool open_end = stitch && stitch[1] == 0;
  *status = ((eob || open_end) && t <= n_ac) ? n_ac : t;
}

template <typename L_T, typename V_T>
__global__ void k_last_sym(const L_T *__restrict__ sym_len, const V_T *__restrict__ sym_val, int64_t nsym,
                           int64_t *__restrict__ out) {
  out[0] = nsym > 0 ? (int64_t)sym_len[nsym - 1] : 1;
  out[1] = nsym > 0 ? (int64_t)sym_val[nsym - 1] : 1;
}

// ---------------------------------------------------------------------------
// Hot-path decode (uint8 lengths, int16 values, 64-slot int16 blocks, AC stream
// < 2^31 positions): every block is written exactly once, in 16-byte chunks.
//  k_rld_tile16   per tile of 4096 symbols: sum of (len + 1)
//  k_scan_inplace tile offsets
//  k_dc_tile / k_scan_inplace / k_dc_values16: integrated DC values -> dcval[nblk]
//  k_rld_blocks16 per symbol tile: the blocks its AC positions [P0, P1) touch are
//                 assembled in an LDS window (zeros, the tile's values, and the DC
//                 of blocks whose first AC lies in the tile), then copied out; the
//                 two edge blocks shared with neighbour tiles element-wise
//  k_rld_tail16   positions past the last symbol (EOB zero-fill) + their DCs
constexpr int kDS = 16;            // symbols per thread
constexpr int kDTS = kTB * kDS;    // symbols per tile
constexpr int kWinBlk = 160;       // LDS window: blocks per pass (20 KiB)

__global__ __launch_bounds__(kTB) void k_rld_tile16(const uint8_t *__restrict__ sym_len, int64_t nsym,
                                                    int64_t *__restrict__ tile_sum) {
  __shared__ int64_t s_buf[8];
  const int64_t s0 = (int64_t)blockIdx.x * kDTS + (int64_t)threadIdx.x * kDS;
  int acc = 0;
  if (s0 + kDS <= nsym) {
    const uint4 v = *reinterpret_cast<const uint4 *>(sym_len + s0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      acc += (int)((w[k] & 255) + ((w[k] >> 8) & 255) + ((w[k] >> 16) & 255) + (w[k] >> 24)) + 4;
  } else {
    for (int k = 0; k < kDS; ++k)
      if (s0 + k < nsym) acc += (int)sym_len[s0 + k] + 1;
  }
  int64_t total;
  block_excl_sum<int64_t, kTB>((int64_t)acc, s_buf, total);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// stitch (a shard's hic_rle_stitch record, or null): the chain starts at the
// previous shard's last DC instead of 0
__global__ __launch_bounds__(kTB) void k_dc_values16(const int32_t *__restrict__ diff, int64_t nblk,
                                                     const int64_t *__restrict__ tile_off,
                                                     const int64_t *__restrict__ stitch, int16_t *__restrict__ dcval) {
  __shared__ int64_t s_buf[8];
  const int64_t s0 = (int64_t)blockIdx.x * kTS + (int64_t)threadIdx.x * kSPT;
  const int64_t base = (stitch && stitch[2]) ? stitch[3] : 0;
  int64_t acc = 0;
  int d[kSPT];
#pragma unroll
  for (int k = 0; k < kSPT; ++k) {
    d[k] = s0 + k < nblk ? diff[s0 + k] : 0;
    acc += d[k];
  }
  int64_t total;
  int64_t run = base + tile_off[blockIdx.x] + block_excl_sum<int64_t, kTB>(acc, s_buf, total);
#pragma unroll
  for (int k = 0; k < kSPT; ++k)
    if (s0 + k < nblk) {
      run += d[k];
      dcval[s0 + k] = (int16_t)run;
    }
}

// element-wise write of the slots of block b that belong to AC range [lo, hi)
// (slot 0, the DC, when the block's first AC position 63 b is in it)
__device__ __forceinline__ void put_block_part(int16_t *__restrict__ blocks, int64_t b, int lo, int hi,
                                               const int16_t *win, int16_t dc, int slot0, int nslot) {
  const int f = (int)(b * 63);
  for (int slot = slot0; slot < slot0 + nslot; ++slot) {
    if (slot == 0) {
      if (f >= lo && f < hi) blocks[b * 64] = dc;
    } else {
      const int p = f + slot - 1;
      if (p >= lo && p < hi) blocks[b * 64 + slot] = win ? win[slot] : 0;
    }
  }
}

template <bool NT>
__global__ __launch_bounds__(kTB) void k_rld_blocks16(const uint8_t *__restrict__ sym_len,
                                                      const int16_t *__restrict__ sym_val, int64_t nsym,
                                                      const int64_t *__restrict__ tile_off, int n_ac,
                                                      const int64_t *__restrict__ stitch,
                                                      const int16_t *__restrict__ dcval, int16_t *__restrict__ blocks) {
  __shared__ uint4 s_win[kWinBlk * 8];
  __shared__ int64_t s_buf[8];
  int16_t *win = reinterpret_cast<int16_t *>(s_win);
  const int tid = threadIdx.x;
  const int64_t s0 = (int64_t)blockIdx.x * kDTS + (int64_t)tid * kDS;
  int len[kDS], val[kDS];
  if (s0 + kDS <= nsym) {
    const uint4 l = *reinterpret_cast<const uint4 *>(sym_len + s0);
    const uint4 v0 = *reinterpret_cast<const uint4 *>(sym_val + s0);
    const uint4 v1 = *reinterpret_cast<const uint4 *>(sym_val + s0 + 8);
    const uint32_t lw[4] = {l.x, l.y, l.z, l.w};
    const uint32_t vw[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int k = 0; k < kDS; ++k) {
      len[k] = (int)((lw[k >> 2] >> (8 * (k & 3))) & 255);
      val[k] = (int)(int16_t)(vw[k >> 1] >> (16 * (k & 1)));
    }
  } else {
#pragma unroll
    for (int k = 0; k < kDS; ++k) {
      len[k] = s0 + k < nsym ? (int)sym_len[s0 + k] : -1;  // -1: no symbol
      val[k] = s0 + k < nsym ? (int)sym_val[s0 + k] : 0;
    }
  }
  int acc = 0;
#pragma unroll
  for (int k = 0; k < kDS; ++k) acc += len[k] + 1;
  int64_t tot64;
  // a shard's stream starts `carry` zeros before its first block (the run it
  // continues from the previous shards: hic_rle_stitch)
  const int64_t skip = stitch ? stitch[0] : 0;
  const int64_t P0l = tile_off[blockIdx.x] - skip;
  const int64_t my = P0l + block_excl_sum<int64_t, kTB>((int64_t)acc, s_buf, tot64);
  // positions fit int32 (the launcher checks n_ac < 2^31); clamp to [0, n_ac]
  const int64_t P1l = P0l + tot64;
  const int P0 = (int)(P0l < 0 ? 0 : (P0l < n_ac ? P0l : n_ac));
  const int P1 = (int)(P1l < 0 ? 0 : (P1l < n_ac ? P1l : n_ac));
  if (P1 <= P0) return;  // uniform
  int pos[kDS];
  {
    int64_t q = my;
#pragma unroll
    for (int k = 0; k < kDS; ++k) {
      q += len[k];
      pos[k] = (len[k] >= 0 && q >= 0 && q < n_ac) ? (int)q : -1;
      ++q;
    }
  }
  const int b_first = P0 / 63, b_last = (P1 - 1) / 63;
  for (int wb0 = b_first; wb0 <= b_last; wb0 += kWinBlk) {
    const int nb = b_last + 1 - wb0 < kWinBlk ? b_last + 1 - wb0 : kWinBlk;
    for (int i = tid; i < nb * 8; i += kTB) s_win[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kDS; ++k) {
      if (pos[k] >= 0) {
        const int b = pos[k] / 63;
        if (b >= wb0 && b < wb0 + nb) win[(b - wb0) * 64 + 1 + (pos[k] - b * 63)] = (int16_t)val[k];
      }
    }
    for (int i = tid; i < nb; i += kTB) {
      const int b = wb0 + i;
      if (b * 63 >= P0) win[i * 64] = dcval[b];  // first AC of the block is ours (and < P1: b <= b_last)
    }
    __syncthreads();
    for (int i = tid; i < nb * 8; i += kTB) {
      const int bi = i >> 3, c = i & 7;
      const int64_t b = wb0 + bi;
      const int f = (int)(b * 63);
      if (f >= P0 && f + 62 < P1) {
        if (NT) {  // nontemporal: a 16K plane's blocks overflow every cache level
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const uint4 t = s_win[i];
          const u32x4 v = {t.x, t.y, t.z, t.w};
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(blocks + b * 64) + c);
        } else {
          reinterpret_cast<uint4 *>(blocks + b * 64)[c] = s_win[i];
        }
      } else {
        put_block_part(blocks, b, P0, P1, win + bi * 64, win[bi * 64], 8 * c, 8);
      }
    }
    __syncthreads();
  }
}

// positions [*total, n_ac): zeros (codec.decode_run_length's EOB fill), and the DC of
// every block whose first AC lies there
__global__ __launch_bounds__(kTB) void k_rld_tail16(const int64_t *__restrict__ total, int64_t nblk,
                                                    const int64_t *__restrict__ stitch,
                                                    const int16_t *__restrict__ dcval, int16_t *__restrict__ blocks) {
  const int64_t n_ac = nblk * 63;
  const int64_t tl = *total - (stitch ? stitch[0] : 0);
  const int64_t t = tl < 0 ? 0 : (tl < n_ac ? tl : n_ac);
  if (t >= n_ac) return;
  const int64_t b0 = t / 63;
  const int64_t nchunk = (nblk - b0) * 8;
  for (int64_t i = (int64_t)blockIdx.x * kTB + threadIdx.x; i < nchunk; i += (int64_t)gridDim.x * kTB) {
    const int64_t b = b0 + (i >> 3);
    const int c = (int)(i & 7);
    if (b * 63 >= t) {
      const int16_t dc = dcval[b];
      reinterpret_cast<uint4 *>(blocks + b * 64)[c] = make_uint4(c == 0 ? (uint32_t)(uint16_t)dc : 0u, 0, 0, 0);
    } else {
      put_block_part(blocks, b, (int)t, (int)n_ac, nullptr, 0, 8 * c, 8);
    }
  }
}

// ---------------------------------------------------------------------------
// Generic split_matrix + zigzag for block size N (any N), int32.
__device__ __forceinline__ void zz_pos(int z, int N, int &y, int &x) {
  int s = 0;
  for (;; ++s) {
    const int len = s < N ? s + 1 : 2 * N - 1 - s;
    if (z < len) break;
    z -= len;
  }
  const int ylo = s - (N - 1) > 0 ? s - (N - 1) : 0;
  const int yhi = s < N - 1 ? s : N - 1;
  y = (s % 2 == 0) ? ylo + z : yhi - z;
  x = s - y;
}

__global__ void k_zigzag_i32(const int32_t *__restrict__ raster, int H, int W, int N, int nbx, int64_t total,
                             int32_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int NN = N * N;
  const int64_t b = i / NN;
  const int z = (int)(i - b * NN);
  const int bi = (int)(b / nbx), bj = (int)(b - (int64_t)bi * nbx);
  int u, v;
  zz_pos(z, N, u, v);
  const int yy = bi * N + u, xx = bj * N + v;
  out[i] = (yy < H && xx < W) ? raster[(int64_t)yy * W + xx] : 0;
}

// 8x8 form into int16 blocks (jpeg_encode's fast path): *wide = 1 when a value is
// outside int16 (the caller then takes the int32 path for the plane)
__global__ __launch_bounds__(256) void k_zigzag8_i16(const int32_t *__restrict__ raster, int H, int W, int nbx,
                                                     int64_t total, int16_t *__restrict__ out, int *__restrict__ wide) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t b = i >> 6;
  const int bi = (int)(b / nbx), bj = (int)(b - (int64_t)bi * nbx);
  int u, v;
  zz_pos((int)(i & 63), 8, u, v);
  const int yy = bi * 8 + u, xx = bj * 8 + v;
  const int x = (yy < H && xx < W) ? raster[(int64_t)yy * W + xx] : 0;
  if (x < -32768 || x > 32767) atomicOr(wide, 1);
  out[i] = (int16_t)x;
}

__global__ void k_izigzag_i32(const int32_t *__restrict__ blocks, int H, int W, int N, int nbx, int64_t total,
                              int32_t *__restrict__ raster) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int NN = N * N;
  const int64_t b = i / NN;
  const int z = (int)(i - b * NN);
  const int bi = (int)(b / nbx), bj = (int)(b - (int64_t)bi * nbx);
  int u, v;
  zz_pos(z, N, u, v);
  const int yy = bi * N + u, xx = bj * N + v;
  if (yy < H && xx < W) raster[(int64_t)yy * W + xx] = blocks[i];
}

// ---------------------------------------------------------------------------
inline int64_t ntiles_of(int64_t nblk) { return (nblk + kTB - 1) / kTB; }

template <typename T, typename L_T, typename V_T>
int rle_encode(const T *blocks, int64_t nblk, StreamGeo g, int M, const int64_t *stitch, int32_t *dc_diff,
               L_T *sym_len, V_T *sym_val, int64_t cap, int64_t *d_count, void *ws, hipStream_t s) {
  if (!blocks || !sym_len || !sym_val || !d_count || !ws) return arg_error("null pointer");
  if (nblk <= 0 || g.A < 1 || g.n_ac < 0) return arg_error("nblk / block_len");
  if (M < 0) return arg_error("max_len");
  const int64_t nt = ntiles_of(nblk);
  int64_t *tiles = static_cast<int64_t *>(ws);
  int64_t *offs = tiles + 3 * nt;
  hipLaunchKernelGGL((k_rle_tile<T>), dim3((unsigned)nt), dim3(kTB), 0, s, blocks, nblk, g, M, tiles);
  if (int e = check_launch("k_rle_tile")) return e;
  hipLaunchKernelGGL((k_rle_scan<L_T, V_T>), dim3(1), dim3(kScanT), 0, s, tiles, offs, nt, g.n_ac, M, stitch,
                     sym_len, sym_val, cap, d_count);
  if (int e = check_launch("k_rle_scan")) return e;
  hipLaunchKernelGGL((k_rle_emit<T, L_T, V_T>), dim3((unsigned)nt), dim3(kTB), 0, s, blocks, nblk, g, M, offs,
                     stitch, dc_diff, sym_len, sym_val, cap);
  return check_launch("k_rle_emit");
}

inline int64_t ntiles16(int64_t nblk) { return (nblk + kWT - 1) / kWT; }

int launch_tile16(const int16_t *blocks, int64_t nblk, int M, int64_t *tiles, hipStream_t s) {
  const dim3 grid((unsigned)((ntiles16(nblk) + 3) / 4));
  if (M == 15)
    hipLaunchKernelGGL((k_rle_tile16<15>), grid, dim3(256), 0, s, blocks, nblk, M, tiles);
  else
    hipLaunchKernelGGL((k_rle_tile16<0>), grid, dim3(256), 0, s, blocks, nblk, M, tiles);
  return check_launch("k_rle_tile16");
}

// K2 + K3 of the hot path on tile records already in the workspaces (from
// k_rle_tile16 or the fused DCT epilogue), for up to kMaxJobs channels at once.
// job geometry (tiles, records, first global tile) and the workspace check
int prepare_batch16(RleJobs16 &jobs) {
  int64_t t0 = 0;
  for (int k = 0; k < jobs.n; ++k) {
    // stream positions and counts travel as int32 through the scan's hand-off
    if (jobs.j[k].nblk > (int64_t)INT32_MAX / 63) return arg_error("nblk too large (AC stream >= 2^31)");
    if (jobs.j[k].rowb > 0) {  // row segments
      const int64_t rows = jobs.j[k].nblk / jobs.j[k].rowb, seg = kWT >> jobs.j[k].rshift;
      jobs.j[k].tpr = (jobs.j[k].rowb + kWT - 1) / kWT;
      jobs.j[k].rpr = (jobs.j[k].rowb + seg - 1) / seg;
      jobs.j[k].ntiles = rows * jobs.j[k].tpr;
      jobs.j[k].nrec = rows * jobs.j[k].rpr;
    } else {
      jobs.j[k].ntiles = ntiles16(jobs.j[k].nblk);
      jobs.j[k].nrec = (jobs.j[k].nblk * (1 << jobs.j[k].rshift) + kWT - 1) / kWT;
    }
    jobs.j[k].tile0 = t0;
    t0 += jobs.j[k].ntiles;
    // the scan reads 5 words per record and the partitions' hand-off granules
    const int64_t need = rle_ws_words(jobs.j[k].nrec) * (int64_t)sizeof(int64_t);
    if (jobs.j[k].rowb > 0 && jobs.j[k].wsb <= 0) return arg_error("job %d: row segments need workspace_bytes", k);
    if (jobs.j[k].wsb > 0 && jobs.j[k].wsb < need)
      return arg_error("job %d: workspace of %lld bytes, %lld needed", k, (long long)jobs.j[k].wsb, (long long)need);
  }
  jobs.total_tiles = t0;
  return HIC_OK;
}

// the batch's scan (SLOTS: the slot layout's close); returns its launch status
template <bool SLOTS>
int scan_batch16(RleJobs16 &jobs, hipStream_t s) {
  const uint32_t ep = next_epoch();
  int64_t nparts = 0;
  for (int k = 0; k < jobs.n; ++k) nparts += (jobs.j[k].nrec + kScan16T - 1) / kScan16T;
  jobs.epoch = ep;
  hipLaunchKernelGGL(k_rle_scan16b<SLOTS>, dim3((unsigned)nparts), dim3(kScan16T), 0, s, jobs, ep);
  return check_launch("k_rle_scan16b");
}

int encode_batch16(RleJobs16 &jobs, hipStream_t s) {
  if (int e = prepare_batch16(jobs)) return e;
  const int64_t t0 = jobs.total_tiles;
  if (int e = scan_batch16<false>(jobs, s)) return e;
  // persistent: 3 workgroups (12 waves) per CU fit the 51 KB LDS stage and the registers
#ifndef HIC_EMIT_WPC
#define HIC_EMIT_WPC 12
#endif
  const int64_t cap = HIC_EMIT_WPC > 0 ? HIC_EMIT_WPC * (int64_t)cu_count() : INT64_MAX;
  const int64_t waves = t0 < cap ? t0 : cap;
  const dim3 grid((unsigned)((waves + 3) / 4));
  // nontemporal symbol stores unless knob RLE_NT = 0 (A/B)
  const bool nt = knob(HIC_KNOB_RLE_NT) != 0;
  if (jobs.M == 15 && nt)
    hipLaunchKernelGGL((k_rle_emit16b<15, true>), grid, dim3(256), 0, s, jobs);
  else if (jobs.M == 15)
    hipLaunchKernelGGL((k_rle_emit16b<15, false>), grid, dim3(256), 0, s, jobs);
  else if (nt)
    hipLaunchKernelGGL((k_rle_emit16b<0, true>), grid, dim3(256), 0, s, jobs);
  else
    hipLaunchKernelGGL((k_rle_emit16b<0, false>), grid, dim3(256), 0, s, jobs);
  return check_launch("k_rle_emit16b");
}

int encode_from_tiles16(const int16_t *blocks, int64_t nblk, int M, const int64_t *stitch, int32_t *dc_diff,
                        uint8_t *sym_len, int16_t *sym_val, int64_t cap, int64_t *d_count, void *ws, hipStream_t s) {
  RleJobs16 jobs{};
  jobs.n = 1;
  jobs.M = M;
  jobs.j[0] = RleJob16{blocks, nblk, stitch, dc_diff, sym_len, sym_val, cap, d_count, static_cast<int64_t *>(ws), 0, 0,
                       0, 0};
  return encode_batch16(jobs, s);
}

inline StreamGeo block_geo(int64_t nblk, int L) { return StreamGeo{L, 1, L - 1, nblk * (L - 1)}; }
inline StreamGeo raw_geo(int64_t n) { return StreamGeo{64, 0, 64, n}; }

template <typename T>
int rle_summary(const T *blocks, int64_t nblk, int L, void *ws, int64_t *d_summary, hipStream_t s) {
  if (!blocks || !ws || !d_summary) return arg_error("null pointer");
  if (nblk <= 0 || L < 2) return arg_error("nblk / block_len");
  const int64_t nt = ntiles_of(nblk);
  const StreamGeo g = block_geo(nblk, L);
  int64_t *tiles = static_cast<int64_t *>(ws);
  hipLaunchKernelGGL((k_rle_tile<T>), dim3((unsigned)nt), dim3(kTB), 0, s, blocks, nblk, g, 15, tiles);
  if (int e = check_launch("k_rle_tile")) return e;
  hipLaunchKernelGGL((k_rle_summary<T>), dim3(1), dim3(kTB), 0, s, blocks, nblk, g, tiles, nt, d_summary);
  return check_launch("k_rle_summary");
}

template <typename L_T, typename V_T, typename T>
int rle_decode(const L_T *sym_len, const V_T *sym_val, int64_t nsym, const int32_t *dc_diff, int64_t nblk,
               StreamGeo g, int64_t length, T *blocks, int64_t *d_status, void *ws, hipStream_t s) {
  if (!sym_len || !sym_val || !blocks || !d_status || !ws) return arg_error("null pointer");
  if (nblk <= 0 || g.A < 1 || nsym < 0) return arg_error("sizes");
  const int64_t nts = (nsym + kTS - 1) / kTS, ntb = (nblk + kTS - 1) / kTS;
  int64_t *w = static_cast<int64_t *>(ws);
  int64_t *tsum = w, *dsum = w + nts + 1, *tot = dsum + ntb + 1, *last = tot + 2;
  if (int e = hip_status(hipMemsetAsync(blocks, 0, (size_t)nblk * g.L * sizeof(T), s), "hipMemsetAsync")) return e;
  if (nsym > 0) {
    hipLaunchKernelGGL((k_rld_tile<L_T>), dim3((unsigned)nts), dim3(kTB), 0, s, sym_len, nsym, tsum);
    if (int e = check_launch("k_rld_tile")) return e;
  }
  hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(kScanT), 0, s, tsum, nts, tot);
  if (nsym > 0) {
    hipLaunchKernelGGL((k_rld_scatter<L_T, V_T, T>), dim3((unsigned)nts), dim3(kTB), 0, s, sym_len, sym_val, nsym,
                       tsum, g, blocks);
    if (int e = check_launch("k_rld_scatter")) return e;
  }
  if (dc_diff) {
    hipLaunchKernelGGL(k_dc_tile, dim3((unsigned)ntb), dim3(kTB), 0, s, dc_diff, nblk, dsum);
    hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(kScanT), 0, s, dsum, ntb, tot + 1);
    hipLaunchKernelGGL((k_dc_apply<T>), dim3((unsigned)ntb), dim3(kTB), 0, s, dc_diff, nblk, dsum, g.L, blocks);
  }
  hipLaunchKernelGGL((k_last_sym<L_T, V_T>), dim3(1), dim3(1), 0, s, sym_len, sym_val, nsym, last);
  hipLaunchKernelGGL(k_rld_status, dim3(1), dim3(1), 0, s, tot, last, length, nullptr, d_status);
  return check_launch("k_rld_status");
}

// The hot-path decode (see k_rld_blocks16).  Workspace as hic_rld_workspace_bytes.
int rle_decode_blocks16(const uint8_t *sym_len, const int16_t *sym_val, int64_t nsym, const int32_t *dc_diff,
                        int64_t nblk, const int64_t *stitch, int16_t *blocks, int64_t *d_status, void *ws,
                        hipStream_t s) {
  const int64_t nts = (nsym + kDTS - 1) / kDTS, ntb = (nblk + kTS - 1) / kTS;
  int64_t *w = static_cast<int64_t *>(ws);
  // same int64 slots as rle_decode (its symbol tiles are smaller, so these fit)
  int64_t *tsum = w, *dsum = w + (nsym + kTS - 1) / kTS + 1, *tot = dsum + ntb + 1, *last = tot + 2;
  int16_t *dcval = reinterpret_cast<int16_t *>(last + 4);
  if (nts > 0) {
    hipLaunchKernelGGL(k_rld_tile16, dim3((unsigned)nts), dim3(kTB), 0, s, sym_len, nsym, tsum);
    if (int e = check_launch("k_rld_tile16")) return e;
  }
  // chunk partials in the tsum slots past nts (the region is sized for kTS tiles,
  // twice the count of kDTS tiles, so ceil(nts / 8192) <= nts slots are free there)
  if (int e = scan_inplace(tsum, nts, tot, tsum + nts, s)) return e;
  hipLaunchKernelGGL(k_dc_tile, dim3((unsigned)ntb), dim3(kTB), 0, s, dc_diff, nblk, dsum);
  hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(kScanT), 0, s, dsum, ntb, tot + 1);
  hipLaunchKernelGGL(k_dc_values16, dim3((unsigned)ntb), dim3(kTB), 0, s, dc_diff, nblk, dsum, stitch, dcval);
  if (int e = check_launch("k_dc_values16")) return e;
  if (nts > 0) {
    const bool nt = knob(HIC_KNOB_RLD_NT) == 1;  // A/B: nontemporal block stores
    if (nt)
      hipLaunchKernelGGL(k_rld_blocks16<true>, dim3((unsigned)nts), dim3(kTB), 0, s, sym_len, sym_val, nsym, tsum,
                       (int)(nblk * 63), stitch, dcval, blocks);
    else
      hipLaunchKernelGGL(k_rld_blocks16<false>, dim3((unsigned)nts), dim3(kTB), 0, s, sym_len, sym_val, nsym, tsum,
                       (int)(nblk * 63), stitch, dcval, blocks);
    if (int e = check_launch("k_rld_blocks16")) return e;
  }
  const int64_t tail_grid = cu_count() * 8 > 0 ? cu_count() * 8 : 1024;
  hipLaunchKernelGGL(k_rld_tail16, dim3((unsigned)tail_grid), dim3(kTB), 0, s, tot, nblk, stitch, dcval, blocks);
  hipLaunchKernelGGL((k_last_sym<uint8_t, int16_t>), dim3(1), dim3(1), 0, s, sym_len, sym_val, nsym, last);
  hipLaunchKernelGGL(k_rld_status, dim3(1), dim3(1), 0, s, tot, last, nblk * 63, stitch, d_status);
  return check_launch("k_rld_status");
}

// ---------------------------------------------------------------------------
// Encoder-side tile index and the indexed decode.  After the scan, the RLE
// workspace holds for every record its stream offset and the last nonzero AC
// position before it; the index keeps, per 64-block tile, {offset of the tile's
// first symbol, last nonzero position before the tile (-1: none), DC of the block
// before the tile}.  With it a decoder needs no symbol-tile pass, no scans and no
// DC chain: one wave per coefficient tile walks exactly the symbols the encoder's
// emit wrote for that tile (codec.decode_run_length, codec.py:102-113, restricted
// to the tile's positions; utils.invert_differences, utils.py:66-73, from the
// previous block's DC).
__global__ __launch_bounds__(256) void k_rle_index16(const int64_t *__restrict__ offs, int rshift, int64_t ntiles,
                                                     const int16_t *__restrict__ blocks, int64_t *__restrict__ index) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= ntiles) return;
  const int64_t r = t << rshift;
  index[3 * t] = offs[2 * r];
  index[3 * t + 1] = offs[2 * r + 1];
  index[3 * t + 2] = t > 0 ? (int64_t)blocks[(t * 64 - 1) * 64] : 0;
}

// SLOTS: the symbols are in the slot layout (slots.h) and `index` is the close's
// int32 record index (rsh: log2 records per 64-block tile).
template <bool NT, bool SLOTS = false>
__global__ __launch_bounds__(256) void k_rld_indexed16(const uint8_t *__restrict__ sym_len,
                                                       const int16_t *__restrict__ sym_val,
                                                       const int64_t *__restrict__ d_nsym,
                                                       const int32_t *__restrict__ dc_diff, int64_t nblk,
                                                       const int64_t *__restrict__ index, int16_t *__restrict__ blocks,
                                                       int64_t *__restrict__ d_status, int rsh = 0) {
  __shared__ uint4 s_tile[4][64 * 8 + 8];  // 64 blocks + 64 trash slots
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t ntiles = (nblk + 63) / 64;
  const int64_t t = (int64_t)blockIdx.x * 4 + wv;
  if (t >= ntiles) return;  // wave-uniform
  uint4 *tile = s_tile[wv];
  int16_t *win = reinterpret_cast<int16_t *>(tile);
  // the encoder's symbol count, read on the device (no host round trip); a failed
  // encode's count (< 1) decodes nothing and reports status -1
  const int64_t nsym_raw = *d_nsym, nsym = nsym_raw > 0 ? nsym_raw : 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) tile[64 * k + lane] = make_uint4(0, 0, 0, 0);
  __builtin_amdgcn_wave_barrier();
  const int64_t tb0 = t * 64 * 63;                    // the tile's first AC position
  const int nvb = (int)(nblk - t * 64 < 64 ? nblk - t * 64 : 64);
  const int span = nvb * 63;                           // its AC positions
  int P = 0, pdc;
  if constexpr (SLOTS) {
    // the tile's records, each from its own slot (trash slots: the 64 after the tile)
    const SlotTileIx six = slot_tile_ix(reinterpret_cast<const int32_t *>(index), t, rsh, nblk);
    P = slots_gather_tile<64>(sym_len, sym_val, six, t, rsh, span, win, 64 * 64 + lane, lane);
    pdc = six.r[0].z;
  } else {
    const int64_t o0 = index[3 * t] < nsym ? index[3 * t] : nsym;
    const int64_t o1 = t + 1 < ntiles ? (index[3 * (t + 1)] < nsym ? index[3 * (t + 1)] : nsym) : nsym;
    // P: the position after the previous tile's last symbol, relative to the tile (a
    // carried run can start far before it; every AC position of the stream fits int32).
    // Trash slots (never read): the 64 after the tile.
    P = gather_tile<64, HIC_DEC_G, HIC_DEC_PF>(sym_len, sym_val, o0, o1, nsym, (int)(index[3 * t + 1] + 1 - tb0), span,
                                               win, 64 * 64 + lane, lane);
    pdc = (int)index[3 * t + 2];
  }
  // DC: the previous block's value plus this tile's differences
  const int64_t b = t * 64 + lane;
  const int d = lane < nvb ? dc_diff[b] : 0;
  win[lane * 64] = (int16_t)(pdc + wave_incl_sum_i32(d));
  __builtin_amdgcn_wave_barrier();
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int ci = 64 * k + lane, bb = ci >> 3;
    if (bb < nvb) {
      const uint4 x = tile[ci];
      u32x4 *o = reinterpret_cast<u32x4 *>(blocks + t * 64 * 64) + ci;
      if (NT)
        __builtin_nontemporal_store(u32x4{x.x, x.y, x.z, x.w}, o);
      else
        *o = u32x4{x.x, x.y, x.z, x.w};
    }
  }
  if (t == ntiles - 1 && lane == 0) {
    // codec.decode_run_length's length: an EOB zero-fills to the end (a slot-layout
    // stream is whole by construction)
    const int64_t total = tb0 + (int64_t)P, n_ac = nblk * 63;
    const bool eob = SLOTS || (nsym > 0 && sym_len[nsym - 1] == 0 && sym_val[nsym - 1] == 0);
    *d_status = nsym_raw < 1 ? -1 : ((eob && (SLOTS || total <= n_ac)) ? n_ac : total);
  }
}

}  // namespace
}  // namespace hic

namespace hic {
int rle_tile16_launch(const int16_t *blocks, int64_t nblk, int max_len, int64_t *tiles, hipStream_t s) {
  if (nblk <= 0) return arg_error("nblk");
  return launch_tile16(blocks, nblk, max_len, tiles, s);
}
}  // namespace hic

using namespace hic;

extern "C" size_t hic_rle_workspace_bytes(int64_t nblk, int block_len) {
  (void)block_len;
  // sized for the hot path's 32-block half-tile records (hic_encode420_u8's chroma;
  // >= its 64-block tiles and the generic 256-block tiles)
  const int64_t n = nblk > 0 ? nblk : 1;
  return (size_t)rle_ws_words((n + kWT / 2 - 1) / (kWT / 2)) * sizeof(int64_t);
}

extern "C" size_t hic_rle_rows_workspace_bytes(int64_t nblk, int64_t row_blocks, int records_per_tile) {
  // records per row segment (hic_encode420_seg_u8 / hic_rle_encode_i16_rows_batch):
  // rows x ceil(row_blocks / segment) records, segment 64 / records_per_tile blocks
  const int64_t n = nblk > 0 ? nblk : 1, rb = row_blocks > 0 ? row_blocks : 1;
  const int64_t seg = records_per_tile == 2 ? kWT / 2 : kWT;
  const int64_t nrec = ((n + rb - 1) / rb) * ((rb + seg - 1) / seg);
  const size_t rows = (size_t)rle_ws_words(nrec) * sizeof(int64_t), tiles = hic_rle_workspace_bytes(nblk, 64);
  return rows > tiles ? rows : tiles;
}

extern "C" int hic_rle_shard_summary_i16(const int16_t *blocks, int64_t nblk, int block_len, void *workspace,
                                         int64_t *d_summary, void *stream) {
  return rle_summary(blocks, nblk, block_len, workspace, d_summary, as_stream(stream));
}
extern "C" int hic_rle_shard_summary_i32(const int32_t *blocks, int64_t nblk, int block_len, void *workspace,
                                         int64_t *d_summary, void *stream) {
  return rle_summary(blocks, nblk, block_len, workspace, d_summary, as_stream(stream));
}

extern "C" int hic_rle_encode_i16(const int16_t *blocks, int64_t nblk, int block_len, int max_len,
                                  const int64_t *d_stitch, int32_t *dc_diff, uint8_t *sym_len, int16_t *sym_val,
                                  int64_t sym_cap, int64_t *d_count, void *workspace, void *stream) {
  // uint8 lengths: fillers are max_len-1 <= 255 and residual runs < max_len
  if (max_len < 1 || max_len > 256) return arg_error("max_len must be in [1, 256] for uint8 symbol lengths");
  if (block_len == 64 && (reinterpret_cast<uintptr_t>(blocks) & 15) == 0) {
    if (!blocks || !dc_diff || !sym_len || !sym_val || !d_count || !workspace) return arg_error("null pointer");
    if (nblk <= 0) return arg_error("nblk");
    hipStream_t s = as_stream(stream);
    if (int e = launch_tile16(blocks, nblk, max_len, static_cast<int64_t *>(workspace), s)) return e;
    return encode_from_tiles16(blocks, nblk, max_len, d_stitch, dc_diff, sym_len, sym_val, sym_cap, d_count,
                               workspace, s);
  }
  if (block_len < 2) return arg_error("block_len");
  if (!dc_diff) return arg_error("null dc_diff");
  return rle_encode(blocks, nblk, block_geo(nblk, block_len), max_len, d_stitch, dc_diff, sym_len, sym_val, sym_cap,
                    d_count, workspace, as_stream(stream));
}

extern "C" int hic_rle_encode_i16_tiles(const int16_t *blocks, int64_t nblk, int max_len, const int64_t *d_stitch,
                                        int32_t *dc_diff, uint8_t *sym_len, int16_t *sym_val, int64_t sym_cap,
                                        int64_t *d_count, void *workspace, void *stream) {
  if (!blocks || !dc_diff || !sym_len || !sym_val || !d_count || !workspace) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (max_len < 1 || max_len > 256) return arg_error("max_len must be in [1, 256] for uint8 symbol lengths");
  if (reinterpret_cast<uintptr_t>(blocks) & 15) return arg_error("blocks must be 16-byte aligned");
  return encode_from_tiles16(blocks, nblk, max_len, d_stitch, dc_diff, sym_len, sym_val, sym_cap, d_count, workspace,
                             as_stream(stream));
}

extern "C" int hic_rle_tile_records_i16(const int16_t *blocks, int64_t nblk, int max_len, void *workspace,
                                        void *stream) {
  if (!blocks || !workspace) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (max_len < 1 || max_len > 256) return arg_error("max_len must be in [1, 256] for uint8 symbol lengths");
  if (reinterpret_cast<uintptr_t>(blocks) & 15) return arg_error("blocks must be 16-byte aligned");
  return launch_tile16(blocks, nblk, max_len, static_cast<int64_t *>(workspace), as_stream(stream));
}

extern "C" int hic_rle_encode_i16_tiles_batch(int n, const hic_rle_job16 *jobs, int max_len, void *stream) {
  if (n < 1 || n > kMaxJobs || !jobs) return arg_error("1 <= n <= %d jobs", kMaxJobs);
  if (max_len < 1 || max_len > 256) return arg_error("max_len must be in [1, 256] for uint8 symbol lengths");
  RleJobs16 J{};
  J.n = n;
  J.M = max_len;
  for (int k = 0; k < n; ++k) {
    const hic_rle_job16 &a = jobs[k];
    if (!a.blocks || !a.dc_diff || !a.sym_len || !a.sym_val || !a.d_count || !a.workspace)
      return arg_error("job %d: null pointer", k);
    if (a.nblk <= 0) return arg_error("job %d: nblk", k);
    if (reinterpret_cast<uintptr_t>(a.blocks) & 15) return arg_error("job %d: blocks must be 16-byte aligned", k);
    if (a.records_per_tile != 0 && a.records_per_tile != 1 && a.records_per_tile != 2)
      return arg_error("job %d: records_per_tile must be 1 or 2", k);
    if (a.d_index && a.d_stitch) return arg_error("job %d: d_index needs a job without d_stitch", k);
    J.j[k] = RleJob16{a.blocks, a.nblk, a.d_stitch, a.dc_diff, a.sym_len, a.sym_val, a.sym_cap, a.d_count,
                      static_cast<int64_t *>(a.workspace), 0, 0, 0, a.records_per_tile == 2 ? 1 : 0, 0, 0, 0,
                      a.workspace_bytes, a.d_index};
  }
  return encode_batch16(J, as_stream(stream));
}

extern "C" int hic_rle_encode_i16_rows_batch(int n, const hic_rle_job16 *jobs, const int64_t *h_row_blocks,
                                             int max_len, void *stream) {
  if (n < 1 || n > kMaxJobs || !jobs || !h_row_blocks) return arg_error("1 <= n <= %d jobs", kMaxJobs);
  if (max_len < 1 || max_len > 256) return arg_error("max_len must be in [1, 256] for uint8 symbol lengths");
  RleJobs16 J{};
  J.n = n;
  J.M = max_len;
  for (int k = 0; k < n; ++k) {
    const hic_rle_job16 &a = jobs[k];
    if (!a.blocks || !a.dc_diff || !a.sym_len || !a.sym_val || !a.d_count || !a.workspace)
      return arg_error("job %d: null pointer", k);
    if (a.nblk <= 0) return arg_error("job %d: nblk", k);
    if (reinterpret_cast<uintptr_t>(a.blocks) & 15) return arg_error("job %d: blocks must be 16-byte aligned", k);
    if (a.records_per_tile != 0 && a.records_per_tile != 1 && a.records_per_tile != 2)
      return arg_error("job %d: records_per_tile must be 1 or 2", k);
    const int64_t rb = h_row_blocks[k];
    if (rb < 1 || a.nblk % rb) return arg_error("job %d: row_blocks must divide nblk", k);
    if (a.d_index) return arg_error("job %d: d_index is for hic_rle_encode_i16_tiles_batch", k);
    J.j[k] = RleJob16{a.blocks, a.nblk, a.d_stitch, a.dc_diff, a.sym_len, a.sym_val, a.sym_cap, a.d_count,
                      static_cast<int64_t *>(a.workspace), 0, 0, 0, a.records_per_tile == 2 ? 1 : 0, rb, 0, 0,
                      a.workspace_bytes};
  }
  return encode_batch16(J, as_stream(stream));
}

extern "C" int hic_rle_tile_index_i16(const int16_t *blocks, int64_t nblk, int records_per_tile, const void *workspace,
                                      int64_t *d_index, void *stream) {
  if (!blocks || !workspace || !d_index) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (records_per_tile != 1 && records_per_tile != 2) return arg_error("records_per_tile must be 1 or 2");
  const int64_t ntiles = (nblk + kWT - 1) / kWT, nrec = (nblk * records_per_tile + kWT - 1) / kWT;
  const int64_t *offs = static_cast<const int64_t *>(workspace) + 3 * nrec;
  hipLaunchKernelGGL(k_rle_index16, dim3((unsigned)((ntiles + 255) / 256)), dim3(256), 0, as_stream(stream), offs,
                     records_per_tile == 2 ? 1 : 0, ntiles, blocks, d_index);
  return check_launch("k_rle_index16");
}

extern "C" int hic_rle_decode_i16_indexed(const uint8_t *sym_len, const int16_t *sym_val, const int64_t *d_nsym,
                                          const int32_t *dc_diff, int64_t nblk, const int64_t *d_index,
                                          int16_t *blocks, int64_t *d_status, void *stream) {
  if (!sym_len || !sym_val || !d_nsym || !dc_diff || !d_index || !blocks || !d_status) return arg_error("null pointer");
  if (nblk <= 0 || nblk * 63 >= ((int64_t)1 << 31)) return arg_error("nblk");
  if ((reinterpret_cast<uintptr_t>(sym_len) | reinterpret_cast<uintptr_t>(sym_val) |
       reinterpret_cast<uintptr_t>(blocks)) % 16)
    return arg_error("symbol arrays and blocks must be 16-byte aligned");
  const int64_t ntiles = (nblk + 63) / 64;
  const dim3 grid((unsigned)((ntiles + 3) / 4)), block(256);
  if (knob(HIC_KNOB_RLD_NT) == 1)
    hipLaunchKernelGGL(k_rld_indexed16<true>, grid, block, 0, as_stream(stream), sym_len, sym_val, d_nsym, dc_diff, nblk,
                       d_index, blocks, d_status);
  else
    hipLaunchKernelGGL(k_rld_indexed16<false>, grid, block, 0, as_stream(stream), sym_len, sym_val, d_nsym, dc_diff,
                       nblk, d_index, blocks, d_status);
  return check_launch("k_rld_indexed16");
}

// ---- slot layout (slots.h) ----
namespace hic {
int64_t slot_rdc_word(int64_t nrec) { return rle_ws_words(nrec); }
}  // namespace hic

extern "C" size_t hic_rle_slots_workspace_bytes(int64_t nblk, int records_per_tile) {
  const int64_t nrec = slot_nrec(nblk > 0 ? nblk : 1, records_per_tile == 2 ? 2 : 1);
  return (size_t)(rle_ws_words(nrec) + (nrec + 1) / 2 + 2) * sizeof(int64_t);
}

// hic_slot_job[n] -> the scan / compaction jobs (validated, nothing launched on error)
static int slot_jobs(int n, const hic_slot_job *jobs, int max_len, bool compact, RleJobs16 &J) {
  if (n < 1 || n > kMaxJobs || !jobs) return arg_error("1 <= n <= %d jobs", kMaxJobs);
  if (max_len != 15) return arg_error("the slot layout needs max_len 15");
  J = RleJobs16{};
  J.n = n;
  J.M = max_len;
  for (int k = 0; k < n; ++k) {
    const hic_slot_job &a = jobs[k];
    if (!a.slot_len || !a.slot_val || !a.dc_diff || !a.d_index || !a.workspace || !a.d_count || !a.sym_len ||
        !a.sym_val)
      return arg_error("job %d: null pointer", k);
    if (a.nblk <= 0 || a.nblk > (int64_t)INT32_MAX / 63) return arg_error("job %d: nblk", k);
    if (a.records_per_tile != 1 && a.records_per_tile != 2) return arg_error("job %d: records_per_tile must be 1 or 2", k);
    const int64_t bpr = 64 / a.records_per_tile;
    if (a.nblk % bpr) return arg_error("job %d: nblk must be a multiple of %lld (whole records)", k, (long long)bpr);
    const int64_t need = (int64_t)hic_rle_slots_workspace_bytes(a.nblk, (int)a.records_per_tile);
    if (a.workspace_bytes < need)
      return arg_error("job %d: workspace of %lld bytes, %lld needed", k, (long long)a.workspace_bytes, (long long)need);
    RleJob16 &j = J.j[k];
    j = RleJob16{};
    j.nblk = a.nblk;
    j.dc_diff = a.dc_diff;
    j.sym_len = a.sym_len;
    j.sym_val = a.sym_val;
    j.cap = a.sym_cap;
    j.d_count = a.d_count;
    j.ws = static_cast<int64_t *>(a.workspace);
    j.rshift = a.records_per_tile == 2 ? 1 : 0;
    j.slot_len = a.slot_len;
    j.slot_val = a.slot_val;
    j.sidx = a.d_index;
    j.bpr = bpr;
    j.nrec = a.nblk / bpr;
    j.rdc = reinterpret_cast<int32_t *>(j.ws + rle_ws_words(j.nrec));
  }
  int64_t r0 = 0;  // tile0 / total_tiles count records here (the compaction's waves)
  for (int k = 0; k < n; ++k) {
    J.j[k].tile0 = r0;
    r0 += J.j[k].nrec;
  }
  J.total_tiles = r0;
  (void)compact;
  return HIC_OK;
}

extern "C" int hic_rle_slots_close(int n, const hic_slot_job *jobs, int max_len, void *stream) {
  RleJobs16 J;
  if (int e = slot_jobs(n, jobs, max_len, false, J)) return e;
  hipStream_t s = as_stream(stream);
  if (int e = scan_batch16<true>(J, s)) return e;
  hipLaunchKernelGGL(k_rle_scan_fold, dim3(1), dim3(64), 0, s, J);
  return check_launch("k_rle_scan_fold");
}

extern "C" int hic_rle_slots_compact(int n, const hic_slot_job *jobs, int max_len, void *stream) {
  RleJobs16 J;
  if (int e = slot_jobs(n, jobs, max_len, true, J)) return e;
  const int64_t waves = J.total_tiles < 16 * (int64_t)cu_count() ? J.total_tiles : 16 * (int64_t)cu_count();
  hipLaunchKernelGGL(k_rle_slots_compact, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, as_stream(stream), J);
  return check_launch("k_rle_slots_compact");
}

extern "C" int hic_rle_decode_i16_slots(const uint8_t *slot_len, const int16_t *slot_val, const int64_t *d_nsym,
                                        const int32_t *dc_diff, int64_t nblk, int records_per_tile,
                                        const int32_t *d_index, int16_t *blocks, int64_t *d_status, void *stream) {
  if (!slot_len || !slot_val || !d_nsym || !dc_diff || !d_index || !blocks || !d_status) return arg_error("null pointer");
  if (nblk <= 0 || nblk * 63 >= ((int64_t)1 << 31)) return arg_error("nblk");
  if (records_per_tile != 1 && records_per_tile != 2) return arg_error("records_per_tile must be 1 or 2");
  if (nblk % (64 / records_per_tile)) return arg_error("nblk must hold whole records");
  if ((reinterpret_cast<uintptr_t>(slot_len) | reinterpret_cast<uintptr_t>(slot_val) |
       reinterpret_cast<uintptr_t>(blocks)) % 16)
    return arg_error("slot arrays and blocks must be 16-byte aligned");
  const int64_t ntiles = (nblk + 63) / 64;
  hipLaunchKernelGGL((k_rld_indexed16<false, true>), dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0,
                     as_stream(stream), slot_len, slot_val, d_nsym, dc_diff, nblk,
                     reinterpret_cast<const int64_t *>(d_index), blocks, d_status, records_per_tile == 2 ? 1 : 0);
  return check_launch("k_rld_indexed16<slots>");
}

extern "C" int hic_rle_shard_summary_records(const int16_t *blocks, int64_t nblk, int records_per_tile,
                                             void *workspace, int64_t *d_summary, void *stream) {
  if (!blocks || !workspace || !d_summary) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (records_per_tile != 1 && records_per_tile != 2) return arg_error("records_per_tile must be 1 or 2");
  hipLaunchKernelGGL((k_rle_summary<int16_t>), dim3(1), dim3(kTB), 0, as_stream(stream), blocks, nblk,
                     block_geo(nblk, 64), static_cast<const int64_t *>(workspace),
                     (nblk * records_per_tile + kWT - 1) / kWT, d_summary);
  return check_launch("k_rle_summary");
}

extern "C" int hic_rle_shard_summary_tiles(const int16_t *blocks, int64_t nblk, void *workspace, int64_t *d_summary,
                                           void *stream) {
  return hic_rle_shard_summary_records(blocks, nblk, 1, workspace, d_summary, stream);
}

extern "C" int hic_rle_encode_i32(const int32_t *blocks, int64_t nblk, int block_len, int max_len,
                                  const int64_t *d_stitch, int32_t *dc_diff, int32_t *sym_len, int32_t *sym_val,
                                  int64_t sym_cap, int64_t *d_count, void *workspace, void *stream) {
  if (block_len < 2) return arg_error("block_len");
  if (!dc_diff) return arg_error("null dc_diff");
  return rle_encode(blocks, nblk, block_geo(nblk, block_len), max_len, d_stitch, dc_diff, sym_len, sym_val, sym_cap,
                    d_count, workspace, as_stream(stream));
}

extern "C" int hic_rle_stream_encode_i32(const int32_t *arr, int64_t n, int max_len, int32_t *sym_len,
                                         int32_t *sym_val, int64_t sym_cap, int64_t *d_count, void *workspace,
                                         void *stream) {
  // codec.run_length_coding on an arbitrary 1-D array (n may be 0: -> [EOB])
  static const int32_t kZero = 0;
  const int64_t nblk = n > 0 ? (n + 63) / 64 : 1;
  return rle_encode(n > 0 ? arr : &kZero, nblk, raw_geo(n), max_len, nullptr, nullptr, sym_len, sym_val, sym_cap,
                    d_count, workspace, as_stream(stream));
}

extern "C" int hic_rle_stitch(const int64_t *d_all_summaries, int world, int rank, int rank_stride, int64_t *d_stitch,
                              void *stream) {
  if (!d_all_summaries || !d_stitch) return arg_error("null pointer");
  if (world < 1 || rank < 0 || rank >= world || rank_stride < 4) return arg_error("world / rank / stride");
  hipLaunchKernelGGL(k_rle_stitch, dim3(1), dim3(64), 0, as_stream(stream), d_all_summaries, world, rank, rank_stride,
                     d_stitch);
  return check_launch("k_rle_stitch");
}

extern "C" size_t hic_rld_workspace_bytes(int64_t nsym, int64_t nblk) {
  // tile sums (symbol tiles, DC tiles), totals, last symbol; then the hot path's
  // integrated DC values (int16 x nblk)
  return (size_t)((nsym + kTS - 1) / kTS + (nblk + kTS - 1) / kTS + 8) * sizeof(int64_t) +
         (size_t)(nblk + 8) * sizeof(int16_t);
}

extern "C" int hic_rle_decode_i16(const uint8_t *sym_len, const int16_t *sym_val, int64_t nsym,
                                  const int32_t *dc_diff, int64_t nblk, int block_len, int16_t *blocks,
                                  int64_t *d_status, void *workspace, void *stream) {
  if (block_len < 2 || !dc_diff) return arg_error("block_len / dc_diff");
  if (block_len == 64 && nblk > 0 && nblk * 63 < ((int64_t)1 << 31) && nsym >= 0 && sym_len && sym_val && blocks &&
      d_status && workspace && reinterpret_cast<uintptr_t>(sym_len) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(sym_val) % 16 == 0 && reinterpret_cast<uintptr_t>(blocks) % 16 == 0 &&
      knob(HIC_KNOB_RLD_GENERIC) == 0)
    return rle_decode_blocks16(sym_len, sym_val, nsym, dc_diff, nblk, nullptr, blocks, d_status, workspace,
                               as_stream(stream));
  return rle_decode(sym_len, sym_val, nsym, dc_diff, nblk, block_geo(nblk, block_len), nblk * (block_len - 1), blocks,
                    d_status, workspace,
                    as_stream(stream));
}

extern "C" int hic_rle_decode_i16_shard(const uint8_t *sym_len, const int16_t *sym_val, int64_t nsym,
                                        const int32_t *dc_diff, int64_t nblk, const int64_t *d_stitch,
                                        int16_t *blocks, int64_t *d_status, void *workspace, void *stream) {
  if (!sym_len || !sym_val || !dc_diff || !d_stitch || !blocks || !d_status || !workspace)
    return arg_error("null pointer");
  if (nblk <= 0 || nblk * 63 >= ((int64_t)1 << 31) || nsym < 0) return arg_error("nblk / nsym");
  if (reinterpret_cast<uintptr_t>(sym_len) % 16 || reinterpret_cast<uintptr_t>(sym_val) % 16 ||
      reinterpret_cast<uintptr_t>(blocks) % 16)
    return arg_error("sym_len / sym_val / blocks must be 16-byte aligned");
  return rle_decode_blocks16(sym_len, sym_val, nsym, dc_diff, nblk, d_stitch, blocks, d_status, workspace,
                             as_stream(stream));
}

extern "C" int hic_rle_decode_i32(const int32_t *sym_len, const int32_t *sym_val, int64_t nsym,
                                  const int32_t *dc_diff, int64_t nblk, int block_len, int32_t *blocks,
                                  int64_t *d_status, void *workspace, void *stream) {
  if (block_len < 2 || !dc_diff) return arg_error("block_len / dc_diff");
  return rle_decode(sym_len, sym_val, nsym, dc_diff, nblk, block_geo(nblk, block_len), nblk * (block_len - 1), blocks,
                    d_status, workspace,
                    as_stream(stream));
}

extern "C" int hic_rle_stream_decode_i32(const int32_t *sym_len, const int32_t *sym_val, int64_t nsym, int64_t length,
                                         int32_t *out, int64_t out_cap, int64_t *d_status, void *workspace,
                                         void *stream) {
  // codec.decode_run_length: out[0:*d_status] is the decoded list; out has room for
  // out_cap >= max(length, sum(len+1)) elements, out_cap a multiple of 64.
  if (out_cap < 64 || out_cap % 64) return arg_error("out_cap must be a positive multiple of 64");
  if (length < 0) return arg_error("length");
  return rle_decode(sym_len, sym_val, nsym, nullptr, out_cap / 64, raw_geo(out_cap), length, out, d_status, workspace,
                    as_stream(stream));
}

extern "C" int hic_zigzag_blocks_i32(const int32_t *raster, int64_t H, int64_t W, int N, int32_t *out, void *stream) {
  if (!raster || !out) return arg_error("null pointer");
  if (H <= 0 || W <= 0 || N <= 0 || N > 256) return arg_error("shape / N");
  const int nbx = (int)((W + N - 1) / N), nby = (int)((H + N - 1) / N);
  const int64_t total = (int64_t)nbx * nby * N * N;
  hipLaunchKernelGGL(k_zigzag_i32, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), raster,
                     (int)H, (int)W, N, nbx, total, out);
  return check_launch("k_zigzag_i32");
}

extern "C" int hic_zigzag8_blocks_i16(const int32_t *raster, int64_t H, int64_t W, int16_t *out, int32_t *d_wide,
                                      void *stream) {
  if (!raster || !out || !d_wide) return arg_error("null pointer");
  if (H <= 0 || W <= 0 || H >= (1LL << 31) || W >= (1LL << 31)) return arg_error("shape");
  const int nbx = (int)((W + 7) / 8), nby = (int)((H + 7) / 8);
  const int64_t total = (int64_t)nbx * nby * 64;
  hipStream_t s = as_stream(stream);
  if (int e = hip_status(hipMemsetAsync(d_wide, 0, 4, s), "hipMemsetAsync")) return e;
  hipLaunchKernelGGL(k_zigzag8_i16, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, raster, (int)H, (int)W,
                     nbx, total, out, d_wide);
  return check_launch("k_zigzag8_i16");
}

extern "C" int hic_izigzag_blocks_i32(const int32_t *blocks, int64_t H, int64_t W, int N, int32_t *raster,
                                      void *stream) {
  if (!raster || !blocks) return arg_error("null pointer");
  if (H <= 0 || W <= 0 || N <= 0 || N > 256) return arg_error("shape / N");
  const int nbx = (int)((W + N - 1) / N), nby = (int)((H + N - 1) / N);
  const int64_t total = (int64_t)nbx * nby * N * N;
  hipLaunchKernelGGL(k_izigzag_i32, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), blocks,
                     (int)H, (int)W, N, nbx, total, raster);
  return check_launch("k_izigzag_i32");
}
