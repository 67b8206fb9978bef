// onepass.h -- the stream hand-off of the one-pass encode (k_encode420<TMF, false,
// true>, hic_encode420_rle_u8): a unit's pass publishes its RLE record's aggregate,
// takes the aggregate of every earlier record of its plane by a decoupled look-back,
// publishes its inclusive prefix, and emits the DC differences and AC symbols of
// its blocks from the unit's LDS stage -- no coefficient re-read, no scan launch.
//
// Reference: codec.differential_coding (codec.py:47-52) and codec.run_length_coding
// (codec.py:55-99) over the plane's AC stream (slots 1..63 of every block, blocks
// in raster order); the record algebra (first / last nonzero, symbols after the
// first) is the scan's (rle.hip: Agg, agg_combine), the emission emit_tile16's.
//
// Look-back (one record = one 64-block Y tile, or one 32-block Cr / Cb half tile):
// record r of a plane owns 8 granules at gran[8 r]: its aggregate A {first, last,
// cnt, dc of its last block} and its inclusive prefix P {first, last, cnt, dc},
// each value a 32-bit int in an 8-byte word with a 32-bit tag (agent-scope atomic
// stores / loads: cross-XCD coherent, no fences).  Tags are (epoch << 2) | 1 for A,
// | 2 for P, | 3 for the launch's failure word; the epoch is unique per launch
// (hic_next_epoch), so stale granules never match and the workspace needs no reset.
// A wave reads a window of 64 (32 per chroma plane) earlier records at once, waits
// until every record up to the nearest P has at least its A, and folds them in
// record order.  Progress: a unit publishes A before it waits on anything, and
// units take their tickets in dispatch order, so every record a waiting wave needs
// belongs to a wave that is running or done.  A bounded spin reports
// HIC_COUNT_SCAN_TIMEOUT instead of hanging.
#pragma once
#include "rle_core.h"

namespace hic {
namespace {

__device__ __forceinline__ void op_put(uint64_t *g, int v, uint32_t tag) {
  __hip_atomic_store(g, (uint64_t)(uint32_t)v | ((uint64_t)tag << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t op_get(const uint64_t *g) {
  return __hip_atomic_load(const_cast<uint64_t *>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a record's aggregate: AC stream positions of its first / last nonzero (-1: none)
// and the symbols of every nonzero after its first (int32: the host bounds a
// plane's AC stream below 2^31)
struct Agg32 {
  int first, last, cnt;
};
__device__ __forceinline__ Agg32 agg32(const Agg32 &A, const Agg32 &B, int M) {
  if (B.last < 0) return A;
  if (A.last < 0) return B;
  return Agg32{A.first, B.last, A.cnt + B.cnt + syms_for_run(B.first - A.last - 1, M)};
}

constexpr int kOpSpin = 1 << 22;  // look-back polls before a launch reports a timeout

// spin-wait helper: back off, a wave far ahead of the published prefixes polls less
__device__ __forceinline__ void op_backoff(int spin) {
  if (spin < 4)
    __builtin_amdgcn_s_sleep(4);
  else if (spin < 32)
    __builtin_amdgcn_s_sleep(16);
  else
    __builtin_amdgcn_s_sleep(64);
}

// fold of lanes sl = 0 .. S-1 of a segment (lane sl holds the sl-th item counting
// back from the newest; lanes past the wanted ones hold the empty aggregate): the
// segment's items folded in stream order, in every lane of the segment
template <int S>
__device__ __forceinline__ Agg32 op_fold(Agg32 v, int sl, int M) {
#pragma unroll
  for (int d = 1; d < S; d <<= 1) {
    const Agg32 o{__shfl_down(v.first, d, S), __shfl_down(v.last, d, S), __shfl_down(v.cnt, d, S)};
    if ((sl & (2 * d - 1)) == 0) v = agg32(o, v, M);
  }
  return Agg32{__shfl(v.first, 0, S), __shfl(v.last, 0, S), __shfl(v.cnt, 0, S)};
}

// granule group {value0..3} with tag t at r (4 words): all four tags must match
__device__ __forceinline__ bool op_read4(const uint64_t *r, uint32_t t, Agg32 &v, int &dc) {
  uint64_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = op_get(r + k);
  const bool ok = ((uint32_t)(w[0] >> 32) == t) & ((uint32_t)(w[1] >> 32) == t) & ((uint32_t)(w[2] >> 32) == t) &
                  ((uint32_t)(w[3] >> 32) == t);
  if (ok) {
    v = Agg32{(int)(uint32_t)w[0], (int)(uint32_t)w[1], (int)(uint32_t)w[2]};
    dc = (int)(uint32_t)w[3];
  }
  return ok;
}

// nearest lane of this segment (32 lanes if SEG) with `has` (S if none)
template <bool SEG>
__device__ __forceinline__ int op_nearest(bool has) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(has);
  if (SEG) {
    const uint32_t h = (uint32_t)(m >> ((threadIdx.x & 63) & 32));
    return h ? __builtin_ctz(h) : 32;
  }
  return m ? __builtin_ctzll(m) : 64;
}

// The look-back windows are the image's unit rows: window u holds the records of
// unit row u in stream order -- Y: rows 2u and 2u + 1 of the plane's tiles (2 ns
// records, offsets 0 .. ns - 1 and ns .. 2 ns - 1), Cr / Cb: ns half tiles.  All
// records of a window belong to the ns units of one unit row, which start together;
// the row's last unit publishes the window's aggregate WA as soon as its row-mates'
// aggregates are out, BEFORE any look-back of its own (published from inside its
// look-back, WA waited on that unit's earlier emissions and chained the rows: 3.1 ms
// per 8K image).
__device__ __forceinline__ int op_rec(int u, int o, int ns, bool luma) {
  return luma ? (o < ns ? 2 * u * ns + o : (2 * u + 1) * ns + o - ns) : u * ns + o;
}

// WA of window u (this lane's plane), by the unit holding its last record (mine,
// mydc: that record's aggregate and last DC): the window-mates' aggregates, folded.
// Returns false on a timeout.
template <bool SEG>
__device__ __forceinline__ bool op_publish_wa(const uint64_t *g, uint64_t *gw, int u, int ns, bool luma,
                                              uint32_t tagA, uint32_t tagW, int M, const Agg32 &mine, int mydc) {
  constexpr int S = SEG ? 32 : 64;
  const int lane = threadIdx.x & 63, sl = lane & (S - 1);
  const int o = (luma ? 2 * ns : ns) - 1;  // the last record's offset
  Agg32 va{-1, -1, 0};
  int dca = 0;
  bool ha = !(sl < o);
  for (int spin = 0;; ++spin) {
    if (!ha) ha = op_read4(g + 8 * (int64_t)op_rec(u, o - 1 - sl, ns, luma), tagA, va, dca);
    if (__builtin_amdgcn_ballot_w64(!ha) == 0) break;
    if (spin >= kOpSpin) return false;
    op_backoff(spin);
  }
  const Agg32 wa = agg32(op_fold<S>(va, sl, M), mine, M);
  if (sl < 4) op_put(gw + 4 * (int64_t)u + sl, sl == 0 ? wa.first : sl == 1 ? wa.last : sl == 2 ? wa.cnt : mydc, tagW);
  return true;
}

// Exclusive aggregate of the record at offset o of window u (this lane's plane:
// record granules g, window granules gw) and the DC of the record before it (0 at
// the plane's start).  SEG: lanes 0-31 and 32-63 look back in two planes at once
// (u, o uniform).
//  1. the window's earlier records (one lane each, one poll when published): their
//     nearest P ends the look-back;
//  2. else the earlier windows (one lane each, 64 / 32 per poll): a window whose last
//     record has P ends it, any other contributes its WA.
// A launch's first waves reach their look-backs together, far from any P; a
// record-by-record walk back cost them ~110 us per 8K image (profiles/r04/onepass).
// Only lanes still missing their granules poll again.  Returns false on a timeout.
template <bool SEG>
__device__ __forceinline__ bool op_lookback(const uint64_t *g, uint64_t *gw, int u, int o, int ns, bool luma,
                                            uint32_t tagA, uint32_t tagP, uint32_t tagW, int M, Agg32 &excl,
                                            int &prevdc) {
  constexpr int S = SEG ? 32 : 64;
  const int lane = threadIdx.x & 63, sl = lane & (S - 1);
  const int wn = luma ? 2 * ns : ns;  // records per window (<= S)
  const Agg32 none{-1, -1, 0};
  // ---- 1. the window's earlier records: lane sl holds offset o - 1 - sl
  Agg32 va = none, vp = none;
  int dca = 0, dcp = 0, lp = o;
  bool ha = false, hp = false;
  for (int spin = 0;; ++spin) {
    if (sl < o && !ha) {  // a lane with the aggregate needs nothing more
      const uint64_t *r = g + 8 * (int64_t)op_rec(u, o - 1 - sl, ns, luma);
      if (!hp) hp = op_read4(r + 4, tagP, vp, dcp);
      ha = op_read4(r, tagA, va, dca);
    }
    const int np = op_nearest<SEG>(hp && sl < o);
    lp = np < o ? np : o;
    // the aggregates up to the nearest P
    if (__builtin_amdgcn_ballot_w64(!ha && sl < lp) == 0) break;
    if (spin >= kOpSpin) return false;
    op_backoff(spin);
  }
  int pdc = __shfl(ha ? dca : dcp, 0, S);  // the previous record's last DC (o > 0)
  const Agg32 own = op_fold<S>(sl < lp ? va : (sl == lp && lp < o ? vp : none), sl, M);
  if (lp < o) {
    excl = own;
    prevdc = pdc;
    return true;
  }
  // ---- 2. earlier windows: lane sl holds window q - sl (its last record's P, or WA)
  Agg32 acc = own;
  int q = u - 1;
  bool done = q < 0, first_win = true;
  while (__builtin_amdgcn_ballot_w64(!done) != 0) {
    const int iw = q - sl;
    const bool live = !done && iw >= 0;
    Agg32 v = none;
    int dcv = 0, lq = S;
    bool hw = false, hq = !live;  // hq: the window's P (windows before the stream: empty)
    for (int spin = 0;; ++spin) {
      if (live && !hq && !hw) {
        hq = op_read4(g + 8 * (int64_t)op_rec(iw, wn - 1, ns, luma) + 4, tagP, v, dcv);
        if (!hq) hw = op_read4(gw + 4 * (int64_t)iw, tagW, v, dcv);
      }
      lq = op_nearest<SEG>(hq);
      if (__builtin_amdgcn_ballot_w64(!hq && !hw && sl < lq) == 0) break;
      if (spin >= kOpSpin) return false;
      op_backoff(spin);
    }
    if (first_win) {
      if (o == 0) pdc = __shfl(dcv, 0, S);  // the previous window's last DC
      first_win = false;
    }
    const Agg32 W = op_fold<S>(sl > lq ? none : v, sl, M);
    if (!done) acc = agg32(W, acc, M);
    done = done || lq < S;
    q -= S;
  }
  excl = acc;
  prevdc = pdc;
  return true;
}

constexpr int kOpSyms = 2048;  // staged symbols per half pass (32 blocks hold <= 2016)

// 64-bit readlane (lane uniform)
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Emission of one pass: lane l's block (w: its zig-zag words; blk: the same block
// in the LDS stage, read at lane-varying indices; bpos: the stream position of its
// AC 0) after the record's look-back.  o_seg / prev_seg (uniform per segment): the
// output position of the segment's first symbol and the stream position of the
// last nonzero before it (-1: none).  SEG: lanes 0-31 write stream 0, 32-63 stream
// 1; else one stream (both the same).  The 32 lanes of a half stage their symbols
// in s_len / s_val (kOpSyms + 32 each) at their stream-relative positions, then
// the wave copies the contiguous range out in 16-byte stores (emit_tile16's scheme
// in two halves: the LDS of a 2-wave-per-SIMD unit holds 2048 staged symbols); a
// half with more (a nonzero after a long carried zero run) writes directly.
template <int MF, bool SEG>
__device__ __forceinline__ void op_emit(const uint32_t (&w)[32], const int16_t *blk, int64_t bpos, int M,
                                        int64_t o_seg, int64_t prev_seg, int first, int last, int nsym, uint64_t ac,
                                        uint8_t *s_len, int16_t *s_val, uint8_t *len0, int16_t *val0, int64_t cap0,
                                        uint8_t *len1, int16_t *val1, int64_t cap1) {
  const int lane = threadIdx.x & 63, sl = SEG ? lane & 31 : lane;
  const int lastr = last >= 0 ? sl * 63 + last : -1;
  const int incl = SEG ? seg32_incl_max_i32(lastr) : wave_incl_max_i32(lastr);
  int prevr = wave_shr1_i32(-1, incl);
  if (sl == 0) prevr = -1;
  const int64_t prev = prevr >= 0 ? bpos - sl * 63 + prevr : prev_seg;
  const int64_t run0 = bpos + first - prev - 1;  // carried run before the first nonzero
  const int cnt = first >= 0 ? nsym + syms_for_run(run0, M) : 0;
  const int icnt = SEG ? seg32_incl_sum_i32(cnt) : wave_incl_sum_i32(cnt);
  const int64_t o_thr = o_seg + icnt - cnt;
  const bool dense = nsym == __builtin_popcountll(ac) - 1;  // no run >= max_len inside the block
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint8_t *const sym_len = h ? len1 : len0;
    int16_t *const sym_val = h ? val1 : val0;
    const int64_t cap = h ? cap1 : cap0;
    const bool mine = (lane >> 5) == h;
    const int64_t hb = readlane64(o_thr, 32 * h), he = readlane64(o_thr + cnt, 32 * h + 31);
    const int n = (int)(he - hb);
    const bool staged = n <= kOpSyms;  // wave-uniform
    const int lo = (int)(hb & 15), vo = (int)(hb & 7);
    int64_t nf0 = 0;
    if (mine && first >= 0) {
      int64_t o = o_thr;
      const int64_t nf = div_run(run0, M);
      const int rem = (int)(run0 - nf * M);
      if (staged) {
        int r = (int)(o - hb);
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
        // one symbol per nonzero from the first, branch-free (emit_tile16): a zero
        // coefficient writes the stage's dummy slot and does not advance
        typedef __attribute__((address_space(3))) uint8_t lds_u8;
        typedef __attribute__((address_space(3))) int16_t lds_i16;
        const uint32_t lbase = (uint32_t)(uintptr_t)(lds_u8 *)s_len;
        const uint32_t vshift = (uint32_t)(uintptr_t)(lds_i16 *)s_val + 2u * (uint32_t)(vo - lo) - 2u * lbase;
        const uint32_t ldummy = lbase + kOpSyms + 16;
        uint32_t la = lbase + (uint32_t)((int)(o - hb) + lo);
        int pl = first - 1 - rem;
#pragma unroll
        for (int j = 0; j < 63; ++j) {
          const int v = zz_ac(w, j);
          const bool nz = v != 0;
          const uint32_t a = nz ? la : ldummy;
          *(lds_u8 *)(uintptr_t)a = (uint8_t)(j - pl - 1);
          uint32_t va;
          asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(va) : "v"(a), "v"(vshift));
          *(lds_i16 *)(uintptr_t)va = (int16_t)v;
          la += nz ? 1u : 0u;
          pl = nz ? j : pl;
        }
      } else if (staged) {
        int r = (int)(o - hb);
        int pl = first;
        for (uint64_t m = ac & (ac - 1); m; m &= m - 1) {  // nonzeros after the first
          const int j = __builtin_ctzll(m);
          const int v = blk[1 + j];
          int run = j - pl - 1;
          const int nfi = div_m<MF>(run, M);
          for (int f = 0; f < nfi; ++f, ++r) {
            s_len[lo + r] = (uint8_t)(M - 1);
            s_val[vo + r] = 0;
          }
          run -= nfi * M;
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
          const int nfi = run / M;
          for (int k = 0; k < nfi; ++k, ++o)
            if (o < cap) {
              sym_len[o] = (uint8_t)(M - 1);
              sym_val[o] = 0;
            }
          run -= nfi * M;
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
    if (staged) {
      copy_out_wave16<uint8_t, true>(s_len, lo, sym_len, hb, n, cap);
      copy_out_wave16<int16_t, true>(s_val, vo, sym_val, hb, n, cap);
    } else {
      // long carried runs: the whole wave writes each lane's fillers
      uint64_t m = __builtin_amdgcn_ballot_w64(mine && nf0 > 0);
      while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        const int64_t s0 = readlane64(o_thr, l), nf = readlane64(nf0, l);
        for (int64_t k = lane; k < nf; k += 64)
          if (s0 + k < cap) {
            sym_len[s0 + k] = (uint8_t)(M - 1);
            sym_val[s0 + k] = 0;
          }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace
}  // namespace hic
