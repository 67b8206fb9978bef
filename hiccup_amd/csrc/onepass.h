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

// Exclusive aggregate of record `rec` of this lane's plane (granules g) and the DC
// of record rec - 1's last block (0 for rec 0).  SEG: lanes 0-31 and 32-63 look
// back in two planes at once (rec uniform per half).  Returns false on a timeout.
template <bool SEG>
__device__ __forceinline__ bool op_lookback(const uint64_t *g, int rec, uint32_t tagA, uint32_t tagP, int M,
                                            Agg32 &excl, int &prevdc) {
  constexpr int S = SEG ? 32 : 64;
  const int lane = threadIdx.x & 63, sl = lane & (S - 1), hf = SEG ? lane >> 5 : 0;
  Agg32 acc{-1, -1, 0};
  int pdc = 0;
  bool ok = true, first_win = true;
  int q = rec - 1;  // newest record of this segment's window
  bool done = q < 0;
  while (__builtin_amdgcn_ballot_w64(!done) != 0) {
    const int idx = q - sl;
    Agg32 v{-1, -1, 0};
    int dcv = 0, lp = S;
    for (int spin = 0;; ++spin) {
      // records before the stream (and finished segments) read as the empty prefix
      int st = 2;
      v = Agg32{-1, -1, 0};
      dcv = 0;
      if (!done && idx >= 0) {
        const uint64_t *r = g + 8 * (int64_t)idx;
        uint64_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = op_get(r + k);
        auto tags = [&](int k0, uint32_t t) {
          return ((uint32_t)(w[k0] >> 32) == t) & ((uint32_t)(w[k0 + 1] >> 32) == t) &
                 ((uint32_t)(w[k0 + 2] >> 32) == t) & ((uint32_t)(w[k0 + 3] >> 32) == t);
        };
        if (tags(4, tagP)) {
          st = 2;
          v = Agg32{(int)(uint32_t)w[4], (int)(uint32_t)w[5], (int)(uint32_t)w[6]};
          dcv = (int)(uint32_t)w[7];
        } else if (tags(0, tagA)) {
          st = 1;
          v = Agg32{(int)(uint32_t)w[0], (int)(uint32_t)w[1], (int)(uint32_t)w[2]};
          dcv = (int)(uint32_t)w[3];
        } else {
          st = 0;
        }
      }
      const uint64_t pm = __builtin_amdgcn_ballot_w64(st == 2);
      if (SEG) {
        const uint32_t ph = (uint32_t)(pm >> (32 * hf));
        lp = ph ? __builtin_ctz(ph) : 32;
      } else {
        lp = pm ? __builtin_ctzll(pm) : 64;
      }
      if (__builtin_amdgcn_ballot_w64(st == 0 && sl < lp) == 0) break;
      if (spin >= kOpSpin) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) break;
    if (first_win) {  // record rec - 1 (this segment's lane 0)
      pdc = __shfl(dcv, 0, S);
      first_win = false;
    }
    if (sl > lp) v = Agg32{-1, -1, 0};
    // lane sl holds record q - sl: fold toward sl = 0, earlier records on the left
#pragma unroll
    for (int d = 1; d < S; d <<= 1) {
      const Agg32 o{__shfl_down(v.first, d, S), __shfl_down(v.last, d, S), __shfl_down(v.cnt, d, S)};
      if ((sl & (2 * d - 1)) == 0) v = agg32(o, v, M);
    }
    const Agg32 W{__shfl(v.first, 0, S), __shfl(v.last, 0, S), __shfl(v.cnt, 0, S)};
    if (!done) acc = agg32(W, acc, M);
    done = done || lp < S;
    q -= S;
  }
  excl = acc;
  prevdc = pdc;
  return ok;
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
