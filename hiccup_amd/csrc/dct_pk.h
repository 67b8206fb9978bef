// dct_pk.h -- the packed-float32 forward 8x8 DCT + quantiser of aligned planes
// (k_dct_pk in dct.hip; DESIGN.md section 5 "Packed float32 plane DCT, round 5").
//
// Reference: transform.dct_channel (transform.py:182-193) = dct2 (:67-84, scipy's
// pocketfft DCT-II) + jpeg_quantize (quantization.py:47-52: round-half-even(y / T)).
//
// One 8x8 block per lane.  The Arai-Agui-Nakajima 8-point DCT runs in float32 on
// <2 x float> pairs, one v_pk_{add,mul,fma}_f32 for two transforms: the row pass
// pairs rows (2m, 2m + 1) of the block, the column pass pairs columns (v, v + 2)
// (a 2 x 2 transpose of the row outputs between the passes).  Every element
// operation is that of aan() in tools/check/dct_bounds.py, so the proven float32
// error bounds E1 (dct_windows.h: kR32 quantiser constants, kThr32Sq flag
// thresholds) hold: per coefficient,
//     t = fma(Y, R, 1.5 2^23)      the low 16 bits of t's bits are rint(Y R)
//     d = fma(Y, R, 1.5 2^23 - t)  = Y R - rint(Y R), exact to 2^-25
//     g = fma(-d, d, thr^2)        negative iff |d| > thr: the coefficient's
//                                  rint may differ from numpy's rint(fl(y / T))
// and g's sign bit is OR-ed into the lane's flag word.  (0,0) is the exact raw-byte
// sum, rounded in integers (dc_quant); luminance (4,4) is y/T = K/34, flagged only
// at its exact ties, which pocketfft's own roundings decide in place (pf_y44 on the
// rows' integer outputs 4).  Any other flag (~0.035 per luminance block on random
// data, dct_bounds.py) sends the lane's block through pk_coop_redo_k: the whole wave
// recomputes that one block in float64 (dct_coef_f64's separable, symmetry-folded
// dot products, error window E2 <= 2^-31, lane = coefficient) and patches its
// stage row before the set leaves.  A coefficient inside E2's window too (an exact
// (2,2)-class tie, ~1e-4 per block) marks the set for the exact pocketfft replica
// after the loop.
#pragma once
#include "dct_core.h"

namespace hic {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pkf(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 sp2(float k) { return (f2){k, k}; }
__device__ __forceinline__ uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }

// float32 roundings of the AAN constants (dct_bounds.py takes |K - c| <= 2^-24 |c|;
// tests/test_dct_bounds.py checks these four)
constexpr float kA1f = (float)kA1, kA2f = (float)kA2, kA4f = (float)kA4, kA5f = (float)kA5;
constexpr float kMagic32 = 0x1.8p23f;  // fl(e + 1.5 2^23) = 1.5 2^23 + rint(e) for |e| < 2^22

// AAN even half (outputs 0, 2, 4, 6) from s_k = x_k + x_{7-k}, and odd half
// (outputs 1, 3, 5, 7) from d7 = x0 - x7, d6 = x1 - x6, d5 = x2 - x5, d4 = x3 - x4:
// aan() of dct_bounds.py, element for element
__device__ __forceinline__ void pk_even(f2 s0, f2 s1, f2 s2, f2 s3, f2 &o0, f2 &o2, f2 &o4, f2 &o6) {
  const f2 t10 = s0 + s3, t13 = s0 - s3, t11 = s1 + s2, t12 = s1 - s2;
  const f2 w = t12 + t13;
  o0 = t10 + t11;
  o4 = t10 - t11;
  o2 = pkf(sp2(kA1f), w, t13);
  o6 = pkf(sp2(-kA1f), w, t13);
}
__device__ __forceinline__ void pk_odd(f2 d7, f2 d6, f2 d5, f2 d4, f2 &o1, f2 &o3, f2 &o5, f2 &o7) {
  const f2 u10 = d4 + d5, u11 = d5 + d6, u12 = d6 + d7;
  const f2 z5 = (u10 - u12) * sp2(kA5f);
  const f2 z2 = pkf(sp2(kA2f), u10, z5), z4 = pkf(sp2(kA4f), u12, z5);
  const f2 z11 = pkf(sp2(kA1f), u11, d7), z13 = pkf(sp2(-kA1f), u11, d7);
  o5 = z13 + z2;
  o3 = z13 - z2;
  o1 = z11 + z4;
  o7 = z11 - z4;
}

// byte n of an 8-byte pixel row as float (v_cvt_f32_ubyte<n>)
__device__ __forceinline__ float pxf(uint2 r, int n) {
  return (float)(((n < 4 ? r.x : r.y) >> (8 * (n & 3))) & 0xFFu);
}

// Row pass of rows (2m, 2m + 1): o[k] = (row 2m's output k, row 2m + 1's output k)
__device__ __forceinline__ void pk_rows(uint2 ra, uint2 rb, f2 (&o)[8]) {
  f2 x[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) x[n] = (f2){pxf(ra, n), pxf(rb, n)};
  pk_even(x[0] + x[7], x[1] + x[6], x[2] + x[5], x[3] + x[4], o[0], o[2], o[4], o[6]);
  pk_odd(x[0] - x[7], x[1] - x[6], x[2] - x[5], x[3] - x[4], o[1], o[3], o[5], o[7]);
}

// Column pass of one column pair: X[r] = (row r's output v, row r's output v + 2)
__device__ __forceinline__ void pk_cols(const f2 (&X)[8], f2 (&Y)[8]) {
  pk_even(X[0] + X[7], X[1] + X[6], X[2] + X[5], X[3] + X[4], Y[0], Y[2], Y[4], Y[6]);
  pk_odd(X[0] - X[7], X[1] - X[6], X[2] - X[5], X[3] - X[4], Y[1], Y[3], Y[5], Y[7]);
}

// The per-lane constants of the cooperative float64 redo (pk_coop_redo_k): the
// separable fallback's factors C_k(n) = 2 cos(pi k (2n + 1) / 16) (dct_coef_f64's
// cos2(kCm, k, n), k = 0..7, n = 0..3) and 1 / T per table, correctly rounded
struct PkRedoTab {
  double c[8][4];
  double rt[2][64];
  constexpr PkRedoTab() : c(), rt() {
    for (int k = 0; k < 8; ++k)
      for (int n = 0; n < 4; ++n) {
        int m = (k * (2 * n + 1)) & 31;
        if (m > 16) m = 32 - m;
        const bool neg = m > 8;
        const double v = kCm[neg ? 16 - m : m];
        c[k][n] = neg ? -v : v;
      }
    for (int t = 0; t < 2; ++t)
      for (int i = 0; i < 64; ++i) rt[t][i] = 1.0 / (double)QT[t][i];
  }
};
__device__ const PkRedoTab kPkRedo{};
// zig-zag slot of raster index i (lane i of the cooperative redo: its (u, v) slot)
__device__ const SlotOf<HIC_LAYOUT_ZIGZAG_I16> kPkSlot{};

// K flagged blocks of the wave's set, each recomputed by the whole wave in float64
// and written over its stage row: lane (m, v) = (lane >> 3, lane & 7) forms
// dct_coef_f64's row sum r_mv from pixel row m of block j (px[j]), the rows' sums
// cross lanes by ds_bpermute, and lane (u, v) = (lane >> 3, lane & 7) folds them
// into y_uv with the same operations, in the same order, as dct_coef_f64 (the E2
// bound of dct_bounds.py) and quantises y / T with the E2 window
// (quant_f64_window).  The DC (exact in the fast path) and, for luminance, (4,4)
// (decided in place) are not rewritten.  stage_row[j]: block j's stage row;
// slot_off: this lane's (u, v) byte offset in a stage row.  The redo of one block is
// a chain of LDS and cross-lane latencies (pixel rows in, the row sums across
// lanes); K independent chains share that wait.  Returns false (wave-uniform) if
// some coefficient lies inside the E2 window: only the exact pocketfft replica
// decides it (the caller redoes the set or block).
template <int K>
__device__ __forceinline__ bool pk_coop_redo_k(const uint2 (&px)[K], int table, int16_t *const (&stage_row)[K],
                                               int slot_off, int lane, const PkRedoTab &tab) {
  const int m = lane >> 3, v = lane & 7;
  // branch-free: odd v takes a_n = x_n - x_{7-n}, even v a_n = x_n + x_{7-n} - 256 (a
  // bit select between the two, each one byte-select add); the DC and (luminance)
  // (4,4) lanes write their value into the stage row's pad instead of their slot
  const uint32_t vm = (v & 1) ? ~0u : 0u;
  const bool keep = lane == 0 || (lane == 36 && table == 0);
  const int woff = keep ? 2 * 64 : slot_off;
  double cv[4], cu[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    cv[n] = tab.c[v][n];
    cu[n] = tab.c[m][n];
  }
  const double rt = tab.rt[table][lane];
  double r[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const uint32_t xn = (px[j].x >> (8 * n)) & 0xFFu, yn = (px[j].y >> (8 * (3 - n))) & 0xFFu;
      const uint32_t sum = xn + yn - 256u, dif = xn - yn;
      const int a = (int)((vm & dif) | (~vm & sum));
      r[j] = n == 0 ? (double)a * cv[0] : __builtin_fma((double)a, cv[n], r[j]);
    }
  }
  double rm[K][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int src = (8 * k + v) * 4;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint64_t rb = __builtin_bit_cast(uint64_t, r[j]);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)rb);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(rb >> 32));
      rm[j][k] = __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
    }
  }
  const double su = (m & 1) ? -1.0 : 1.0;
  uint32_t bad = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double y = __builtin_fma(su, rm[j][7], rm[j][0]) * cu[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) y = __builtin_fma(__builtin_fma(su, rm[j][7 - k], rm[j][k]), cu[k], y);
    const unsigned long long t =
        __builtin_bit_cast(unsigned long long, __builtin_fma(y, rt, 0x1.8p20 + 0.5 + 0x1p-30));
    const int q = (int)((uint32_t)(t >> 32) - kQHi);
    bad |= (uint32_t)t <= 9u;
    *reinterpret_cast<int16_t *>(reinterpret_cast<uint8_t *>(stage_row[j]) + woff) = (int16_t)q;
  }
  return __builtin_amdgcn_ballot_w64(bad != 0 && !keep) == 0;
}

// Every flagged block of a wave's 64 (fb: bit L = lane L's block; w: this lane's
// pixel rows) redone by pk_coop_redo_k two at a time; s_px: the wave's 128-byte LDS
// area for the pixel rows in flight; st2: the wave's stage.  s_tab_d: the
// workgroup's LDS copy of kPkRedo, filled here by this wave on its first call
// (tab_ready: wave-uniform; waves write identical values, so no barrier; s_slot,
// when given, gets kPkSlot's 64 slots the same way).  Returns false if some block
// needs the exact replica.
__device__ __forceinline__ void pk_tab_fill(double *s_tab_d, uint8_t *s_slot, int lane, bool &tab_ready) {
  if (tab_ready) return;
  const double *src = &kPkRedo.c[0][0];
#pragma unroll
  for (int k = 0; k < (int)(sizeof(PkRedoTab) / sizeof(double)); k += 64)
    if (k + lane < (int)(sizeof(PkRedoTab) / sizeof(double))) s_tab_d[k + lane] = src[k + lane];
  if (s_slot) s_slot[lane] = (uint8_t)kPkSlot.s[lane];
  __builtin_amdgcn_wave_barrier();
  tab_ready = true;
}
__device__ __forceinline__ bool pk_redo_flagged(uint64_t fb, const uint2 (&w)[8], uint2 *s_px, uint2 *st2,
                                                int stage_u2, int table, int slot_off, int lane, double *s_tab_d,
                                                bool &tab_ready) {
  pk_tab_fill(s_tab_d, nullptr, lane, tab_ready);
  const PkRedoTab &tab = *reinterpret_cast<const PkRedoTab *>(s_tab_d);
  bool ok = true;
  while (fb) {
    const int L0 = __builtin_ctzll(fb);
    fb &= fb - 1;
    __builtin_amdgcn_wave_barrier();
    if (fb) {
      const int L1 = __builtin_ctzll(fb);
      fb &= fb - 1;
      if (lane == L0 || lane == L1) {
        uint2 *d = s_px + (lane == L0 ? 0 : 8);
#pragma unroll
        for (int r = 0; r < 8; ++r) d[r] = w[r];
      }
      __builtin_amdgcn_wave_barrier();
      const uint2 px[2] = {s_px[lane >> 3], s_px[8 + (lane >> 3)]};
      __builtin_amdgcn_wave_barrier();
      int16_t *const rows[2] = {reinterpret_cast<int16_t *>(st2 + L0 * stage_u2),
                                reinterpret_cast<int16_t *>(st2 + L1 * stage_u2)};
      ok = pk_coop_redo_k<2>(px, table, rows, slot_off, lane, tab) && ok;
    } else {
      if (lane == L0) {
#pragma unroll
        for (int r = 0; r < 8; ++r) s_px[r] = w[r];
      }
      __builtin_amdgcn_wave_barrier();
      const uint2 px[1] = {s_px[lane >> 3]};
      __builtin_amdgcn_wave_barrier();
      int16_t *const rows[1] = {reinterpret_cast<int16_t *>(st2 + L0 * stage_u2)};
      ok = pk_coop_redo_k<1>(px, table, rows, slot_off, lane, tab) && ok;
    }
  }
  return ok;
}

// Quantise column pair (v0, v0 + 2) (Y[u]: the pair's column outputs u) into the
// lane's stage row; OR the flag bits of its coefficients into fl, and (TABLE 0) the
// (4,4) flag into t44 instead (an exact tie there, decided by the caller)
template <int TABLE>
__device__ __forceinline__ void pk_quant_pair(const f2 (&Y)[8], int v0, int16_t *st, f2 kM2, uint32_t &fl,
                                              uint32_t &t44) {
  constexpr SlotOf<HIC_LAYOUT_ZIGZAG_I16> kSlot{};
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int i0 = 8 * u + v0, i1 = i0 + 2;
    const f2 Rq = (f2){kR32[TABLE][i0], kR32[TABLE][i1]};
    const f2 Tq = (f2){kThr32Sq[TABLE][i0], kThr32Sq[TABLE][i1]};
    const f2 tq = pkf(Y[u], Rq, kM2);
#if defined(HIC_DEV) && defined(HIC_PK_DEV) && (HIC_PK_DEV & 4)
    const f2 gq = Tq;  // dev timing (results invalid): no flag arithmetic
#else
    const f2 d = pkf(Y[u], Rq, kM2 - tq);
    const f2 gq = pkf(-d, d, Tq);
#endif
    st[kSlot.s[i1]] = (int16_t)(fbits(tq.y) & 0xFFFFu);
    if (i0 == 0) {
      // DC: Y = the raw-byte sum of the block (exact); y00 = 4 (Y - 64 * 128)
      st[kSlot.s[0]] = (int16_t)dc_quant<TABLE>((int)Y[0].x - 8192);
      fl |= fbits(gq.y);
    } else if (i0 == 36 && TABLE == 0) {
      // luminance (4,4): y/T = K/34, so a flag is an exact tie (decided by the caller)
      st[kSlot.s[36]] = (int16_t)(fbits(tq.x) & 0xFFFFu);
      t44 = fbits(gq.x);
      fl |= fbits(gq.y);
    } else {
      st[kSlot.s[i0]] = (int16_t)(fbits(tq.x) & 0xFFFFu);
      fl |= fbits(gq.x) | fbits(gq.y);
    }
  }
}

// One 8x8 block per lane on the packed path (w: its eight 8-byte pixel rows): the 64
// quantised coefficients into st (the lane's stage row, zig-zag slots), luminance
// (4,4) ties decided in place; returns the lane's flag word (sign bit set: some
// coefficient needs the float64 redo, pk_coop_redo_k).  TABLE -1: the wave-uniform
// table `trt`, the quantiser constants as literals behind a scalar branch per
// column pair (runtime-indexed constants were 128 scalar loads per set, spilled to
// VGPR lanes; a branch around the whole block spilled its row outputs).
template <int TABLE>
__device__ __forceinline__ uint32_t pk_block(const uint2 (&w)[8], int16_t *st, int trt = 0) {
  constexpr SlotOf<HIC_LAYOUT_ZIGZAG_I16> kSlot{};
  const f2 kM2 = sp2(kMagic32);
  // row pass: R[m][k] = (row 2m's output k, row 2m + 1's output k)
  f2 R[4][8];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    pk_rows(w[2 * m], w[2 * m + 1], R[m]);
    // pinned where they are made: the compiler otherwise sinks each output's
    // arithmetic to its column pass and keeps the 64 converted pixels live
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(R[m][k]));
  }
  // column pairs (v, v + 2); (4, 6) last, so its column-4 inputs (the rows' integer
  // outputs 4) are at hand for the luminance (4,4) ties
  uint32_t fl = 0, t44 = 0;
  f2 X[8];
  constexpr int kPairs[4] = {0, 1, 5, 4};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int v0 = kPairs[c];
    // 2 x 2 transposes in place: one v_swap_b32 each (the compiler's own moves took
    // ~14 VALU per column pair)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float a = R[m][v0].y, b = R[m][v0 + 2].x;
#ifdef __HIP_DEVICE_COMPILE__
      asm volatile("v_swap_b32 %0, %1" : "+v"(a), "+v"(b));
#else
      const float t = a;
      a = b;
      b = t;
#endif
      X[2 * m] = (f2){R[m][v0].x, a};
      X[2 * m + 1] = (f2){b, R[m][v0 + 2].y};
    }
    f2 Y[8];
    pk_cols(X, Y);
    if (TABLE == 0 || (TABLE < 0 && trt == 0))
      pk_quant_pair<0>(Y, v0, st, kM2, fl, t44);
    else
      pk_quant_pair<1>(Y, v0, st, kM2, fl, t44);
  }
#if defined(HIC_DEV) && defined(HIC_PK_DEV) && (HIC_PK_DEV & 2)
  t44 = 0;  // dev timing (results invalid): no (4,4) tie resolution
#endif
  if ((TABLE == 0 || (TABLE < 0 && trt == 0)) && __builtin_amdgcn_ballot_w64((int)t44 < 0)) {
    if ((int)t44 < 0) {
      // pocketfft's half-scaled y'[4][4] from the rows' outputs 4 (X[r].x, exact
      // integers): pf_y44's operations
      double y[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) y[r] = (double)X[r].x * TW3;
      const double c1 = y[1] + y[2], c3 = y[3] + y[4], c5 = y[5] + y[6], H0 = y[0] + y[7];
      const double h1 = c1 + c5, T2 = H0 + c3;
      st[kSlot.s[36]] = (int16_t)quant_fast<0>((T2 - h1) * TW3, 36);
    }
  }
  return fl;
}

}  // namespace
}  // namespace hic
