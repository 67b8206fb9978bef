// slots.h -- the slot-layout symbol emission of the fused encoder (round 6): each
// RLE record's AC symbols go straight from the kernel's LDS stage into a fixed
// slot of the channel, so the int16 coefficients never reach HBM and no emit
// kernel re-reads them.
//
// Reference: codec.run_length_coding (codec.py:55-99) over a channel's AC stream
// (zig-zag slots 1..63 of every block in raster order, codec.py:292-301) and
// codec.differential_coding (codec.py:47-52).
//
// The stream in slot layout.  A record r (a 64-block Y tile, or a 32-block Cr / Cb
// half tile) owns slot r: symbols [r * cap, r * cap + n_r) of slot_len / slot_val,
// cap = 63 x its blocks.  The channel's symbol stream (what the contiguous emit
// writes) is, over the records in order,
//     nfill_r fillers (max_len - 1, 0)  +  slot r's n_r symbols,
// followed by the EOB (0, 0) when the stream ends in a zero.  Every symbol of a
// record depends only on the record's own blocks except the length of its FIRST
// one and the fillers before it, which carry the zero run from earlier records:
// the fused kernel writes that length as 0 and the close (k_rle_scan16b<true>,
// after the records' scan) writes the true length and the per-record index
// {n_r, P_r, pdc_r, nfill_r} (P_r: the record-relative AC position before the
// first symbol's zeros, pdc_r: the DC of the block before the record).  A decoder
// walks the slots through that index (k_rld_idct_indexed<.., SLOTS>); a caller
// that wants the contiguous stream gets it from hic_rle_slots_compact.
//
// Emission of one pass (one record, or two in the chroma pass) in the kernel:
//   1. every lane reads its block from the stage into 32 registers (zig-zag
//      int16 pairs) and summarises it (first / last nonzero, symbols);
//   2. DPP scans over the lanes give each lane its symbols' offset in the record;
//   3. each lane writes its symbols into the stage IN PLACE (all blocks are in
//      registers by then; a record's symbols never outnumber its AC slots): one
//      packed 16-bit word per symbol, value << 4 | length (length <= 14 for max_len
//      15; every chrominance AC and every luminance AC but zig-zag slot 3 fits 12
//      bits, tools/check/wire_widths.py; a wave whose slot 3 does not writes its
//      symbols straight to HBM instead);
//   4. the wave copies the packed words out, unpacked to the SoA (uint8 length,
//      int16 value) slot arrays, in 16-byte nontemporal stores.
#pragma once
#include "rle_core.h"

namespace hic {
namespace {

constexpr int kSlotM = 15;                  // the slot layout's max_len (4-bit lengths)
constexpr int kStageRowU16 = 4 * kStageU2;  // stage row stride in int16 (68)
constexpr int kSlotY = 64 * 63;             // slot capacity of a 64-block record (symbols)
constexpr int kSlotC = 32 * 63;             // ... of a 32-block record

// pointers of one record's outputs
struct SlotRec {
  uint8_t *len;    // slot base
  int16_t *val;
  int32_t *dc;     // dc_diff of the record's first block
  int64_t *rec;    // its RLE record {first, last, symbols after the first}
  int32_t *rdc;    // its last block's DC (the close's DC hand-off)
  int64_t pos;     // AC stream position of its first block
};

typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
typedef short i16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const lds_u16 *)reinterpret_cast<const uint16_t *>(p);
}

// The symbols of a lane's block after its first nonzero (plus, for a lane that
// does not hold its record's first nonzero, the fillers of the zero run carried in
// from the blocks before it), written through put(index, length, value):
//   o    : the record-relative index of the lane's first symbol;
//   nf0  : fillers before the first nonzero; rem: its length (0 for the record's
//          head, whose true length the close writes).
// Runs inside the block of >= 15 zeros get their fillers.
template <typename Put>
__device__ __forceinline__ void slot_symbols_general(const uint32_t (&zw)[32], int first, int o, int nf0, int rem,
                                                     Put put) {
  int w = o;
  for (int k = 0; k < nf0; ++k, ++w) put(w, kSlotM - 1, 0);
  int pl = first - 1 - rem;
#pragma unroll
  for (int j = 0; j < 63; ++j) {
    const int v = zz_ac(zw, j);
    if (v != 0) {
      int run = j - pl - 1;
      const int nfi = div_m<kSlotM>(run, kSlotM);
      for (int f = 0; f < nfi; ++f, ++w) put(w, kSlotM - 1, 0);
      run -= nfi * kSlotM;
      put(w, run, v);
      ++w;
      pl = j;
    }
  }
}

// One pass's emission (see the file comment).  zw: this lane's block; st2: the
// wave's stage, still holding every block (this lane's in row `lane`).  SEG: lanes
// 0-31 hold record A's 32 blocks and 32-63 record B's (the chroma pass, Cr and
// Cb); else one 64-block record A.  CHECK_WIDE: the luminance table (zig-zag slot 3
// can need 13 bits).  Every lane must call it.
template <bool SEG, bool CHECK_WIDE, bool NT = true>
__device__ __forceinline__ void slot_pass(const uint32_t (&zw)[32], uint2 *st2, int lane, const SlotRec &A,
                                          const SlotRec &B) {
  const int sl = SEG ? (lane & 31) : lane;
  const bool hi = SEG && lane >= 32;
  const SlotRec &R = hi ? B : A;
  // ---- 1. the block's summary
  const uint64_t ac = nz_mask16(zw) >> 1;  // bit j = AC j
  int first, last, nsym;
  summarize_ac<kSlotM>(ac, kSlotM, first, last, nsym);
  const bool dense = nsym == __builtin_popcountll(ac) - 1;  // no run >= 15 inside the block
  // the first nonzero's value, from the stage before it is overwritten
  const int vfirst = first >= 0 ? reinterpret_cast<const int16_t *>(st2 + lane * kStageU2)[1 + first] : 0;
  // DC differences inside the record; its first block keeps its raw DC (the close
  // subtracts the previous record's last DC)
  const int dc = (int)(int16_t)(zw[0] & 0xFFFFu);
  const int dprev = wave_shr1_i32(0, dc);
  R.dc[sl] = sl == 0 ? dc : dc - dprev;
  // ---- 2. offsets inside the record (positions relative to its first AC: int32)
  const int lastr = last >= 0 ? sl * 63 + last : -1;
  const int incl = SEG ? seg32_incl_max_i32(lastr) : wave_incl_max_i32(lastr);
  int prev = wave_shr1_i32(-1, incl);
  if (sl == 0) prev = -1;
  const bool head = first >= 0 && prev < 0;  // holds the record's first nonzero
  const int run0 = sl * 63 + first - prev - 1;
  const int nf0 = (first < 0 || head) ? 0 : div_m<kSlotM>(run0, kSlotM);
  const int rem = (first < 0 || head) ? 0 : run0 - nf0 * kSlotM;
  const int cnt = first < 0 ? 0 : nsym + 1 + nf0;
  const int icnt = SEG ? seg32_incl_sum_i32(cnt) : wave_incl_sum_i32(cnt);
  const int o = icnt - cnt;
  const int nA = __builtin_amdgcn_readlane(icnt, SEG ? 31 : 63), nB = __builtin_amdgcn_readlane(icnt, 63);
  const int lA = __builtin_amdgcn_readlane(incl, SEG ? 31 : 63), lB = __builtin_amdgcn_readlane(incl, 63);
  const int dA = __builtin_amdgcn_readlane(dc, SEG ? 31 : 63), dB = __builtin_amdgcn_readlane(dc, 63);
  const int nR = hi ? nB : nA, lR = hi ? lB : lA;
  // the record: its first nonzero's position (head lane, or lane 0 of an empty
  // record), the last one's and the symbols after the first; its last DC
  if (lR < 0 ? sl == 0 : head) R.rec[0] = lR < 0 ? -1 : R.pos + sl * 63 + first;
  if (sl == 0) {
    R.rec[1] = lR >= 0 ? R.pos + lR : -1;
    R.rec[2] = lR >= 0 ? nR - 1 : 0;
    *R.rdc = hi ? dB : dA;
  }
  bool wide = false;
  if (CHECK_WIDE) {  // zig-zag slot 3 (AC 2) outside 12 bits: no packed stage
    const int v3 = (int)(int16_t)(zw[1] >> 16);
    wide = __builtin_amdgcn_ballot_w64(v3 > 2047 || v3 < -2048) != 0;
  }
  __builtin_amdgcn_wave_barrier();  // every block is in registers: the stage is free
  if (wide) {  // rare: each lane writes its symbols straight to the slot
    if (first >= 0) {
      uint8_t *gl = R.len;
      int16_t *gv = R.val;
      slot_symbols_general(zw, first, o, nf0, rem, [&](int i, int len, int v) {
        gl[i] = (uint8_t)len;
        gv[i] = (int16_t)v;
      });
    }
    __builtin_amdgcn_wave_barrier();
    return;
  }
  // ---- 3. packed symbols into the stage, in place
  uint16_t *sb = reinterpret_cast<uint16_t *>(st2) + (hi ? 32 * kStageRowU16 : 0);
  {
    // Branch-free over the block's 63 AC: EVERY coefficient writes the lane's next
    // free slot, which only a nonzero advances -- a zero's word is overwritten by the
    // next nonzero's.  After a lane's last nonzero (or in an all-zero block) its
    // writes land on the first slot of the next lane with symbols, and are undone
    // below, after the loop, where every lane writes its carried fillers and its
    // first symbol again.  A block with a run >= 15 inside (not dense) writes within
    // its own symbols here, and the general loop after writes them all.
    uint32_t la = lds_addr(sb + o + nf0);
    int pl = first - 1 - rem;
    // AC j is zig-zag slot j + 1: the low half of zw[(j + 1) / 2] for odd j, the
    // high half for even j.  The packed word is formed without extracting the value:
    // low half, (w << 4) | len (the store keeps 16 bits); high half, (w >> 12) with
    // its low nibble replaced by len.
#pragma unroll
    for (int j = 0; j < 63; ++j) {
      const uint32_t w = zw[(j + 1) >> 1];
      const bool lo = ((j + 1) & 1) == 0;
      const bool nz = lo ? (uint16_t)w != 0 : w > 0xFFFFu;
      const uint32_t len = (uint32_t)(j - pl - 1);
      const uint32_t pk = lo ? ((w << 4) | len) : (((w >> 12) & 0xFFF0u) | len);
      *(lds_u16 *)(uintptr_t)la = (uint16_t)pk;
      la += nz ? 2u : 0u;
      pl = nz ? j : pl;
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (first >= 0) {
    for (int k = 0; k < nf0; ++k) sb[o + k] = (uint16_t)(kSlotM - 1);
    sb[o + nf0] = (uint16_t)(((uint32_t)vfirst << 4) | (uint32_t)rem);
  }
  if (__builtin_amdgcn_ballot_w64(!dense && first >= 0)) {
    if (!dense && first >= 0)
      slot_symbols_general(zw, first, o, nf0, rem, [&](int i, int len, int v) {
        sb[i] = (uint16_t)(((uint32_t)v << 4) | (uint32_t)len);
      });
  }
  __builtin_amdgcn_wave_barrier();
  // ---- 4. copy out, every store instruction 1 KiB contiguous: lengths 16 symbols
  // per lane (32 B of packed words -> 16 B), values 8 per lane (16 B -> 16 B)
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int h = 0; h < (SEG ? 2 : 1); ++h) {
    const SlotRec &S = h ? B : A;
    const int n = h ? nB : nA;
    const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<uint16_t *>(st2) + h * 32 * kStageRowU16);
    for (int c = lane; 16 * c < n; c += 64) {
      const uint4 p = src[2 * c], q = src[2 * c + 1];
      // lengths: the low nibbles of the words' low bytes
      const u32x4 L = {__builtin_amdgcn_perm(p.y, p.x, 0x06040200u) & 0x0F0F0F0Fu,
                       __builtin_amdgcn_perm(p.w, p.z, 0x06040200u) & 0x0F0F0F0Fu,
                       __builtin_amdgcn_perm(q.y, q.x, 0x06040200u) & 0x0F0F0F0Fu,
                       __builtin_amdgcn_perm(q.w, q.z, 0x06040200u) & 0x0F0F0F0Fu};
      u32x4 *ol = reinterpret_cast<u32x4 *>(S.len) + c;
      if (NT)
        __builtin_nontemporal_store(L, ol);
      else
        *ol = L;
    }
    for (int c = lane; 8 * c < n; c += 64) {
      const uint4 p = src[c];
      const uint32_t w[4] = {p.x, p.y, p.z, p.w};
      uint32_t vv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)  // value = the word >> 4 (arithmetic), both halves
        vv[k] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(i16x2_t, w[k]) >> (i16x2_t){4, 4});
      const u32x4 V = {vv[0], vv[1], vv[2], vv[3]};
      u32x4 *ov = reinterpret_cast<u32x4 *>(S.val) + c;
      if (NT)
        __builtin_nontemporal_store(V, ov);
      else
        *ov = V;
    }
  }
  __builtin_amdgcn_wave_barrier();
}

}  // namespace
}  // namespace hic
