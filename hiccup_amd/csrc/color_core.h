// color_core.h -- OpenCV 8U colour conversion helpers (cv2.cvtColor RGB2YCrCb /
// YCrCb2RGB fixed point, yuv_shift 14) and the DPP wave shifts shared by the
// colour kernels (color.hip) and the fused 4:2:0 encoder (encode.hip).
// Reference call sites: compression.py:21,56.  PARITY UNPINNED (OpenCV absent:
// see color.hip).
#pragma once
#include "hic_common.h"

namespace hic {
namespace {

constexpr int kR2Y = 4899, kG2Y = 9617, kB2Y = 1868, kYCRI = 11682, kYCBI = 9241;
constexpr int kCR2R = 22987, kCR2G = -11698, kCB2G = -5636, kCB2B = 29049;

__device__ __forceinline__ int descale14(int x) { return (x + (1 << 13)) >> 14; }
__device__ __forceinline__ uint32_t sat8(int v) { return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

struct YCC {
  uint32_t y, cr, cb;
};
__device__ __forceinline__ YCC rgb2ycc(int r, int g, int b) {
  const int y = descale14(r * kR2Y + g * kG2Y + b * kB2Y);
  return {(uint32_t)y, sat8(descale14((r - y) * kYCRI + (128 << 14))),
          sat8(descale14((b - y) * kYCBI + (128 << 14)))};
}

__device__ __forceinline__ int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

// DPP wave shifts.  The edge lane's value is selected explicitly afterwards: relying
// on update_dpp's `old` operand for the disabled lane miscompiles once the move is
// folded into a consumer (bits 16-31 of lane 0 came out wrong).
__device__ __forceinline__ uint32_t shr1(uint32_t v) {  // lane i <- lane i-1
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t shl1(uint32_t v) {  // lane i <- lane i+1
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}

// Packs four bytes.  The asm barrier keeps the backend from fusing the preceding
// descale + saturate of two of them into v_ashr_pk_u8_i32: gfx950 codegen
// assumes that instruction zeroes bits 16-31 of its destination, but they
// came back holding the source's stale high half, OR-ed into the upper two bytes.
__device__ __forceinline__ uint32_t pack4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
  asm volatile("" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
  return b0 | b1 << 8 | b2 << 16 | b3 << 24;
}

// Packed 16-bit pairs (cr | cb << 16) and the YCrCb -> RGB dot products of the
// decode colour kernels (color.hip k_ycrcb420_rgb_walk, dct.hip k_rld_idct_rgb_indexed).
typedef unsigned short u16x2c __attribute__((ext_vector_type(2)));
typedef short s16x2c __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2c, a) + __builtin_bit_cast(u16x2c, b));
}
__device__ __forceinline__ uint32_t pk_mad_u16(uint32_t a, uint32_t k, uint32_t c) {  // a * k + c per half
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2c, a) * __builtin_bit_cast(u16x2c, k) +
                                          __builtin_bit_cast(u16x2c, c));
}
__device__ __forceinline__ uint32_t pk_sra6(uint32_t a) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2c, a) >> (short)6);
}
// acc + lo(crcb) * lo(k) + hi(crcb) * hi(k), signed 16-bit halves; the
// three-operand form (k in an SGPR), so no copy of acc per channel
__device__ __forceinline__ int ycc_dot(uint32_t crcb, uint32_t k, int acc) {
  int d;
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(crcb), "s"(k), "v"(acc));
  return d;
}
__device__ __forceinline__ uint32_t sreg(uint32_t k) {  // opaque wave-uniform constant
  asm volatile("" : "+s"(k));
  return k;
}
// low 16 bits: sat8(a >> 14) | sat8(b >> 14) << 8 (gfx950 v_ashr_pk_u8_i32)
__device__ __forceinline__ uint32_t sat_pk2(int a, int b) {
  uint32_t d;
  asm("v_ashr_pk_u8_i32 %0, %1, %2, 14" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

}  // namespace
}  // namespace hic
