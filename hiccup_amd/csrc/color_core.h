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

}  // namespace
}  // namespace hic
