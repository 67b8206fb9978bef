// probe.hip -- memory-only probes that measure, in the bench's own run, the floors
// the hot kernels are judged against ("also report the box's
// measured device-copy bandwidth").  No arithmetic; not part of the codec path.
//
//  hic_probe_copy:  a plain streaming copy, 8 KiB per wave per step (8 x 1 KiB
//                   loads in flight, nontemporal stores), persistent grid: the
//                   device-copy rate of the box.
//  hic_probe_plane: the forward plane pass's own byte pattern without the DCT --
//                   lane = one 8x8 block (8 row loads of 8 B), the 64 blocks of a
//                   wave's set staged in LDS and written as 1 KiB nontemporal
//                   stores in block order (k_dct_planes' copy-out), the next set's
//                   rows loading during the current set's stage and store: 1 B
//                   read and 2 B written per pixel, the luma DCT pass's traffic.
#include "hic_common.h"

namespace hic {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Each wave copies contiguous 8 KiB chunks (8 loads of 1 KiB in flight per wave,
// then 8 stores), chunks dealt round-robin over the persistent grid.
__global__ __launch_bounds__(256) void k_probe_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, int64_t n16) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * 4, nchunk = n16 / 512;
  for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunk; c += nwaves) {
    const u32x4 *s = src + c * 512 + lane;
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s[64 * k];
    u32x4 *d = dst + c * 512 + lane;
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(v[k], d + 64 * k);
  }
  // the tail (< 8 KiB)
  for (int64_t i = nchunk * 512 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
    dst[i] = src[i];
}

constexpr int kProbeStageU2 = 17;  // 136 B stage rows, as the DCT kernels' stage

__global__ __launch_bounds__(256) void k_probe_plane(const uint8_t *__restrict__ plane, int64_t stride, int nbx,
                                                     int nblk, int16_t *__restrict__ out) {
  __shared__ uint2 s_stage[4 * 64 * kProbeStageU2];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nsets = (nblk + 63) / 64, nwaves = gridDim.x * 4;
  uint2 *st2 = s_stage + wv * 64 * kProbeStageU2;
  auto load = [&](int set, uint2 (&w)[8]) {
    int blk = set * 64 + lane;
    blk = blk < nblk ? blk : nblk - 1;
    const int bi = blk / nbx, bj = blk - bi * nbx;
    const uint8_t *p = plane + (int64_t)bi * 8 * stride + bj * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + r * stride);
  };
  int g = blockIdx.x * 4 + wv;
  if (g >= nsets) return;
  uint2 wn[8];
  load(g, wn);
  for (; g < nsets; g += nwaves) {
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = wn[r];
    if (g + nwaves < nsets) load(g + nwaves, wn);
    // a 128 B "coefficient block" per lane: the 64 pixel bytes twice, so the
    // stores carry data the loads produced
    uint2 *row = st2 + lane * kProbeStageU2;
#pragma unroll
    for (int r = 0; r < 8; ++r) row[r] = w[r];
#pragma unroll
    for (int r = 0; r < 8; ++r) row[8 + r] = make_uint2(w[r].y, w[r].x);
    __builtin_amdgcn_wave_barrier();
    u32x4 *o = reinterpret_cast<u32x4 *>(out + (int64_t)g * 64 * 64);
    const uint2 *src = st2 + (lane >> 3) * kProbeStageU2 + 2 * (lane & 7);
    const int rem = nblk - g * 64;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint2 lo = src[8 * k * kProbeStageU2], hi = src[8 * k * kProbeStageU2 + 1];
      const u32x4 v = {lo.x, lo.y, hi.x, hi.y};
      if (rem >= 64)
        __builtin_nontemporal_store(v, o + 64 * k + lane);
      else if (8 * k + (lane >> 3) < rem)
        o[64 * k + lane] = v;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" int hic_probe_copy(const void *src, void *dst, int64_t bytes, int waves_per_cu, void *stream,
                              void *ev_start, void *ev_stop) {
  if (!src || !dst) return arg_error("null pointer");
  if (bytes <= 0 || bytes % 16) return arg_error("bytes must be a positive multiple of 16");
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16) return arg_error("16-byte alignment");
  if (waves_per_cu < 0 || waves_per_cu > 32) return arg_error("waves_per_cu (0 = 16, at most 32)");
  const int64_t n16 = bytes / 16;
  const int64_t want = (n16 / 512 + 3) / 4;  // one 8 KiB chunk per wave at least
  const int cap = (waves_per_cu ? waves_per_cu : 16) * cu_count() / 4;
  const dim3 grid((unsigned)(want < cap ? (want > 0 ? want : 1) : cap)), block(256);
  const hipStream_t s = as_stream(stream);
  const hipEvent_t e0 = static_cast<hipEvent_t>(ev_start), e1 = static_cast<hipEvent_t>(ev_stop);
  const auto *a = static_cast<const u32x4 *>(src);
  auto *b = static_cast<u32x4 *>(dst);
  if (e0 || e1)
    hipExtLaunchKernelGGL(k_probe_copy, grid, block, 0, s, e0, e1, 0, a, b, n16);
  else
    hipLaunchKernelGGL(k_probe_copy, grid, block, 0, s, a, b, n16);
  return check_launch("k_probe_copy");
}

extern "C" int hic_probe_plane(const uint8_t *plane, int64_t H, int64_t W, int16_t *out, int waves_per_cu,
                               void *stream, void *ev_start, void *ev_stop) {
  if (!plane || !out) return arg_error("null pointer");
  if (waves_per_cu < 0 || waves_per_cu > 16) return arg_error("waves_per_cu (0 = 12, at most 16: LDS)");
  if (H < 8 || W < 8 || H % 8 || W % 8 || H >= (1 << 20) || W >= (1 << 20)) return arg_error("plane shape (multiples of 8)");
  if ((H / 8) * (W / 8) >= (1LL << 31) / 64) return arg_error("plane too large");
  if (reinterpret_cast<uintptr_t>(plane) % 8 || reinterpret_cast<uintptr_t>(out) % 16) return arg_error("alignment");
  const int nbx = (int)(W / 8), nblk = (int)((H / 8) * nbx), nsets = (nblk + 63) / 64;
  const int cap = (waves_per_cu ? waves_per_cu : 12) * cu_count();  // default: k_dct_planes' one-plane grid
  const int waves = nsets < cap ? nsets : cap;
  const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
  const hipStream_t s = as_stream(stream);
  const hipEvent_t e0 = static_cast<hipEvent_t>(ev_start), e1 = static_cast<hipEvent_t>(ev_stop);
  if (e0 || e1)
    hipExtLaunchKernelGGL(k_probe_plane, grid, block, 0, s, e0, e1, 0, plane, (int64_t)W, nbx, nblk, out);
  else
    hipLaunchKernelGGL(k_probe_plane, grid, block, 0, s, plane, (int64_t)W, nbx, nblk, out);
  return check_launch("k_probe_plane");
}
