// dev micro-benchmark: memory-only patterns of the plane DCT pass (k_dct_planes) on
// the 8K luminance plane (SURVEY.md 8(d)'s measurement point: 33.2 MB of uint8
// pixels read, 66.4 MB of int16 coefficients written, >= 0.70 of 8 TB/s = <= 17.8
// us).  No arithmetic: what the access pattern alone costs.
//   blk8       lane = one 8x8 block, 8 x 8 B row loads, 1 KiB nontemporal stores
//              (k_dct_planes' pattern; persistent grid)
//   blk8_1w    the same, one wave per 64-block set (k_dct_planes' default grid)
//   blk8_plain the same with plain (cached) stores
//   blk16      lane = two horizontally adjacent blocks, 8 x 16 B row loads
//   rows16     lane = 16 B of one pixel row (a wave reads 1 KiB of 8 consecutive
//              rows = 128 blocks), coefficients written 1 KiB per instruction
//   stream     linear: 16 B per lane read, 2 x 16 B per lane written (the ceiling
//              of a 1:2 read / write mix)
// Build: hipcc --offload-arch=gfx950 -O3 -o plane_patterns plane_patterns.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void put(uint8_t *out, int64_t i16, u32x4 v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(out) + i16);
  else
    reinterpret_cast<u32x4 *>(out)[i16] = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_blk8(const uint8_t *__restrict__ plane, int W, int nsets,
                                              uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63, nbx = W / 8;
  for (int set = blockIdx.x * 4 + (threadIdx.x >> 6); set < nsets; set += gridDim.x * 4) {
    const int b = set * 64 + lane, by = b / nbx, bx = b - by * nbx;
    const uint8_t *p = plane + (int64_t)by * 8 * W + bx * 8;
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + (int64_t)r * W);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      put<NT>(out, ((int64_t)set * 8 + u) * 64 + lane, (u32x4){w[u].x, w[u].y, w[(u + 1) & 7].x ^ u, w[(u + 1) & 7].y});
  }
}

__global__ __launch_bounds__(256) void k_blk16(const uint8_t *__restrict__ plane, int W, int nsets2,
                                               uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63, nbx = W / 8;
  for (int set = blockIdx.x * 4 + (threadIdx.x >> 6); set < nsets2; set += gridDim.x * 4) {
    const int b = set * 128 + 2 * lane, by = b / nbx, bx = b - by * nbx;
    const uint8_t *p = plane + (int64_t)by * 8 * W + bx * 8;
    uint4 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint4 *>(p + (int64_t)r * W);
#pragma unroll
    for (int u = 0; u < 16; ++u)
      put<true>(out, ((int64_t)set * 16 + u) * 64 + lane,
                (u32x4){w[u & 7].x, w[u & 7].y ^ u, w[(u + 1) & 7].z, w[(u + 3) & 7].w});
  }
}

// lane = two blocks, each lane stores its own 2 x 128 B (16 x 16 B at its block
// addresses: every store instruction touches 64 lines, 16 B each), no LDS stage
template <bool NT>
__global__ __launch_bounds__(256) void k_blk16_lane(const uint8_t *__restrict__ plane, int W, int nsets2,
                                                    uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63, nbx = W / 8;
  for (int set = blockIdx.x * 4 + (threadIdx.x >> 6); set < nsets2; set += gridDim.x * 4) {
    const int b = set * 128 + 2 * lane, by = b / nbx, bx = b - by * nbx;
    const uint8_t *p = plane + (int64_t)by * 8 * W + bx * 8;
    uint4 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint4 *>(p + (int64_t)r * W);
#pragma unroll
    for (int u = 0; u < 16; ++u)
      put<NT>(out, ((int64_t)set * 128 + 2 * lane) * 8 + u,
              (u32x4){w[u & 7].x, w[u & 7].y ^ u, w[(u + 1) & 7].z, w[(u + 3) & 7].w});
  }
}

// a wave reads 8 rows x 1 KiB (128 blocks of one block row; the row's last chunk
// is 512 B, 64 blocks), lane = 16 B of a row; the chunk's coefficients are written
// 1 KiB per instruction
__global__ __launch_bounds__(256) void k_rows16(const uint8_t *__restrict__ plane, int W, int H,
                                                uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63, per_row = (W + 1023) / 1024, nsets = (H / 8) * per_row;
  for (int set = blockIdx.x * 4 + (threadIdx.x >> 6); set < nsets; set += gridDim.x * 4) {
    const int by = set / per_row, cx = set - by * per_row;
    const int nv = (W - cx * 1024) / 16 < 64 ? (W - cx * 1024) / 16 : 64;  // valid lanes (wave-uniform)
    uint4 w[8];
    if (lane < nv) {
      const uint8_t *p = plane + (int64_t)by * 8 * W + cx * 1024 + 16 * lane;
#pragma unroll
      for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint4 *>(p + (int64_t)r * W);
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) w[r] = make_uint4(0, 0, 0, 0);
    }
    // the chunk's blocks start at block by * W / 8 + 128 cx: 128 B each
    const int64_t o16 = ((int64_t)by * (W / 8) + 128 * cx) * 8;
    for (int u = 0; u < nv / 4; ++u)
      put<true>(out, o16 + u * 64 + lane, (u32x4){w[u & 7].x, w[u & 7].y ^ u, w[(u + 1) & 7].z, w[(u + 3) & 7].w});
  }
}

__global__ __launch_bounds__(256) void k_stream(const uint8_t *__restrict__ in, int64_t n, uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = n / 1024, nw = (int64_t)gridDim.x * 4;
  for (int64_t r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const u32x4 v = reinterpret_cast<const u32x4 *>(in + r * 1024)[lane];
    put<true>(out, r * 128 + lane, v);
    put<true>(out, r * 128 + 64 + lane, v ^ (u32x4){1u, 2u, 3u, 4u});
  }
}

int main() {
  const int H = 4320, W = 7680, rot = 12;
  const int64_t np = (int64_t)H * W;
  uint8_t *in[rot], *out[rot];
  for (int i = 0; i < rot; ++i) {
    if (hipMalloc(&in[i], np) != hipSuccess || hipMalloc(&out[i], 2 * np) != hipSuccess) return 1;
    (void)hipMemset(in[i], i, np);
  }
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int nsets = (int)(np / 64 / 64), nsets2 = nsets / 2;
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  struct V {
    const char *name;
    int kind, grid;
  } vs[] = {
      {"blk8 persist 8/CU", 0, cus * 2},  {"blk8 persist 16/CU", 0, cus * 4}, {"blk8 persist 32/CU", 0, cus * 8},
      {"blk8_1w", 0, (nsets + 3) / 4},    {"blk8_plain 1w", 1, (nsets + 3) / 4},
      {"blk16 1w", 2, (nsets2 + 3) / 4}, {"blk16 persist 16/CU", 2, cus * 4},
      {"rows16 1w", 3, ((H / 8) * ((W + 1023) / 1024) + 3) / 4}, {"rows16 persist 16/CU", 3, cus * 4},
      {"stream 1:2", 4, cus * 8},
      {"blk16_lane nt 1w", 5, (nsets2 + 3) / 4}, {"blk16_lane nt persist 8/CU", 5, cus * 2},
      {"blk16_lane plain 1w", 6, (nsets2 + 3) / 4}, {"blk16_lane plain persist 8/CU", 6, cus * 2},
      {"blk16 persist 8/CU", 2, cus * 2},
  };
  const int n = 14;
  for (const V &v : vs) {
    float tot = 0;
    for (int i = 0; i < n; ++i) {
      (void)hipEventRecord(s);
      const dim3 g(v.grid), b(256);
      if (v.kind == 0) hipLaunchKernelGGL(k_blk8<true>, g, b, 0, 0, in[i % rot], W, nsets, out[i % rot]);
      if (v.kind == 1) hipLaunchKernelGGL(k_blk8<false>, g, b, 0, 0, in[i % rot], W, nsets, out[i % rot]);
      if (v.kind == 2) hipLaunchKernelGGL(k_blk16, g, b, 0, 0, in[i % rot], W, nsets2, out[i % rot]);
      if (v.kind == 3) hipLaunchKernelGGL(k_rows16, g, b, 0, 0, in[i % rot], W, H, out[i % rot]);
      if (v.kind == 4) hipLaunchKernelGGL(k_stream, g, b, 0, 0, in[i % rot], np, out[i % rot]);
      if (v.kind == 5) hipLaunchKernelGGL(k_blk16_lane<true>, g, b, 0, 0, in[i % rot], W, nsets2, out[i % rot]);
      if (v.kind == 6) hipLaunchKernelGGL(k_blk16_lane<false>, g, b, 0, 0, in[i % rot], W, nsets2, out[i % rot]);
      (void)hipEventRecord(e);
      (void)hipEventSynchronize(e);
      float ms;
      (void)hipEventElapsedTime(&ms, s, e);
      if (i >= 4) tot += ms;
    }
    const double us = tot / (n - 4) * 1e3;
    printf("%-24s %7.2f us  %6.1f GB/s  %.3f of 8 TB/s (8K luma: read %.1f MB, write %.1f MB)\n", v.name, us,
           3.0 * np / us / 1e3, 3.0 * np / us / 8e6, np / 1e6, 2.0 * np / 1e6);
  }
  return (int)hipGetLastError();
}
