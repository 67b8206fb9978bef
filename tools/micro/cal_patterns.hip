// Calibration for rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 (dev tool, see
// MI355X_MICROARCH.md HBM section: FETCH_SIZE reports half the bytes of wide
// streaming reads; other widths are uncalibrated).  Each kernel reads a known
// number of bytes with the load pattern of one of the encode kernels and writes a
// known number of bytes with 16-B-per-lane stores, so counter / known bytes is the
// correction factor for that pattern:
//   k_cal_rgb24 : k_encode420's RGB rows -- lane l reads 24 B at 24 l (3 x 8 B),
//                 1536 B per wave-row
//   k_cal_blk8  : k_dct_planes' plane rows -- lane = 8x8 block, 8 x 8 B row loads
//   k_cal_q12   : the colour kernels' RGB quads -- 12 B per lane, dense
//   k_cal_d16   : k_rle_emit16b's blocks -- 16 B per lane, dense
// Build: hipcc --offload-arch=gfx950 -O3 -o cal_patterns cal_patterns.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void put(uint8_t *out, int64_t i16, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(out) + i16);
}

// k_encode420's geometry: an H x W RGB image (W % 512 == 0) in units of 16 rows x
// 512 pixels, one wave per unit, lane l reading 24 B at 24 l of each of the unit's
// rows (here without the pyrDown halo rows, so every byte is read once); writes a
// sixth of the bytes read
__global__ __launch_bounds__(256) void k_cal_rgb24(const uint8_t *__restrict__ in, int H, int W,
                                                   uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63, ns = W / 512;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= ns * (H / 16)) return;
  const int u = g / ns, s = g - u * ns;
  const int64_t pitch = (int64_t)W * 3;
  uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint2 *p = reinterpret_cast<const uint2 *>(in + (int64_t)(16 * u + r) * pitch + 1536 * s + 24 * lane);
    const uint2 a = p[0], b = p[1], c = p[2];
    acc[r & 3] ^= a.x ^ b.y;
    acc[(r + 1) & 3] ^= a.y ^ c.x;
    acc[(r + 2) & 3] ^= b.x ^ c.y;
    if ((r & 3) == 3) {  // 16 B per lane per 4 rows = 1/6 of the 24 B x 4 read
      put(out, ((int64_t)g * 4 + (r >> 2)) * 64 + lane, (u32x4){acc[0], acc[1], acc[2], acc[3]});
    }
  }
}

// plane W x H (W % 512 == 0): reads n = W * H, writes 2n (as the DCT)
__global__ __launch_bounds__(256) void k_cal_blk8(const uint8_t *__restrict__ plane, int W, int nblk,
                                                  uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63, nbx = W / 8;
  for (int set = blockIdx.x * 4 + (threadIdx.x >> 6); set < nblk / 64; set += gridDim.x * 4) {
    const int b = set * 64 + lane, by = b / nbx, bx = b - by * nbx;
    const uint8_t *p = plane + (int64_t)by * 8 * W + bx * 8;
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + (int64_t)r * W);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      put(out, ((int64_t)set * 8 + u) * 64 + lane, (u32x4){w[u].x, w[u].y, w[(u + 1) & 7].x ^ u, w[(u + 1) & 7].y});
  }
}

// reads n (multiple of 768) with 12 B per lane, writes n
__global__ __launch_bounds__(256) void k_cal_q12(const uint8_t *__restrict__ in, int64_t n, uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = n / 768, nw = (int64_t)gridDim.x * 4;
  for (int64_t r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(in + r * 768 + 12 * lane);
    const uint32_t a = p[0], b = p[1], c = p[2];
    if (lane < 48) put(out, r * 48 + lane, (u32x4){a, b, c, a ^ b});
  }
}

// reads n (multiple of 1024) with 16 B per lane, writes n
__global__ __launch_bounds__(256) void k_cal_d16(const uint8_t *__restrict__ in, int64_t n, uint8_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = n / 1024, nw = (int64_t)gridDim.x * 4;
  for (int64_t r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    const u32x4 v = reinterpret_cast<const u32x4 *>(in + r * 1024)[lane];
    put(out, r * 64 + lane, v ^ (u32x4){1u, 2u, 3u, 4u});
  }
}

int main() {
  const int H = 4320, W = 7680, rot = 8;
  const int64_t nrgb = (int64_t)H * W * 3, nplane = (int64_t)H * W;
  uint8_t *in[rot], *out[rot];
  for (int i = 0; i < rot; ++i) {
    hipMalloc(&in[i], nrgb);
    hipMemset(in[i], i, nrgb);
    hipMalloc(&out[i], nrgb);
  }
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const dim3 grid(cus * 8), block(256);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  const int n = 12;
  const char *names[4] = {"k_cal_rgb24", "k_cal_blk8", "k_cal_q12", "k_cal_d16"};
  const double rd[4] = {(double)nrgb, (double)nplane, (double)nrgb, (double)nrgb};
  const double wr[4] = {(double)nrgb / 6, 2.0 * nplane, (double)nrgb, (double)nrgb};
  for (int k = 0; k < 4; ++k) {
    float tot = 0;
    for (int i = 0; i < n; ++i) {
      hipEventRecord(s);
      if (k == 0)
        hipLaunchKernelGGL(k_cal_rgb24, dim3((W / 512) * (H / 16) / 4), block, 0, 0, in[i % rot], H, W, out[i % rot]);
      if (k == 1) hipLaunchKernelGGL(k_cal_blk8, grid, block, 0, 0, in[i % rot], W, (int)(nplane / 64), out[i % rot]);
      if (k == 2) hipLaunchKernelGGL(k_cal_q12, grid, block, 0, 0, in[i % rot], nrgb, out[i % rot]);
      if (k == 3) hipLaunchKernelGGL(k_cal_d16, grid, block, 0, 0, in[i % rot], nrgb, out[i % rot]);
      hipEventRecord(e);
      hipEventSynchronize(e);
      float ms;
      hipEventElapsedTime(&ms, s, e);
      if (i >= 2) tot += ms;
    }
    const double us = tot / (n - 2) * 1e3;
    printf("%s: %.2f us/launch, read %.0f B, write %.0f B, %.1f GB/s\n", names[k], us, rd[k], wr[k],
           (rd[k] + wr[k]) / us / 1e3);
  }
  return 0;
}
