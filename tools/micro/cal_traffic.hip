// Calibration for the DCT kernel's HBM counters (dev tool).
// k_pattern reads an 8K uint8 plane with exactly k_dct_planes' access
// pattern: lane = one 8x8 block, 8 x 8-byte row loads.  It writes int16 [nblk][64]
// with 16-B-per-lane streaming stores, and does no arithmetic.  Known bytes:
// 1 B/px read, 2 B/px written.  rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over this
// binary gives the counter/byte ratio for that pattern.  The event time gives the
// bandwidth this access pattern reaches.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_pattern(const uint8_t *__restrict__ plane, int64_t stride, int W, int nbx,
                                                 int nblk, int16_t *__restrict__ out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nsets = nblk / 64;
  for (int set = blockIdx.x * 4 + wv; set < nsets; set += gridDim.x * 4) {
    const int b = set * 64 + lane;
    const int by = b / nbx, bx = b - by * nbx;
    const uint8_t *p = plane + (int64_t)by * 8 * stride + bx * 8;
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + r * stride);
    uint4 *o = reinterpret_cast<uint4 *>(out + (int64_t)set * 64 * 64);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint2 a = w[u], c = w[(u + 1) & 7];
      o[u * 64 + lane] = make_uint4(a.x, a.y, c.x ^ u, c.y);
    }
  }
}

int main() {
  const int H = 4320, W = 7680, nbx = W / 8, nblk = (H / 8) * nbx, rot = 12;
  uint8_t *in[rot];
  int16_t *out[rot];
  for (int i = 0; i < rot; ++i) {
    hipMalloc(&in[i], (size_t)H * W);
    hipMemset(in[i], i, (size_t)H * W);
    hipMalloc(&out[i], (size_t)nblk * 128);
  }
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  float tot = 0;
  const int n = 24;
  for (int i = 0; i < n; ++i) {
    hipEventRecord(s);
    hipLaunchKernelGGL(k_pattern, dim3(cus * 8), dim3(256), 0, 0, in[i % rot], (int64_t)W, W, nbx, nblk, out[i % rot]);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    if (i >= 4) tot += ms;
  }
  const double us = tot / (n - 4) * 1e3, bytes = 3.0 * H * W;
  printf("k_pattern: %.2f us/launch, %.1f GB/s algorithmic (read %.1f MB, write %.1f MB)\n", us, bytes / us / 1e3,
         H * W / 1e6, 2.0 * H * W / 1e6);
  return 0;
}
