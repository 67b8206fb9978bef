// dev: the packed-float32 fast path's flag rate on random blocks (the share of
// blocks pk_block sends to the float64 redo), per table, against dct_bounds.py's
// expectation (~0.035 per luminance block).  hipcc --offload-arch=gfx950 -O3
// -I hiccup_amd/csrc -o /tmp/pk_flags tools/micro/pk_flags.hip && /tmp/pk_flags
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "dct_pk.h"

using namespace hic;

__device__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int TABLE>
__global__ __launch_bounds__(256) void k_flags(uint32_t seed, unsigned long long *count) {
  __shared__ uint2 s_stage[4 * 64 * kStageU2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int16_t *st = reinterpret_cast<int16_t *>(s_stage + (wv * 64 + lane) * kStageU2);
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  uint2 w[8];
  for (int r = 0; r < 8; ++r) w[r] = make_uint2(hash32(seed ^ (b * 16 + 2 * r)), hash32(seed ^ (b * 16 + 2 * r + 1)));
  const uint32_t fl = pk_block<TABLE>(w, st);
  const unsigned long long n = __builtin_popcountll(__builtin_amdgcn_ballot_w64((int)fl < 0));
  if (lane == 0) atomicAdd(count, n);
}

int main() {
  unsigned long long *d;
  hipMalloc(&d, 16);
  const int grid = 65536;  // 16.8 M blocks per table
  for (int t = 0; t < 2; ++t) {
    hipMemset(d, 0, 16);
    if (t == 0)
      hipLaunchKernelGGL(k_flags<0>, dim3(grid), dim3(256), 0, 0, 12345u, d);
    else
      hipLaunchKernelGGL(k_flags<1>, dim3(grid), dim3(256), 0, 0, 12345u, d);
    unsigned long long h = 0;
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("table %d: %llu of %d blocks flagged = %.5f per block (%.2f per 64-block set)\n", t, h, grid * 256,
           (double)h / (grid * 256.0), 64.0 * h / (grid * 256.0));
  }
  hipFree(d);
  return 0;
}
