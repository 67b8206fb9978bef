// Microbenchmark: fp64 add throughput vs independent chains per lane and waves per SIMD (gfx950).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int C>
__global__ void k(double *out, double seed, int iters) {
  double a[C];
#pragma unroll
  for (int i = 0; i < C; ++i) a[i] = seed + threadIdx.x + i;
  const double c = seed * 0.5 + 1.0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < C; ++i) a[i] = a[i] * c + 0.25;  // mul + add (no contraction)
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < C; ++i) s += a[i];
  if (s == 12345.678) out[threadIdx.x] = s;
}
template <int C>
void run(int waves_per_simd) {
  double *d; (void)hipMalloc(&d, 1024 * sizeof(double));
  const int iters = 2048;
  const int blocks = 256 * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD per block
  hipEvent_t s, e; (void)hipEventCreate(&s); (void)hipEventCreate(&e);
  hipLaunchKernelGGL((k<C>), dim3(blocks), dim3(256), 0, 0, d, 1.0001, iters);
  (void)hipEventRecord(s);
  hipLaunchKernelGGL((k<C>), dim3(blocks), dim3(256), 0, 0, d, 1.0001, iters);
  (void)hipEventRecord(e); (void)hipEventSynchronize(e);
  float ms; (void)hipEventElapsedTime(&ms, s, e);
  const double instr_per_simd = (double)waves_per_simd * iters * C * 2;
  printf("chains=%d waves/SIMD=%d: %.3f ms  %.2f ns/instr/SIMD\n", C, waves_per_simd, ms, ms * 1e6 / instr_per_simd);
  (void)hipFree(d);
}
int main() {
  for (int w : {1, 2, 3, 4, 8}) { run<1>(w); run<2>(w); run<4>(w); run<8>(w); }
  return 0;
}
