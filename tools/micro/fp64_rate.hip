// Microbenchmark: per-SIMD issue rate of v_add_f64 / v_mul_f64 / v_fma_f64 / v_add_f32 / v_add_u32 on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <typename T, int OP>
__global__ __launch_bounds__(256) void k(T *out, T seed, int iters) {
  T a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed + (T)(threadIdx.x + i);
  const T c = seed * (T)0.5 + (T)1;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = a[i] + c;
      else if (OP == 1) a[i] = a[i] * c;
      else if (OP == 2) a[i] = __builtin_fma(a[i], c, c);
      else if (OP == 3) a[i] = a[i] + (T)(int)(it ^ i);  // + int->T convert (add counted separately)
    }
  }
  T s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
  if (s == (T)12345.678) out[threadIdx.x] = s;
}
template <typename T, int OP>
void run(const char *name) {
  T *d; hipMalloc(&d, 1024 * sizeof(T));
  const int iters = 4096, blocks = 256 * 16;
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  hipLaunchKernelGGL((k<T, OP>), dim3(blocks), dim3(256), 0, 0, d, (T)1.0001, iters);
  hipEventRecord(s);
  hipLaunchKernelGGL((k<T, OP>), dim3(blocks), dim3(256), 0, 0, d, (T)1.0001, iters);
  hipEventRecord(e); hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e);
  double waves = blocks * 4.0, instr = waves * iters * 8;
  double per_simd_per_s = instr / 1024 / (ms * 1e-3);
  printf("%-10s %.3f ms  %.2f G wave-instr/s/SIMD  => %.2f cycles/instr @2.4GHz\n", name, ms, per_simd_per_s / 1e9, 2.4e9 / per_simd_per_s);
  hipFree(d);
}
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void kpk(float *out, float seed, int iters) {
  f2 a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (f2){seed + i, seed - i};
  const f2 c = (f2){seed * 0.5f, seed * 0.25f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __builtin_elementwise_fma(a[i], c, c);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
  if (s == 12345.678f) out[threadIdx.x] = s;
}
int main() {
  {
    float *d; hipMalloc(&d, 1024 * sizeof(float));
    const int iters = 4096, blocks = 256 * 16;
    hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
    hipLaunchKernelGGL(kpk, dim3(blocks), dim3(256), 0, 0, d, 1.0001f, iters);
    hipEventRecord(s);
    hipLaunchKernelGGL(kpk, dim3(blocks), dim3(256), 0, 0, d, 1.0001f, iters);
    hipEventRecord(e); hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, s, e);
    double instr = blocks * 4.0 * iters * 8, per = instr / 1024 / (ms * 1e-3);
    printf("%-10s %.3f ms  %.2f G wave-instr/s/SIMD  => %.2f cycles/instr @2.4GHz\n", "pk_fma_f32", ms, per / 1e9, 2.4e9 / per);
  }
  run<double, 0>("add_f64"); run<double, 1>("mul_f64"); run<double, 2>("fma_f64");
  run<float, 0>("add_f32"); run<float, 2>("fma_f32"); run<int, 0>("add_u32");
  run<double, 3>("cvt+add_f64"); run<float, 3>("cvt+add_f32");
  return 0;
}
