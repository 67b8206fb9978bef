// Dev micro-benchmark: SIMD cycles per wave64 instruction on gfx950 for the
// instruction classes of the DCT / colour code (float64 add / fma / mul, int->f64
// convert, int32 add, 24-bit mad, dot4, f32 fma), at 1, 2 and 4 waves per SIMD.
// Each wave runs 8 independent chains of N instructions (inline asm, so the
// compiler cannot fold them); SIMD cycles per wave-instruction = wall time x clock
// / (waves per SIMD x 8 N).  The clock is read in-kernel (s_memtime /
// s_memrealtime ratio, 100 MHz real-time counter).
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rates valu_rates.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int N = 8192;  // instructions per chain

#define CHAIN8(OP) \
  OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

template <int K>
__global__ __launch_bounds__(256) void k_rate(double *out, unsigned long long *clk, int seed) {
  const int lane = threadIdx.x;
  double d[8];
  int v[8];
  float f[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    d[i] = (double)(lane + i + seed);
    v[i] = lane * 7 + i + seed;
    f[i] = (float)(lane + i);
  }
  const double c = 1.0000001;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < N; ++it) {
#define OPK(i)                                                                                        \
  if (K == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(c));                              \
  if (K == 1) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(c));                          \
  if (K == 2) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(c));                              \
  if (K == 3) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[i]) : "v"(v[i]));                           \
  if (K == 4) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(lane));                           \
  if (K == 5) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(v[i]) : "v"(lane));                   \
  if (K == 6) asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(v[i]) : "v"(lane));                   \
  if (K == 7) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"((float)c));                   \
  if (K == 8) asm volatile("v_cvt_f32_i32 %0, %1" : "=v"(f[i]) : "v"(v[i]));                           \
  if (K == 9) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(d[i]));                               \
  if (K == 10) asm volatile("v_mov_b64 %0, %1" : "=v"(d[i]) : "v"(d[(i + 1) & 7]));                    \
  if (K == 11) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(d[i]));                              \
  if (K == 12) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(f[i]) : "v"((float)c));                     \
  if (K == 13) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[i]) : "v"(lane));                           \
  if (K == 14) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(v[i]));                                    \
  if (K == 15) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[i]) : "v"(lane));                       \
  if (K == 16) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(lane));                      \
  if (K == 17) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v[i]) : "v"(lane));                        \
  if (K == 18) asm volatile("v_med3_i32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(lane));                      \
  if (K == 19) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(lane));                      \
  if (K == 20) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(v[i]) : "v"(lane));                       \
  if (K == 21) asm volatile("v_sub_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(v[i]) : "v"(lane)); \
  if (K == 22) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(lane));                 \
  if (K == 23) asm volatile("v_pk_mad_u16 %0, %0, %1, %1" : "+v"(v[i]) : "v"(lane));
    CHAIN8(OPK)
#undef OPK
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += d[i] + v[i] + f[i];
  out[blockIdx.x * 256 + lane] = s;
  if (lane == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

int main() {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double *out;
  unsigned long long *clk;
  hipMalloc(&out, sizeof(double) * 256 * cus * 8);
  hipMalloc(&clk, 16);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  const char *names[24] = {"v_add_f64", "v_fma_f64", "v_mul_f64", "v_cvt_f64_i32", "v_add_u32", "v_mad_u32_u24",
                           "v_dot4_u32_u8", "v_fma_f32", "v_cvt_f32_i32", "v_lshl_add_u64", "v_mov_b64",
                           "v_pk_fma_f32", "v_fmac_f32", "v_sub_u32", "v_lshlrev_b32", "v_mul_u32_u24",
                           "v_perm_b32", "v_pk_add_u16", "v_med3_i32", "v_add3_u32", "v_add_u32_e64",
                           "v_sub_u32_sdwa", "v_cndmask_b32", "v_pk_mad_u16"};
  for (int wps : {2, 4}) {  // waves per SIMD: workgroups of 4 waves, wps per CU
    const int blocks = cus * wps;
    for (int k = 0; k < 24; ++k) {
      float best = 1e9;
      unsigned long long h[2] = {0, 0};
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(s);
#define L(K) \
  if (k == K) hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, clk, rep);
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17)
        L(18) L(19) L(20) L(21) L(22) L(23)
#undef L
        hipEventRecord(e);
        hipEventSynchronize(e);
        float ms;
        hipEventElapsedTime(&ms, s, e);
        if (ms < best) best = ms;
        hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
      }
      const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0;  // memrealtime = 100 MHz
      // SIMD cycles per wave-instruction from the wall time at the in-kernel clock:
      // every SIMD runs wps waves x 8 N instructions
      const double cyc = best * 1e-3 * ghz * 1e9 / ((double)wps * 8.0 * N);
      printf("%-16s waves/SIMD %d: %6.2f SIMD cycles per wave-instruction (clock %.2f GHz, wall %.3f ms)\n",
             names[k], wps, cyc, ghz, best);
    }
  }
  return 0;
}
