// Dev micro-benchmark: the fused encoder's RGB row reads (k_encode420: a wave per
// 512-px x 16-row unit, 19 input rows of 1536 B, lane l's pixels at bytes 24 l ..
// 24 l + 23) with the unit's 24 KiB of coefficient writes, under alternative load
// shapes.  No colour / DCT work: this is the memory side alone.
//   A  buffer b128 @ 24 l + b64 @ 24 l + 16 (the kernel's current shape)
//   B  coalesced b128 @ 16 l + b64 @ 1024 + 8 l (1.5 KiB in two dense instructions)
//   C  LDS-DMA: global_load_lds 16 B @ 16 l (64 lanes) + (32 lanes), then 3 x ds_read_b64 @ 24 l
//   D  3 x global b64 @ 24 l (the round-1 shape)
//   E  2 x buffer b96 @ 24 l, 24 l + 12
// Occupancy is held at 2 waves per SIMD (dynamic LDS), rows in flight = LA.
// Build: hipcc --offload-arch=gfx950 -O3 -o rgb_rows rgb_rows.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int V, int LA = 6, bool WR = true>
__global__ __launch_bounds__(256) void k_rows(const uint8_t *__restrict__ img, int H, int W, uint8_t *__restrict__ out,
                                              int nunits) {
  extern __shared__ uint8_t dyn[];  // occupancy pad + the LDS ring of variant C
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
  if (g >= nunits) return;
  const int ns = W / 512, u = __builtin_amdgcn_readfirstlane(g / ns), s = __builtin_amdgcn_readfirstlane(g - u * ns);
  const int pitch = 3 * W, y0 = 16 * u;
  int roff;
  {
    int sy = y0 + lane - 2;
    sy = sy < 0 ? -sy : (sy >= H ? 2 * H - 2 - sy : sy);
    roff = sy * pitch;
  }
  const uint8_t *base = img + 1536 * s;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, H * pitch - 1536 * s, 0x00020000);
  uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
  uint8_t *ring = dyn + wv * (LA + 1) * 1536;
  u32x4 ra[LA + 1];
  u32x2 rb[LA + 1];
  u32x2 rc[LA + 1];
  u32x3 rd[LA + 1], re[LA + 1];
  auto load = [&](int r) {
    const int so = __builtin_amdgcn_readlane(roff, r), k = r % (LA + 1);
    if (V == 0) {
      ra[k] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 24 * lane, so, 0);
      rb[k] = __builtin_amdgcn_raw_buffer_load_b64(rsrc, 24 * lane + 16, so, 0);
    } else if (V == 1) {
      ra[k] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * lane, so, 0);
      rb[k] = __builtin_amdgcn_raw_buffer_load_b64(rsrc, 1024 + 8 * lane, so, 0);
    } else if (V == 2) {
      const uint8_t *p = base + so;
      __builtin_amdgcn_global_load_lds((const void *)(p + 16 * lane), (__attribute__((address_space(3))) void *)(ring + k * 1536), 16, 0, 0);
      if (lane < 32)
        __builtin_amdgcn_global_load_lds((const void *)(p + 1024 + 16 * lane),
                                         (__attribute__((address_space(3))) void *)(ring + k * 1536 + 1024), 16, 0, 0);
    } else if (V == 3) {
      const uint2 *p = reinterpret_cast<const uint2 *>(base + so + 24 * lane);
      const uint2 a = p[0], b = p[1], c = p[2];
      ra[k] = (u32x4){a.x, a.y, b.x, b.y};
      rb[k] = (u32x2){c.x, c.y};
    } else {
      rd[k] = __builtin_amdgcn_raw_buffer_load_b96(rsrc, 24 * lane, so, 0);
      re[k] = __builtin_amdgcn_raw_buffer_load_b96(rsrc, 24 * lane + 12, so, 0);
    }
  };
#pragma unroll
  for (int r = 0; r < LA; ++r) load(r);
#pragma unroll
  for (int r = 0; r < 19; ++r) {
    if (r + LA < 19) load(r + LA);
    const int k = r % (LA + 1);
    uint32_t d[6];
    if (V == 2) {
      // rows r + 1 .. r + LA - 1 may still be in flight: wait for row r only
      if (r + LA < 19)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LA) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint2 *q = reinterpret_cast<const uint2 *>(ring + k * 1536 + 24 * lane);
      const uint2 a = q[0], b = q[1], c = q[2];
      d[0] = a.x, d[1] = a.y, d[2] = b.x, d[3] = b.y, d[4] = c.x, d[5] = c.y;
    } else if (V == 4) {
      d[0] = rd[k].x, d[1] = rd[k].y, d[2] = rd[k].z, d[3] = re[k].x, d[4] = re[k].y, d[5] = re[k].z;
    } else {
      d[0] = ra[k].x, d[1] = ra[k].y, d[2] = ra[k].z, d[3] = ra[k].w, d[4] = rb[k].x, d[5] = rb[k].y;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) acc[i] = acc[i] * 0x9E3779B1u + d[i];
    __builtin_amdgcn_sched_barrier(0);
  }
  // 24 KiB of writes per unit, 1 KiB per store instruction
  if (!WR) {
    if (acc[0] == 0x12345678u && acc[1] == 1u) out[lane] = 1;
    return;
  }
  u32x4 *o = reinterpret_cast<u32x4 *>(out) + (int64_t)g * 24 * 64 + lane;
#pragma unroll
  for (int k = 0; k < 24; ++k) o[64 * k] = (u32x4){acc[k % 6], acc[(k + 1) % 6] ^ k, acc[(k + 2) % 6], acc[(k + 3) % 6]};
}

int main() {
  const int H = 4320, W = 7680, rot = 12;
  const int64_t nrgb = (int64_t)H * W * 3;
  const int nunits = (W / 512) * (H / 16);
  const int64_t nout = (int64_t)nunits * 24 * 1024;
  uint8_t *in[rot], *out[rot];
  for (int i = 0; i < rot; ++i) {
    hipMalloc(&in[i], nrgb);
    hipMemset(in[i], i, nrgb);
    hipMalloc(&out[i], nout);
  }
  const size_t lds = 64 * 1024;  // 2 workgroups (8 waves) per CU
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  const char *names[5] = {"A buffer b128@24l+b64", "B coalesced b128+b64", "C LDS-DMA 16B + ds_read_b64",
                          "D global 3 x b64", "E buffer 2 x b96"};
  const double bytes = (double)nrgb * 19 / 16 + (double)nout;
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 5; ++v) {
      float tot = 0;
      const int n = 14;
      for (int i = 0; i < n; ++i) {
        hipEventRecord(s);
        const dim3 grid((nunits + 3) / 4), block(256);
        if (v == 0) hipLaunchKernelGGL(k_rows<0>, grid, block, lds, 0, in[i % rot], H, W, out[i % rot], nunits);
        if (v == 1) hipLaunchKernelGGL(k_rows<1>, grid, block, lds, 0, in[i % rot], H, W, out[i % rot], nunits);
        if (v == 2) hipLaunchKernelGGL(k_rows<2>, grid, block, lds, 0, in[i % rot], H, W, out[i % rot], nunits);
        if (v == 3) hipLaunchKernelGGL(k_rows<3>, grid, block, lds, 0, in[i % rot], H, W, out[i % rot], nunits);
        if (v == 4) hipLaunchKernelGGL(k_rows<4>, grid, block, lds, 0, in[i % rot], H, W, out[i % rot], nunits);
        hipEventRecord(e);
        hipEventSynchronize(e);
        float ms;
        hipEventElapsedTime(&ms, s, e);
        if (i >= 4) tot += ms;
      }
      const double us = tot / (n - 4) * 1e3;
      printf("%-32s %7.2f us  %6.0f GB/s (reads 19/16 of the image + 24 KiB per unit)\n", names[v], us, bytes / us / 1e3);
    }
  // variant A: rows in flight x occupancy (LDS pad: 64 KiB -> 2 waves / SIMD, 32 KiB -> 4), with / without the writes
  auto sweep = [&](auto kern, const char *name, size_t pad, bool wr) {
    float tot = 0;
    const int n = 14;
    for (int i = 0; i < n; ++i) {
      hipEventRecord(s);
      hipLaunchKernelGGL(kern, dim3((nunits + 3) / 4), dim3(256), pad, 0, in[i % rot], H, W, out[i % rot], nunits);
      hipEventRecord(e);
      hipEventSynchronize(e);
      float ms;
      hipEventElapsedTime(&ms, s, e);
      if (i >= 4) tot += ms;
    }
    const double us = tot / (n - 4) * 1e3, b = (double)nrgb * 19 / 16 + (wr ? (double)nout : 0.0);
    printf("%-32s pad %2zu KiB %7.2f us  %6.0f GB/s\n", name, pad >> 10, us, b / us / 1e3);
  };
  for (size_t pad : {(size_t)65536, (size_t)32768}) {
    sweep(k_rows<0, 4>, "A LA=4", pad, true);
    sweep(k_rows<0, 6>, "A LA=6", pad, true);
    sweep(k_rows<0, 10>, "A LA=10", pad, true);
    sweep(k_rows<0, 14>, "A LA=14", pad, true);
    sweep(k_rows<0, 6, false>, "A LA=6 reads only", pad, false);
    sweep(k_rows<0, 10, false>, "A LA=10 reads only", pad, false);
  }
  hipError_t err = hipGetLastError();
  printf("status: %s\n", hipGetErrorString(err));
  return 0;
}
