// HBM bandwidth ceilings for the access shapes this path uses (dev tool).
// Every kernel streams >= 1.2 GB of rotated buffers, so the 256 MiB Infinity
// Cache does not help.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_read16(const uint4 *__restrict__ a, int64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_write16(uint4 *__restrict__ a, int64_t n) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    a[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ __launch_bounds__(256) void k_copy16(const uint4 *__restrict__ a, uint4 *__restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}
// 2:1 read:write (the colour op's 3 B in, 1.5 B out): reads 2 uint4, writes 1 uint4
__global__ __launch_bounds__(256) void k_r2w1(const uint4 *__restrict__ a, uint4 *__restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint4 x = a[2 * i], y = a[2 * i + 1];
    b[i] = make_uint4(x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w);
  }
}
// 1:2 read:write (the DCT's 1 B in, 2 B out)
__global__ __launch_bounds__(256) void k_r1w2(const uint4 *__restrict__ a, uint4 *__restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint4 x = a[i];
    b[2 * i] = x;
    b[2 * i + 1] = make_uint4(x.w, x.z, x.y, x.x);
  }
}

// narrow stores: T per lane, consecutive lanes consecutive
template <typename T>
__global__ __launch_bounds__(256) void k_writeT(T *__restrict__ a, int64_t n) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) a[i] = (T)i;
}
// dwordx3 loads at 12-byte lane stride (the colour kernel's pattern)
__global__ __launch_bounds__(256) void k_read12(const uint8_t *__restrict__ a, int64_t n12, uint32_t *out) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n12; i += (int64_t)gridDim.x * 256) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(a + 12 * i);
    acc ^= p[0] ^ p[1] ^ p[2];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int rot = 8;
  const size_t bytes = 256ull << 20;  // 256 MiB per buffer
  uint4 *buf[rot];
  for (int i = 0; i < rot; ++i) {
    hipMalloc(&buf[i], bytes);
    hipMemset(buf[i], i, bytes);
  }
  uint32_t *o;
  hipMalloc(&o, 64);
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  const int64_t n16 = bytes / 16;
  for (int gmul : {4, 8, 16}) {
    const dim3 g(cus * gmul), b(256);
    auto time = [&](const char *name, double moved, auto launch) {
      for (int w = 0; w < 2; ++w) launch(w);
      hipEventRecord(s);
      const int reps = 8;
      for (int r = 0; r < reps; ++r) launch(r);
      hipEventRecord(e);
      hipEventSynchronize(e);
      float ms;
      hipEventElapsedTime(&ms, s, e);
      printf("grid=%4dxCU %-8s %8.1f GB/s\n", gmul, name, moved * reps / (ms * 1e-3) / 1e9);
    };
    time("read16", bytes, [&](int r) { hipLaunchKernelGGL(k_read16, g, b, 0, 0, buf[r % rot], n16, o); });
    time("write16", bytes, [&](int r) { hipLaunchKernelGGL(k_write16, g, b, 0, 0, buf[r % rot], n16); });
    time("copy16", 2.0 * bytes / 2, [&](int r) {
      hipLaunchKernelGGL(k_copy16, g, b, 0, 0, buf[r % rot], buf[(r + 4) % rot], n16 / 2);
    });
    time("r2w1", 1.5 * bytes, [&](int r) {
      hipLaunchKernelGGL(k_r2w1, g, b, 0, 0, buf[r % rot], buf[(r + 4) % rot], n16 / 2);
    });
    time("r1w2", 1.5 * bytes, [&](int r) {
      hipLaunchKernelGGL(k_r1w2, g, b, 0, 0, buf[r % rot], buf[(r + 4) % rot], n16 / 2);
    });
    time("write2", bytes, [&](int r) {
      hipLaunchKernelGGL((k_writeT<uint16_t>), g, b, 0, 0, reinterpret_cast<uint16_t *>(buf[r % rot]), (int64_t)bytes / 2);
    });
    time("write4", bytes, [&](int r) {
      hipLaunchKernelGGL((k_writeT<uint32_t>), g, b, 0, 0, reinterpret_cast<uint32_t *>(buf[r % rot]), (int64_t)bytes / 4);
    });
    time("write8", bytes, [&](int r) {
      hipLaunchKernelGGL((k_writeT<uint64_t>), g, b, 0, 0, reinterpret_cast<uint64_t *>(buf[r % rot]), (int64_t)bytes / 8);
    });
    time("read12", bytes, [&](int r) {
      hipLaunchKernelGGL(k_read12, g, b, 0, 0, reinterpret_cast<const uint8_t *>(buf[r % rot]), (int64_t)bytes / 12, o);
    });
  }
  return 0;
}
