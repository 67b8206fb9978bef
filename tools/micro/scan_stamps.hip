// dev: phase timestamps of the RLE scan kernel on synthetic tile records.
#define HIC_STAMPS 1
#include "../../hiccup_amd/csrc/rle.hip"
#include "../../hiccup_amd/csrc/common.hip"
#include <vector>
int main() {
  const int64_t nblk = 518400, nt = (nblk + 63) / 64;
  std::vector<int64_t> h(5 * nt + 8, 0);
  for (int64_t t = 0; t < nt; ++t) {
    h[t * 3 + 0] = t * 64 * 63 + 2;
    h[t * 3 + 1] = t * 64 * 63 + 64 * 63 - 3;
    h[t * 3 + 2] = 3900;
  }
  int64_t *ws, *cnt;
  uint8_t *L;
  int16_t *V;
  hipMalloc(&ws, h.size() * 8);
  hipMalloc(&cnt, 8);
  hipMalloc(&L, nblk * 63 + 1);
  hipMalloc(&V, 2 * (nblk * 63 + 1));
  hipMemcpy(ws, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int it = 0; it < 5; ++it) {
    hipEventRecord(a);
    hipLaunchKernelGGL((k_rle_scan<uint8_t, int16_t>), dim3(1), dim3(kScanT), 0, 0, ws, ws + 3 * nt, nt, nblk * 63, 15,
                       nullptr, L, V, nblk * 63 + 1, cnt);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long st[64];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof st);
    printf("event %.2f us | phases (cycles of s_memtime from stamp 0):", ms * 1e3);
    for (int i = 1; i <= 5; ++i) printf(" %llu", st[i] - st[0]);
    printf("\n");
  }
  return 0;
}
