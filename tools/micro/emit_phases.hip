// dev: per-phase wave-cycles of the batched RLE emit on dense random blocks (8K luma).
#define HIC_STAMPS 1
#include "../../hiccup_amd/csrc/rle.hip"
#include "../../hiccup_amd/csrc/common.hip"
#include <random>
#include <vector>
int main() {
  const int64_t nblk = 518400, nt = (nblk + 63) / 64;
  std::vector<int16_t> h(nblk * 64);
  std::mt19937 rng(1);
  for (auto &x : h) x = (int16_t)((rng() % 41) - 20);
  int16_t *blocks, *V;
  uint8_t *L;
  int32_t *dc;
  int64_t *ws, *cnt;
  const size_t wsb = hic_rle_workspace_bytes(nblk, 64);
  hipMalloc(&blocks, h.size() * 2);
  hipMemcpy(blocks, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMalloc(&ws, wsb);
  hipMemset(ws, 0, wsb);
  hipMalloc(&cnt, 8);
  hipMalloc(&dc, nblk * 4);
  hipMalloc(&L, nblk * 63 + 1);
  hipMalloc(&V, 2 * (nblk * 63 + 1));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int it = 0; it < 4; ++it) {
    unsigned long long z[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z);
    hipEventRecord(a);
    hic_rle_encode_i16(blocks, nblk, 64, 15, nullptr, dc, L, V, nblk * 63 + 1, cnt, ws, 0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    static unsigned long long tp[1 << 16][8];
    hipMemcpyFromSymbol(tp, HIP_SYMBOL(g_tphase), sizeof tp);
    unsigned long long ph[16] = {0};
    for (int64_t t = 0; t < nt; ++t)
      for (int i = 0; i < 8; ++i) ph[i] += tp[t][i];
    int64_t n;
    hipMemcpy(&n, cnt, 8, hipMemcpyDeviceToHost);
    printf("total %.1f us, %lld symbols | cycles per wave-tile: summarize %llu scans %llu stage %llu wait %llu copyout %llu\n",
           ms * 1e3, (long long)n, ph[1] / nt, ph[2] / nt, ph[3] / nt, ph[4] / nt, ph[5] / nt);
  }
  return 0;
}
