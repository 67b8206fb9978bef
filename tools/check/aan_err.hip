// dev: largest |fast estimate - pocketfft| of y/T over many blocks (host), to size
// the quantiser's tie window.  Build: see tools/check/README.
#include "../../hiccup_amd/csrc/dct_core.h"
#include <math.h>
#include <random>
#include <stdio.h>
extern "C" void orc_dct8(double *c);
using namespace hic;
int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 rng(11);
  double worst = 0;
  for (long i = 0; i < n; ++i) {
    uint8_t px[64];
    const int mode = i % 4;
    for (int k = 0; k < 64; ++k)
      px[k] = mode == 0 ? (uint8_t)rng() : mode == 1 ? (uint8_t)((rng() & 1) * 255)
            : mode == 2 ? (uint8_t)(((k / 8 + k % 8) & 1) ? 255 : 0) ^ (uint8_t)(rng() % 3) : (uint8_t)(rng() % 4 * 85);
    uint2 w[8];
    for (int r = 0; r < 8; ++r) {
      w[r].x = px[8 * r] | px[8 * r + 1] << 8 | px[8 * r + 2] << 16 | (uint32_t)px[8 * r + 3] << 24;
      w[r].y = px[8 * r + 4] | px[8 * r + 5] << 8 | px[8 * r + 6] << 16 | (uint32_t)px[8 * r + 7] << 24;
    }
    int16_t st[64];
    double est[64];
    for (int t = 0; t < 2; ++t) {
      if (t == 0) dct_block_aan<0, HIC_LAYOUT_RASTER_I16>(w, st, nullptr, est);
      else dct_block_aan<1, HIC_LAYOUT_RASTER_I16>(w, st, nullptr, est);
      double b[64];
      for (int k = 0; k < 64; ++k) b[k] = (double)px[k] - 128.0;
      double col[8];
      for (int r = 0; r < 8; ++r) orc_dct8(b + 8 * r);
      for (int j = 0; j < 8; ++j) {
        for (int r = 0; r < 8; ++r) col[r] = b[8 * r + j];
        orc_dct8(col);
        for (int r = 0; r < 8; ++r) b[8 * r + j] = col[r];
      }
      for (int k = 0; k < 64; ++k) {
        if (k == 0 || k == 36) continue;  // computed exactly, not by the fast path
        const double e = fabs(est[k] - b[k] / (double)QT[t][k]);
        if (e > worst) {
          worst = e;
          printf("block %ld table %d coef %d: fast %.17g pocket %.17g err %.3g (2^%.1f)\n", i, t, k, est[k],
                 b[k] / QT[t][k], e, log2(e));
        }
      }
    }
  }
  printf("worst |fast - pocketfft| of y/T: %.3g (2^%.1f)\n", worst, log2(worst));
  return 0;
}
