// dev: the AAN fast path + tie fallback vs the exact pocketfft replica, on the
// host (same __host__ __device__ code as the kernels): random blocks, flat and
// striped blocks, and the tie-stress planes.  Reports mismatches and the
// fallback rate.
#include "../../hiccup_amd/csrc/dct_core.h"
#include <random>
#include <stdio.h>
using namespace hic;
template <int TABLE>
static void run(const char *name, std::mt19937_64 &rng, int mode, long n, long &bad, long &flags) {
  for (long i = 0; i < n; ++i) {
    uint8_t px[64];
    for (int k = 0; k < 64; ++k) {
      switch (mode) {
        case 0: px[k] = (uint8_t)rng(); break;                                   // uniform
        case 1: px[k] = (uint8_t)(128 + (int)(rng() % 9) - 4); break;            // near-flat
        case 2: px[k] = (uint8_t)(((k & 7) < 4) ? rng() % 256 : px[k - 4]); break;  // mirrored rows
        case 3: px[k] = (uint8_t)((k / 8 + k % 8) % 2 ? 255 : 0); break;         // checkerboard
        case 4: px[k] = (uint8_t)(rng() % 2 ? 128 + 2 * (int)(rng() % 64) : 128 - 2 * (int)(rng() % 64)); break;
        default: px[k] = (uint8_t)((rng() % 4) * 85); break;                     // 4 levels
      }
    }
    uint2 w[8];
    for (int r = 0; r < 8; ++r) {
      w[r].x = px[8 * r] | px[8 * r + 1] << 8 | px[8 * r + 2] << 16 | (uint32_t)px[8 * r + 3] << 24;
      w[r].y = px[8 * r + 4] | px[8 * r + 5] << 8 | px[8 * r + 6] << 16 | (uint32_t)px[8 * r + 7] << 24;
    }
    int16_t a[64], e[64];
    bool t26 = false;
    const bool f = dct_block_aan<TABLE, HIC_LAYOUT_RASTER_I16>(w, a, &t26);
    if (t26) {
      int q[4];
      dct_fix26<TABLE>(w, q);
      a[18] = (int16_t)q[0], a[22] = (int16_t)q[1], a[50] = (int16_t)q[2], a[54] = (int16_t)q[3];
    }
    uint2 w2[8];
    for (int r = 0; r < 8; ++r) w2[r] = w[r];
    dct_block_2ph<TABLE, HIC_LAYOUT_RASTER_I16>(w2, e);
    flags += f;
    if (!f)
      for (int k = 0; k < 64; ++k)
        if (a[k] != e[k]) {
          if (bad < 5) printf("  %s mode %d: coef %d fast %d exact %d\n", name, mode, k, a[k], e[k]);
          ++bad;
        }
  }
}
int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 rng(7);
  for (int mode = 0; mode < 6; ++mode) {
    long bad = 0, flags = 0;
    run<0>("lum", rng, mode, n, bad, flags);
    run<1>("chr", rng, mode, n, bad, flags);
    printf("mode %d: %ld blocks, mismatches %ld, fallback %.5f%%\n", mode, 2 * n, bad, 100.0 * flags / (2.0 * n));
  }
  return 0;
}
