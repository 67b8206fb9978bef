// dev: the float32 fast path + float64 fallback + exact replica (the production
// forward kernel's three tiers, same __host__ __device__ code) vs the exact
// pocketfft replica, on the host.  Reports mismatches (must be 0), fast-path flag
// rates, zero-ambiguous flags per 64-block set and fallback-window escalations.
//   hipcc -O2 -std=c++17 -ffp-contract=off -x hip --offload-arch=gfx950 -o /tmp/f32_check tools/check/f32_check.hip
//   /tmp/f32_check 2000000
#include "../../hiccup_amd/csrc/dct_core.h"
#include <random>
#include <stdio.h>
#include <vector>
using namespace hic;

static void gen(std::mt19937_64 &rng, int mode, uint8_t (&px)[64]) {
  if (mode == 6) {  // chroma-like: 5x5 binomial blur of uniform noise (pyrDown of random RGB)
    static const int k5[5] = {1, 4, 6, 4, 1};
    int src[12][12];
    for (auto &r : src)
      for (int &v : r) v = (int)(rng() % 256);
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        int s = 0;
        for (int i = 0; i < 5; ++i)
          for (int j = 0; j < 5; ++j) s += k5[i] * k5[j] * src[y + i][x + j];
        px[8 * y + x] = (uint8_t)((s + 128) >> 8);
      }
    return;
  }
  for (int k = 0; k < 64; ++k) {
    switch (mode) {
      case 0: px[k] = (uint8_t)rng(); break;                                      // uniform
      case 1: px[k] = (uint8_t)(128 + (int)(rng() % 9) - 4); break;               // near-flat
      case 2: px[k] = (uint8_t)(((k & 7) < 4) ? rng() % 256 : px[k - 4]); break;  // mirrored rows
      case 3: px[k] = (uint8_t)(rng() % 2 ? 255 : 0); break;                      // saturated
      case 4: px[k] = (uint8_t)(rng() % 2 ? 128 + 2 * (int)(rng() % 64) : 128 - 2 * (int)(rng() % 64)); break;
      default: px[k] = (uint8_t)((rng() % 4) * 85); break;                        // 4 levels
    }
  }
}

static long g_hist[2][64];
struct Stats {
  long blocks = 0, bad = 0, flags = 0, zamb = 0, t3 = 0, sets = 0, sets_zamb = 0, sets_flag = 0;
};

template <int TABLE>
static void run(std::mt19937_64 &rng, int mode, long n, Stats &S) {
  for (long i0 = 0; i0 < n; i0 += 64) {
    bool set_z = false, set_f = false;
    for (int b = 0; b < 64; ++b) {
      uint8_t px[64];
      gen(rng, mode, px);
      uint2 w[8];
      for (int r = 0; r < 8; ++r) {
        w[r].x = px[8 * r] | px[8 * r + 1] << 8 | px[8 * r + 2] << 16 | (uint32_t)px[8 * r + 3] << 24;
        w[r].y = px[8 * r + 4] | px[8 * r + 5] << 8 | px[8 * r + 6] << 16 | (uint32_t)px[8 * r + 7] << 24;
      }
      int16_t a[64], e[64];
      std::vector<int> fl;
      dct_block_f32<TABLE, HIC_LAYOUT_RASTER_I16>(w, a, [&](int v, const float (&rr)[8], const float (&d)[8],
                                                            const bool (&f)[8]) {
        for (int u = 0; u < 8; ++u) {
          if (!f[u]) continue;
          fl.push_back(u * 8 + v);
          const bool z = rr[u] == 0.f || (rr[u] == 1.f && d[u] < 0.f) || (rr[u] == -1.f && d[u] > 0.f);
          S.zamb += z;
          set_z |= z;
        }
      });
      S.flags += (long)fl.size();
      set_f |= !fl.empty();
      bool redo = false;
      for (int i : fl) {
        int q;
        if (resolve_coef(w, TABLE, i, q))
          a[i] = (int16_t)q;
        else {
          redo = true;
          ++g_hist[TABLE][i];
        }
      }
      uint2 w2[8];
      for (int r = 0; r < 8; ++r) w2[r] = w[r];
      dct_block_2ph<TABLE, HIC_LAYOUT_RASTER_I16>(w2, e);
      if (redo) {
        ++S.t3;
        for (int k = 0; k < 64; ++k) a[k] = e[k];
      }
      for (int k = 0; k < 64; ++k)
        if (a[k] != e[k]) {
          if (S.bad < 8) printf("  mode %d table %d: coef %d fast %d exact %d\n", mode, TABLE, k, a[k], e[k]);
          ++S.bad;
        }
      ++S.blocks;
    }
    ++S.sets;
    S.sets_zamb += set_z;
    S.sets_flag += set_f;
  }
}

int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 rng(11);
  long bad = 0;
  const char *names[7] = {"uniform", "near-flat", "mirrored", "saturated", "tie-stress", "4-level", "chroma-blur"};
  for (int mode = 0; mode < 7; ++mode)
    for (int t = 0; t < 2; ++t) {
      Stats S;
      if (t == 0)
        run<0>(rng, mode, n, S);
      else
        run<1>(rng, mode, n, S);
      bad += S.bad;
      printf("%-11s table %d: %ld blocks, mismatches %ld, flags/block %.4f, zero-amb/block %.5f, "
             "sets w/ flag %.3f, sets w/ zero-amb %.4f, exact redo/block %.2e\n",
             names[mode], t, S.blocks, S.bad, (double)S.flags / S.blocks, (double)S.zamb / S.blocks,
             (double)S.sets_flag / S.sets, (double)S.sets_zamb / S.sets, (double)S.t3 / S.blocks);
    }
  for (int t = 0; t < 2; ++t) {
    printf("redo triggers table %d:", t);
    for (int i = 0; i < 64; ++i)
      if (g_hist[t][i]) printf(" (%d,%d):%ld", i / 8, i % 8, g_hist[t][i]);
    printf("\n");
  }
  printf(bad ? "FAIL: %ld mismatches\n" : "OK: 0 mismatches\n", bad);
  return bad != 0;
}
