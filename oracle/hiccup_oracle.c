/*
 * hiccup_oracle.c -- CPU ORACLE (scalar C restatement) of hiccup's
 * 8x8 DCT / quantize / zig-zag / DC-DPCM / RLE path and its inverse.
 *
 * TEST INFRASTRUCTURE ONLY.  It is never linked into the product library
 * (hiccup_amd/lib/libhiccup_hip.so).  tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it (via oracle/oracle_c.py) purely as the
 * checker / the CPU baseline.
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off: IEEE binary64, no FMA).
 *
 * What it restates (reference = /root/reference, hiccup @ v0):
 *   orc_dct8 / orc_idct8   scipy.fftpack.dct / idct (type II/III, norm=None) as
 *                          called by transform.dct2 / idct2 (transform.py:67-103);
 *                          scipy 1.15.3 pocketfft length-8 arithmetic, op by op
 *                          (pinned bitwise by
 *                          tests/golden/transform_cases.npz dct2_out/idct2_out).
 *   orc_dct_channel        transform.dct_channel (transform.py:182-193) with
 *                          quantization.jpeg_quantize (quantization.py:47-52,80-81).
 *   orc_inv_dct_channel    transform.inv_dct_channel (transform.py:169-179) with
 *                          quantization.invert_jpeg_quantize (quantization.py:55-57);
 *                          astype(uint8) = truncate toward zero, wrap mod 256.
 *   orc_zigzag_indices     transform._zigzag_indices (transform.py:106-124).
 *   orc_dpcm               codec.differential_coding / utils.differences
 *                          (codec.py:47-52, utils.py:51-63).
 *   orc_rle_encode         codec.run_length_coding (codec.py:55-99), linear time.
 *   orc_rle_decode         codec.decode_run_length (codec.py:102-113).
 *   orc_rgb_to_ycrcb, orc_ycrcb_to_rgb, orc_pyr_down, orc_pyr_up
 *                          OpenCV 8U cvtColor / pyrDown / pyrUp as called at
 *                          compression.py:21,56 and transform.py:151-166.
 *                          PARITY UNPINNED (OpenCV absent; restated from its
 *                          published fixed-point algorithm).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const double WR = 0x1.6a09e667f3bccp-1;
static const double WI = 0x1.6a09e667f3bcdp-1;
static const double TW[7] = {0x1.f6297cff75cb0p-1, 0x1.d906bcf328d46p-1, 0x1.a9b66290ea1a3p-1,
                             0x1.6a09e667f3bccp-1, 0x1.1c73b39ae68c8p-1, 0x1.87de2a6aea963p-2,
                             0x1.8f8b83c69a60ap-3};

/* quantization.py:14-37 */
static const int32_t QT[2][64] = {
    {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
     14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
     18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
     49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99},
    {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
     24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99}};

const int32_t *orc_qtable(int table_id) { return QT[table_id ? 1 : 0]; }

/* scipy.fftpack.dct(c, type=2), n = 8, in place */
void orc_dct8(double *c) {
  double h[8], d[8];
  c[0] *= 2.0;
  c[7] *= 2.0;
  for (int k = 1; k <= 5; k += 2) {
    double a = c[k + 1], b = c[k];
    c[k + 1] = a - b;
    c[k] = b + a;
  }
  h[0] = c[0] + c[7];
  h[4] = c[0] - c[7];
  h[3] = 2.0 * c[3];
  h[7] = -2.0 * c[4];
  h[1] = c[1] + c[5];
  double tr2 = c[1] - c[5];
  double ti2 = c[2] + c[6];
  h[2] = c[2] - c[6];
  h[6] = WR * ti2 + WI * tr2;
  h[5] = WR * tr2 - WI * ti2;
  for (int k = 0; k < 2; ++k) {
    double t2 = h[4 * k] + h[4 * k + 3];
    double t1 = h[4 * k] - h[4 * k + 3];
    double t3 = 2.0 * h[4 * k + 1];
    double t4 = 2.0 * h[4 * k + 2];
    d[k] = t2 + t3;
    d[k + 4] = t2 - t3;
    d[k + 6] = t1 + t4;
    d[k + 2] = t1 - t4;
  }
  static const int KS[3][2] = {{1, 7}, {2, 6}, {3, 5}};
  for (int i = 0; i < 3; ++i) {
    int k = KS[i][0], kc = KS[i][1];
    double t1 = TW[k - 1] * d[kc] + TW[kc - 1] * d[k];
    double t2 = TW[k - 1] * d[k] - TW[kc - 1] * d[kc];
    d[k] = 0.5 * (t1 + t2);
    d[kc] = 0.5 * (t1 - t2);
  }
  d[4] *= TW[3];
  memcpy(c, d, sizeof d);
}

/* scipy.fftpack.idct(c, type=2) = unnormalised DCT-III, n = 8, in place */
void orc_idct8(double *c) {
  double h[8], d[8];
  static const int KS[3][2] = {{1, 7}, {2, 6}, {3, 5}};
  for (int i = 0; i < 3; ++i) {
    int k = KS[i][0], kc = KS[i][1];
    double t1 = c[k] + c[kc];
    double t2 = c[k] - c[kc];
    c[k] = TW[k - 1] * t2 + TW[kc - 1] * t1;
    c[kc] = TW[k - 1] * t1 - TW[kc - 1] * t2;
  }
  c[4] *= (2.0 * TW[3]);
  for (int k = 0; k < 2; ++k) {
    double tr1 = c[k + 6] + c[k + 2];
    h[4 * k + 2] = c[k + 6] - c[k + 2];
    double tr2 = c[k] + c[k + 4];
    h[4 * k + 1] = c[k] - c[k + 4];
    h[4 * k] = tr2 + tr1;
    h[4 * k + 3] = tr2 - tr1;
  }
  d[0] = h[0] + h[4];
  d[7] = h[0] - h[4];
  d[4] = -h[7];
  d[3] = h[3];
  double tr2 = WR * h[5] + WI * h[6];
  double ti2 = WR * h[6] - WI * h[5];
  d[1] = h[1] + tr2;
  d[5] = h[1] - tr2;
  d[2] = ti2 + h[2];
  d[6] = ti2 - h[2];
  for (int k = 1; k <= 5; k += 2) {
    double a = d[k], b = d[k + 1];
    d[k] = a - b;
    d[k + 1] = b + a;
  }
  memcpy(c, d, sizeof d);
}

/* transform.dct2: rows then columns */
static void dct2_block(double b[64]) {
  double col[8];
  for (int r = 0; r < 8; ++r) orc_dct8(b + 8 * r);
  for (int j = 0; j < 8; ++j) {
    for (int i = 0; i < 8; ++i) col[i] = b[8 * i + j];
    orc_dct8(col);
    for (int i = 0; i < 8; ++i) b[8 * i + j] = col[i];
  }
}

/* transform.idct2: rows, columns, then /256 */
static void idct2_block(double b[64]) {
  double col[8];
  for (int r = 0; r < 8; ++r) orc_idct8(b + 8 * r);
  for (int j = 0; j < 8; ++j) {
    for (int i = 0; i < 8; ++i) col[i] = b[8 * i + j];
    orc_idct8(col);
    for (int i = 0; i < 8; ++i) b[8 * i + j] = col[i];
  }
  for (int i = 0; i < 64; ++i) b[i] = b[i] / 256.0;
}

void orc_dct2(const int64_t *in, double *out) {
  for (int i = 0; i < 64; ++i) out[i] = (double)in[i];
  dct2_block(out);
}

void orc_idct2(const double *in, double *out) {
  memcpy(out, in, 64 * sizeof(double));
  idct2_block(out);
}

/* One block row range [br0, br1) of dct_channel. */
static void dct_rows(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                     int32_t *out, int64_t br0, int64_t br1) {
  const int32_t *T = orc_qtable(table_id);
  const int64_t nbx = (W + 7) / 8;
  double b[64];
  for (int64_t bi = br0; bi < br1; ++bi)
    for (int64_t bj = 0; bj < nbx; ++bj) {
      for (int u = 0; u < 8; ++u)
        for (int v = 0; v < 8; ++v) {
          int64_t y = 8 * bi + u, x = 8 * bj + v;
          /* pad_matrix pads the int64 (pixel - 128) plane with 0 */
          b[8 * u + v] = (y < H && x < W) ? (double)((int64_t)plane[y * stride + x] - 128) : 0.0;
        }
      dct2_block(b);
      for (int u = 0; u < 8; ++u)
        for (int v = 0; v < 8; ++v) {
          int64_t y = 8 * bi + u, x = 8 * bj + v;
          if (y < H && x < W)  /* merge_blocks crops */
            out[y * W + x] = (int32_t)nearbyint(b[8 * u + v] / (double)T[8 * u + v]);
        }
    }
}

int orc_dct_channel(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                    int32_t *out) {
  if (H <= 0 || W <= 0) return -1;
  dct_rows(plane, H, W, stride, table_id, out, 0, (H + 7) / 8);
  return 0;
}

typedef struct {
  const uint8_t *plane;
  int64_t H, W, stride;
  int table_id;
  int32_t *out;
  int64_t br0, br1;
} dct_job;

static void *dct_thread(void *p) {
  dct_job *j = (dct_job *)p;
  dct_rows(j->plane, j->H, j->W, j->stride, j->table_id, j->out, j->br0, j->br1);
  return NULL;
}

/* Same as orc_dct_channel, block rows split across nthreads pthreads. */
int orc_dct_channel_mt(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                       int32_t *out, int nthreads) {
  if (H <= 0 || W <= 0) return -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  int64_t nby = (H + 7) / 8;
  pthread_t th[256];
  dct_job jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (dct_job){plane, H, W, stride, table_id, out, nby * t / nthreads, nby * (t + 1) / nthreads};
    pthread_create(&th[t], NULL, dct_thread, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}

int orc_inv_dct_channel(const int32_t *coef, int64_t H, int64_t W, int table_id, uint8_t *out) {
  if (H <= 0 || W <= 0) return -1;
  const int32_t *T = orc_qtable(table_id);
  const int64_t nby = (H + 7) / 8, nbx = (W + 7) / 8;
  double b[64];
  for (int64_t bi = 0; bi < nby; ++bi)
    for (int64_t bj = 0; bj < nbx; ++bj) {
      for (int u = 0; u < 8; ++u)
        for (int v = 0; v < 8; ++v) {
          int64_t y = 8 * bi + u, x = 8 * bj + v;
          int64_t q = (y < H && x < W) ? (int64_t)coef[y * W + x] : 0;
          b[8 * u + v] = (double)(q * (int64_t)T[8 * u + v]);
        }
      idct2_block(b);
      for (int u = 0; u < 8; ++u)
        for (int v = 0; v < 8; ++v) {
          int64_t y = 8 * bi + u, x = 8 * bj + v;
          if (y < H && x < W) {
            double p = b[8 * u + v] + 128.0;
            out[y * W + x] = (uint8_t)((int64_t)p & 0xFF);  /* trunc, wrap */
          }
        }
    }
  return 0;
}

/* transform._zigzag_indices for an h x w matrix: raster indices. */
void orc_zigzag_indices(int h, int w, int32_t *idx) {
  int n = 0;
  for (int s = 0; s <= h + w - 2; ++s) {
    int ylo = s - (w - 1) > 0 ? s - (w - 1) : 0;
    int yhi = s < h - 1 ? s : h - 1;
    if (s % 2 == 0)
      for (int y = ylo; y <= yhi; ++y) idx[n++] = y * w + (s - y);
    else
      for (int y = yhi; y >= ylo; --y) idx[n++] = y * w + (s - y);
  }
}

/* split_matrix(raster, N) + zigzag per block: out[nblk][N*N] */
int64_t orc_zigzag_blocks(const int32_t *raster, int64_t H, int64_t W, int N, int32_t *out) {
  int32_t zz[4096];
  if (N <= 0 || N > 64) return -1;
  orc_zigzag_indices(N, N, zz);
  int64_t nby = (H + N - 1) / N, nbx = (W + N - 1) / N, b = 0;
  for (int64_t bi = 0; bi < nby; ++bi)
    for (int64_t bj = 0; bj < nbx; ++bj, ++b)
      for (int z = 0; z < N * N; ++z) {
        int64_t y = bi * N + zz[z] / N, x = bj * N + zz[z] % N;
        out[b * N * N + z] = (y < H && x < W) ? raster[y * W + x] : 0;
      }
  return b;
}

void orc_dpcm(const int32_t *dc, int64_t n, int32_t *out) {
  for (int64_t i = n - 1; i > 0; --i) out[i] = dc[i] - dc[i - 1];
  if (n > 0) out[0] = dc[0];
}

/* codec.run_length_coding; returns the symbol count or -1 if cap is short. */
int64_t orc_rle_encode(const int32_t *arr, int64_t n, int64_t max_len, int32_t *out_len,
                       int32_t *out_val, int64_t cap) {
  int64_t ns = 0, run = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (arr[i] == 0) {
      ++run;
      continue;
    }
    if (max_len > 0) {
      int64_t div = run / max_len;
      for (int64_t k = 0; k < div; ++k) {
        if (ns >= cap) return -1;
        out_len[ns] = (int32_t)(max_len - 1);
        out_val[ns++] = 0;
      }
      run -= div * max_len;
    }
    if (ns >= cap) return -1;
    out_len[ns] = (int32_t)run;
    out_val[ns++] = arr[i];
    run = 0;
  }
  if (n == 0 || arr[n - 1] == 0) {
    if (ns >= cap) return -1;
    out_len[ns] = 0;
    out_val[ns++] = 0;
  }
  return ns;
}

/* codec.decode_run_length; returns the decoded length or -1 if cap is short. */
int64_t orc_rle_decode(const int32_t *len, const int32_t *val, int64_t nsym, int64_t length,
                       int32_t *out, int64_t cap) {
  int64_t p = 0;
  for (int64_t s = 0; s < nsym; ++s) {
    if (p + len[s] + 1 > cap) return -1;
    for (int32_t k = 0; k < len[s]; ++k) out[p++] = 0;
    out[p++] = val[s];
  }
  if (nsym > 0 && len[nsym - 1] == 0 && val[nsym - 1] == 0)
    while (p < length) {
      if (p >= cap) return -1;
      out[p++] = 0;
    }
  return p;
}

/* ---------------- OpenCV 8U restatements (PARITY UNPINNED) ---------------- */
static inline uint8_t sat8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
#define DESCALE14(x) (((x) + (1 << 13)) >> 14)

void orc_rgb_to_ycrcb(const uint8_t *rgb, int64_t npix, uint8_t *y, uint8_t *cr, uint8_t *cb) {
  for (int64_t i = 0; i < npix; ++i) {
    int r = rgb[3 * i], g = rgb[3 * i + 1], b = rgb[3 * i + 2];
    int Y = DESCALE14(r * 4899 + g * 9617 + b * 1868);
    y[i] = sat8(Y);
    cr[i] = sat8(DESCALE14((r - Y) * 11682 + (128 << 14)));
    cb[i] = sat8(DESCALE14((b - Y) * 9241 + (128 << 14)));
  }
}

void orc_ycrcb_to_rgb(const uint8_t *y, const uint8_t *cr, const uint8_t *cb, int64_t npix,
                      uint8_t *rgb) {
  for (int64_t i = 0; i < npix; ++i) {
    int Y = y[i], Cr = cr[i] - 128, Cb = cb[i] - 128;
    rgb[3 * i + 0] = sat8(Y + DESCALE14(Cr * 22987));
    rgb[3 * i + 1] = sat8(Y + DESCALE14(Cb * -5636 + Cr * -11698));
    rgb[3 * i + 2] = sat8(Y + DESCALE14(Cb * 29049));
  }
}

static inline int64_t refl101(int64_t i, int64_t n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

void orc_pyr_down(const uint8_t *src, int64_t H, int64_t W, uint8_t *dst, int64_t DH, int64_t DW) {
  static const int K[5] = {1, 4, 6, 4, 1};
  for (int64_t oy = 0; oy < DH; ++oy)
    for (int64_t ox = 0; ox < DW; ++ox) {
      int acc = 0;
      for (int a = 0; a < 5; ++a) {
        int64_t sy = refl101(2 * oy + a - 2, H);
        int row = 0;
        for (int b = 0; b < 5; ++b) row += K[b] * src[sy * W + refl101(2 * ox + b - 2, W)];
        acc += K[a] * row;
      }
      dst[oy * DW + ox] = sat8((acc + 128) >> 8);
    }
}

void orc_pyr_up(const uint8_t *src, int64_t H, int64_t W, uint8_t *dst, int64_t DH, int64_t DW) {
  for (int64_t oy = 0; oy < DH; ++oy)
    for (int64_t ox = 0; ox < DW; ++ox) {
      int64_t sy = oy >> 1, sx = ox >> 1;
      int64_t ys[3] = {sy > 0 ? sy - 1 : (H > 1 ? 1 : 0), sy, sy + 1 < H ? sy + 1 : H - 1};
      int64_t xs[3] = {sx > 0 ? sx - 1 : (W > 1 ? 1 : 0), sx, sx + 1 < W ? sx + 1 : W - 1};
      int wy[3], wx[3];
      if (oy & 1) { wy[0] = 0; wy[1] = 4; wy[2] = 4; } else { wy[0] = 1; wy[1] = 6; wy[2] = 1; }
      if (ox & 1) { wx[0] = 0; wx[1] = 4; wx[2] = 4; } else { wx[0] = 1; wx[1] = 6; wx[2] = 1; }
      int acc = 0;
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) acc += wy[a] * wx[b] * src[ys[a] * W + xs[b]];
      dst[oy * DW + ox] = sat8((acc + 32) >> 6);
    }
}
