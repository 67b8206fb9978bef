// color.hip -- RGB <-> YCrCb (OpenCV 8U fixed point) and the 4:2:0 chroma
// pyramid (cv2.pyrDown / cv2.pyrUp), as called by compression.jpeg_compression /
// jpeg_decompression (compression.py:16-56) and transform.down_sample / up_sample
// (transform.py:151-166).
//
// PARITY UNPINNED: OpenCV is absent from this image, so these kernels restate
// OpenCV's published 8U algorithms (yuv_shift = 14 fixed point; pyrDown 5x5
// [1 4 6 4 1]^2 / 256 with BORDER_REFLECT_101; pyrUp [1 6 1]/[4 4] taps with
// OpenCV's reflect-101-left / replicate-right edge rule) and are checked against
// the oracle's restatement (oracle/oracle.py), not against cv2 itself.
#include <stdlib.h>

#include <type_traits>

#include "color_core.h"

namespace hic {
namespace {

// ---------------------------------------------------------------------------
// Fused cvtColor(RGB2YCrCb) + pyrDown(Cr), pyrDown(Cb): one workgroup per
// TX x TY tile of chroma output; the full-resolution Cr/Cb region it needs
// (with a 2-pixel halo, reflect-101 at image borders) lives only in LDS.
constexpr int TX = 32, TY = 16;
constexpr int RW = 2 * TX + 8;  // region columns [2*ox0 - 4, 2*ox0 + 2*TX + 4): 4-pixel aligned
constexpr int RH = 2 * TY + 4;  // region rows    [2*oy0 - 2, 2*oy0 + 2*TY + 2)

// Row-shard form: the input holds image rows [in_row0, in_row0 + in_rows) of an
// H x W image (a shard plus its 2-row pyrDown halo); the kernel writes Y rows
// [out_row0, out_row0 + out_rows) (to y, relative to out_row0) and chroma rows
// [out_row0/2, out_row0/2 + dh_out) (relative).  Reflect-101 happens only at the
// true image border, so a shard's output equals the same rows of the whole image.
__global__ __launch_bounds__(256) void k_rgb_ycrcb420(const uint8_t *__restrict__ rgb, int in_row0, int in_rows, int H, int W,
                                                      int out_row0, int out_rows, uint8_t *__restrict__ Y,
                                                      uint8_t *__restrict__ Cr, uint8_t *__restrict__ Cb, int dh_out,
                                                      int dw) {
  __shared__ uint8_t s_c[2][RH][RW];
  __shared__ int s_h[2][RH][TX];
  const int ox0 = blockIdx.x * TX, oyl0 = blockIdx.y * TY;  // chroma tile origin (shard-relative row)
  const int oy0 = out_row0 / 2 + oyl0;                       // global chroma row
  const int gxs = 2 * ox0 - 4, gys = 2 * oy0 - 2;
  // Y pixels this tile writes: its 2x chroma footprint; the last tile row / column
  // of the shard also owns the odd leftover row / column of the image
  const int cx0 = 2 * ox0, cx1 = (ox0 + TX >= dw) ? W : 2 * (ox0 + TX);
  const int cy0 = 2 * oy0;
  const int cy1 = (oyl0 + TY >= dh_out) ? out_row0 + out_rows : 2 * (oy0 + TY);
  const int in_row1 = in_row0 + in_rows;
  const bool interior = gxs >= 0 && gys >= in_row0 && gxs + RW <= W && gys + RH <= in_row1 && (W % 4) == 0;

  if (interior) {
    // 4 pixels (3 dwords) per lane per step: 18 quads x 36 rows
    constexpr int QW = RW / 4;
    for (int i = threadIdx.x; i < RH * QW; i += 256) {
      const int ry = i / QW, qx = i - ry * QW;
      const int gy = gys + ry, gx = gxs + 4 * qx;
      const uint32_t *p = reinterpret_cast<const uint32_t *>(rgb + ((int64_t)(gy - in_row0) * W + gx) * 3);
      const uint32_t w0 = p[0], w1 = p[1], w2 = p[2];
      const int px[12] = {(int)(w0 & 255), (int)((w0 >> 8) & 255), (int)((w0 >> 16) & 255), (int)(w0 >> 24),
                          (int)(w1 & 255), (int)((w1 >> 8) & 255), (int)((w1 >> 16) & 255), (int)(w1 >> 24),
                          (int)(w2 & 255), (int)((w2 >> 8) & 255), (int)((w2 >> 16) & 255), (int)(w2 >> 24)};
      uint32_t yq = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const YCC c = rgb2ycc(px[3 * k], px[3 * k + 1], px[3 * k + 2]);
        yq |= c.y << (8 * k);
        s_c[0][ry][4 * qx + k] = (uint8_t)c.cr;
        s_c[1][ry][4 * qx + k] = (uint8_t)c.cb;
      }
      if (gy >= cy0 && gy < cy1 && gx >= cx0 && gx + 4 <= cx1)
        *reinterpret_cast<uint32_t *>(Y + (int64_t)(gy - out_row0) * W + gx) = yq;
    }
  } else {
    for (int i = threadIdx.x; i < RH * RW; i += 256) {
      const int ry = i / RW, rx = i - ry * RW;
      const int gy = gys + ry, gx = gxs + rx;
      int sy = refl101(gy, H);
      // rows outside the provided span only feed chroma rows past the shard (discarded)
      sy = sy < in_row0 ? in_row0 : (sy >= in_row1 ? in_row1 - 1 : sy);
      const int sx = refl101(gx, W);
      const uint8_t *p = rgb + ((int64_t)(sy - in_row0) * W + sx) * 3;
      const YCC c = rgb2ycc(p[0], p[1], p[2]);
      s_c[0][ry][rx] = (uint8_t)c.cr;
      s_c[1][ry][rx] = (uint8_t)c.cb;
      if (gy >= cy0 && gy < cy1 && gx >= cx0 && gx < cx1) Y[(int64_t)(gy - out_row0) * W + gx] = (uint8_t)c.y;
    }
  }
  __syncthreads();
  // horizontal [1 4 6 4 1] at even columns: center column 2*lox + 4 of the region
  for (int i = threadIdx.x; i < 2 * RH * TX; i += 256) {
    const int pl = i / (RH * TX), rem = i - pl * RH * TX;
    const int ry = rem / TX, lx = rem - ry * TX;
    const uint8_t *row = &s_c[pl][ry][2 * lx + 2];
    s_h[pl][ry][lx] = row[0] + 4 * (row[1] + row[3]) + 6 * row[2] + row[4];
  }
  __syncthreads();
  // vertical: center row 2*loy + 2 of the region
  for (int i = threadIdx.x; i < 2 * TY * TX; i += 256) {
    const int pl = i / (TY * TX), rem = i - pl * TY * TX;
    const int ly = rem / TX, lx = rem - ly * TX;
    const int oyl = oyl0 + ly, ox = ox0 + lx;
    if (oyl < dh_out && ox < dw) {
      const int v = s_h[pl][2 * ly][lx] + 4 * (s_h[pl][2 * ly + 1][lx] + s_h[pl][2 * ly + 3][lx]) +
                    6 * s_h[pl][2 * ly + 2][lx] + s_h[pl][2 * ly + 4][lx];
      (pl ? Cb : Cr)[(int64_t)oyl * dw + ox] = (uint8_t)sat8((v + 128) >> 8);
    }
  }
}

// ---------------------------------------------------------------------------
// Fast form of the same fused op for W % 4 == 0: no LDS, no barriers.
// A wave owns a strip of 64 RGB quads (4 pixels = 12 B per lane) and walks down
// kSegC chroma rows:
//  - each input row is loaded as one dwordx3 per lane (768 contiguous bytes per
//    wave);
//  - it is converted to Y (stored as one dword per lane: 256 B per wave, whole
//    cache lines when W % 256 == 0), Cr, Cb;
//  - the horizontal [1 4 6 4 1] at the two even columns of each quad takes its
//    neighbour pixels through DPP wave shifts (wave_shr / wave_shl);
//  - the strip's own halo pixels (x0-2, x0-1 and x0+256) for every row of the
//    segment are converted once per segment, one row per lane, and enter the
//    shifts at lanes 0 / 63 (v_readlane);
//  - the vertical pass keeps a 5-row register window and writes each chroma row
//    (2 B per lane per plane) as soon as its last input row is in.
// All rows of a segment are loaded up front (2*kSegC + 3 rows).  Reflect-101 at
// the left / right image border only ever needs pixels of the border quad
// itself (x = -2, -1 -> 2, 1; x = W -> W - 2).
constexpr int kStripQ = 64;

// [1 4 6 4 1] over five packed taps (k4 = 4 | 4 << 16, k6 = 6 | 6 << 16, registers:
// a literal 4 is strength-reduced to a shift and an add)
__device__ __forceinline__ uint32_t pk_taps5(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e, uint32_t k4,
                                             uint32_t k6) {
  return pk_mad_u16(c, k6, pk_mad_u16(pk_add_u16(b, d), k4, pk_add_u16(a, e)));
}
__device__ __forceinline__ uint32_t vreg(uint32_t k) {  // a constant held in a VGPR
  asm volatile("" : "+v"(k));
  return k;
}

// cvtColor RGB2YCrCb of the 4 pixels in 12 RGB bytes w[0..2] on the dot-product
// unit -- the fused encoder's ycc8 (encode.hip) for 4 pixels, equal to rgb2ycc on
// all 2^24 inputs (tools/check/colour_dot4.py): y in byte 1 of Yh[k], c[k] = Cr |
// Cb << 16.
constexpr uint32_t kYLo4 = 140u | 68u << 8 | 48u << 16, kYHi4 = 76u | 150u << 8 | 29u << 16;
constexpr int kCr4x = 4 * kYCRI, kCb4x = 4 * kYCBI, kCC4x = 4 * ((128 << 14) + (1 << 13));
struct YccK4 {
  uint32_t lo0, lo1, hi0, hi1, acc, cc4;
};
__device__ __forceinline__ void ycc4(uint32_t w0, uint32_t w1, uint32_t w2, const YccK4 &K, uint32_t (&Yh)[4],
                                     uint32_t (&c)[4]) {
  const uint32_t x[4] = {w0, __builtin_amdgcn_alignbyte(w1, w0, 3), __builtin_amdgcn_alignbyte(w2, w1, 2), w2};
  uint32_t L[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) L[k] = __builtin_amdgcn_udot4(x[k], k == 3 ? K.lo1 : K.lo0, K.acc, false);
#pragma unroll
  for (int k = 0; k < 4; ++k) Yh[k] = __builtin_amdgcn_udot4(x[k], k == 3 ? K.hi1 : K.hi0, L[k] >> 8, false);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int sh = k == 3 ? 8 : 0;
    const int y = (int)((Yh[k] >> 8) & 255u);
    const int r = (int)((x[k] >> sh) & 255u), b = (int)((x[k] >> (sh + 16)) & 255u);
    int vr = (r - y) * kCr4x + (int)K.cc4, vb = (b - y) * kCb4x + (int)K.cc4;
    vr = vr < 0 ? 0 : (vr > 0xFFFFFF ? 0xFFFFFF : vr);
    vb = vb < 0 ? 0 : (vb > 0xFFFFFF ? 0xFFFFFF : vb);
    c[k] = __builtin_amdgcn_perm((uint32_t)vb, (uint32_t)vr, 0x07060302u);
  }
}

template <typename T>
__device__ __forceinline__ void st_plane(T *p, T v, bool nt) {
  if (nt)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

template <int kSegC, bool NT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kSegC == 8 ? 4 : 3))) void k_rgb_ycrcb420_walk(const uint8_t *__restrict__ rgb, int in_row0, int in_rows,
                                                           int H, int W, int out_row0, int out_rows,
                                                           uint8_t *__restrict__ Y, uint8_t *__restrict__ Cr,
                                                           uint8_t *__restrict__ Cb, int dh_out, int nstrips,
                                                           int nwaves) {
  constexpr int kSegR = 2 * kSegC + 3;
  static_assert(kSegR <= 64, "one halo row per lane");
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= nwaves) return;
  const int seg = wid / nstrips, strip = wid - seg * nstrips;
  const int nq = W >> 2, dw = W >> 1;
  const int q0 = strip * kStripQ, q = q0 + lane;
  const bool owner = q < nq;
  const int qc = owner ? q : nq - 1;
  const int oyl0 = seg * kSegC;                                  // shard-relative chroma row
  const int ncr = dh_out - oyl0 < kSegC ? dh_out - oyl0 : kSegC;  // chroma rows of this segment
  const int nr = 2 * ncr + 3;                                    // input rows of this segment
  const int oy0 = out_row0 / 2 + oyl0;
  const int gy0 = 2 * oy0 - 2;
  const int in_row1 = in_row0 + in_rows;
  // Y rows this wave writes: the 2x footprint of its chroma rows; the last segment
  // of the shard also owns the odd leftover row of the image
  const int yw0 = 2 * oy0;
  const int yw1 = (oyl0 + kSegC >= dh_out) ? out_row0 + out_rows : 2 * (oy0 + ncr);
  auto src_row = [&](int r) {
    int sy = refl101(gy0 + r, H);
    sy = sy < in_row0 ? in_row0 : (sy >= in_row1 ? in_row1 - 1 : sy);
    return rgb + (int64_t)(sy - in_row0) * W * 3;
  };

  uint32_t raw[kSegR][3];
#pragma unroll
  for (int r = 0; r < kSegR; ++r) {
    if (r < nr) {
      const uint32_t *p = reinterpret_cast<const uint32_t *>(src_row(r) + 12 * qc);
      raw[r][0] = p[0];
      raw[r][1] = p[1];
      raw[r][2] = p[2];
    }
  }
  // halo of row `lane`, packed Cr | Cb << 16: x0-2, x0-1 (left) and x0+256 (right)
  uint32_t hal_l2 = 0, hal_l1 = 0, hal_r = 0;
  if (lane < nr) {
    const uint8_t *row = src_row(lane);
    const int x0 = 4 * q0;
    if (x0 >= 2) {
      const uint8_t *p = row + 3 * (x0 - 2);
      const YCC a = rgb2ycc(p[0], p[1], p[2]), b = rgb2ycc(p[3], p[4], p[5]);
      hal_l2 = a.cr | a.cb << 16;
      hal_l1 = b.cr | b.cb << 16;
    }
    if (x0 + 256 < W) {
      const uint8_t *p = row + 3 * (x0 + 256);
      const YCC c = rgb2ycc(p[0], p[1], p[2]);
      hal_r = c.cr | c.cb << 16;
    }
  }
  const YccK4 K{sreg(kYLo4), sreg(kYLo4 << 8), sreg(kYHi4), sreg(kYHi4 << 8), vreg(32768u), vreg((uint32_t)kCC4x)};
  const uint32_t k4 = sreg(0x00040004u), k6 = sreg(0x00060006u), k128 = 0x00800080u;
  // Interior waves (a full segment clear of the image / shard top and bottom, a
  // full strip that is neither the first nor the last) run a variant with no
  // per-lane conditions: every row's Y store and every chroma store is decided at
  // compile time, and the strip-edge halo comes in by v_cndmask.
  const bool interior = ncr == kSegC && oyl0 + kSegC < dh_out && gy0 >= (in_row0 > 0 ? in_row0 : 0) &&
                        gy0 + nr <= (in_row1 < H ? in_row1 : H) && gy0 + nr <= out_row0 + out_rows &&
                        gy0 >= out_row0 && strip > 0 && q0 + 64 < nq;
  auto body = [&](auto edge_tag) {
    constexpr bool EDGE = decltype(edge_tag)::value;
    // horizontally filtered rows, packed Cr | Cb << 16: chroma columns 2q (h0) and
    // 2q+1 (h2); one v_pk op filters both planes (sums <= 16 * 255, and the
    // vertical pass's <= 65280 + 128 fits 16 bits too)
    uint32_t h0[kSegR], h2[kSegR];
#pragma unroll
    for (int r = 0; r < kSegR; ++r) {
      if (EDGE && r >= nr) continue;
      uint32_t Yh[4], c[4];
      ycc4(raw[r][0], raw[r][1], raw[r][2], K, Yh, c);
      const uint32_t yq = __builtin_amdgcn_perm(__builtin_amdgcn_perm(Yh[3], Yh[2], 0x0C0C0501u),
                                                __builtin_amdgcn_perm(Yh[1], Yh[0], 0x0C0C0501u), 0x05040100u);
      const int gy = gy0 + r;
      if (EDGE) {
        if (owner && gy >= yw0 && gy < yw1)
          st_plane(reinterpret_cast<uint32_t *>(Y + (int64_t)(gy - out_row0) * W + 4 * q), yq, NT);
      } else if (r >= 2 && r < 2 + 2 * kSegC) {
        st_plane(reinterpret_cast<uint32_t *>(Y + (int64_t)(gy - out_row0) * W + 4 * q), yq, NT);
      }
      // neighbours: pixels x-2, x-1 from the left quad, x+4 from the right quad
      uint32_t l2 = shr1(c[2]), l1 = shr1(c[3]), rt = shl1(c[0]);
      l2 = lane == 0 ? (uint32_t)__builtin_amdgcn_readlane((int)hal_l2, r) : l2;
      l1 = lane == 0 ? (uint32_t)__builtin_amdgcn_readlane((int)hal_l1, r) : l1;
      rt = lane == 63 ? (uint32_t)__builtin_amdgcn_readlane((int)hal_r, r) : rt;
      if (EDGE) {
        if (q == 0) {  // reflect-101: x-2 -> x+2, x-1 -> x+1
          l2 = c[2];
          l1 = c[1];
        }
        if (q == nq - 1) rt = c[2];  // x+4 = W -> W-2
      }
      h0[r] = pk_taps5(l2, l1, c[0], c[1], c[2], k4, k6);
      h2[r] = pk_taps5(c[0], c[1], c[2], c[3], rt, k4, k6);
      if (r >= 4 && r % 2 == 0 && (!EDGE || owner)) {  // chroma row k = r/2 - 2 is complete
        const int a = r - 4, k = r / 2 - 2;
        const uint32_t v0 = pk_add_u16(pk_taps5(h0[a], h0[a + 1], h0[a + 2], h0[a + 3], h0[a + 4], k4, k6), k128);
        const uint32_t v2 = pk_add_u16(pk_taps5(h2[a], h2[a + 1], h2[a + 2], h2[a + 3], h2[a + 4], k4, k6), k128);
        const int64_t o = (int64_t)(oyl0 + k) * dw + 2 * q;
        // (v + 128) >> 8 = the high byte of each half (<= 255: no saturation)
        st_plane(reinterpret_cast<uint16_t *>(Cr + o), (uint16_t)__builtin_amdgcn_perm(v2, v0, 0x0C0C0501u), NT);
        st_plane(reinterpret_cast<uint16_t *>(Cb + o), (uint16_t)__builtin_amdgcn_perm(v2, v0, 0x0C0C0703u), NT);
      }
    }
  };
  if (interior)
    body(std::false_type{});
  else
    body(std::true_type{});
}

__global__ void k_rgb_ycrcb(const uint8_t *__restrict__ rgb, int64_t npix, uint8_t *__restrict__ Y,
                            uint8_t *__restrict__ Cr, uint8_t *__restrict__ Cb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint8_t *p = rgb + 3 * i;
  const YCC c = rgb2ycc(p[0], p[1], p[2]);
  Y[i] = (uint8_t)c.y;
  Cr[i] = (uint8_t)c.cr;
  Cb[i] = (uint8_t)c.cb;
}

__global__ void k_pyr_down(const uint8_t *__restrict__ src, int H, int W, uint8_t *__restrict__ dst, int DH,
                           int DW) {
  const int ox = blockIdx.x * blockDim.x + threadIdx.x, oy = blockIdx.y;
  if (ox >= DW || oy >= DH) return;
  constexpr int K[5] = {1, 4, 6, 4, 1};
  int acc = 0;
#pragma unroll
  for (int a = 0; a < 5; ++a) {
    const int sy = refl101(2 * oy + a - 2, H);
    int row = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) row += K[b] * src[(int64_t)sy * W + refl101(2 * ox + b - 2, W)];
    acc += K[a] * row;
  }
  dst[(int64_t)oy * DW + ox] = (uint8_t)sat8((acc + 128) >> 8);
}

// pyrUp taps for output index o of a length-n source: even o -> [1 6 1] around o/2,
// odd o -> [4 4] on (o/2, o/2+1); left border reflect-101, right border replicate.
__device__ __forceinline__ void up_taps(int o, int n, int (&idx)[3], int (&w)[3]) {
  const int s = o >> 1;
  idx[0] = s > 0 ? s - 1 : (n > 1 ? 1 : 0);
  idx[1] = s;
  idx[2] = s + 1 < n ? s + 1 : n - 1;
  if (o & 1) {
    w[0] = 0; w[1] = 4; w[2] = 4;
  } else {
    w[0] = 1; w[1] = 6; w[2] = 1;
  }
}

// row0: the image row src's first row holds (a shard's buffer starts mid-image)
__device__ __forceinline__ int pyr_up_at(const uint8_t *__restrict__ src, int H, int W, int oy, int ox,
                                         int row0 = 0) {
  int iy[3], wy[3], ix[3], wx[3];
  up_taps(oy, H, iy, wy);
  up_taps(ox, W, ix, wx);
  int acc = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    int row = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) row += wx[b] * src[(int64_t)(iy[a] - row0) * W + ix[b]];
    acc += wy[a] * row;
  }
  return (int)sat8((acc + 32) >> 6);
}

__global__ void k_pyr_up(const uint8_t *__restrict__ src, int H, int W, uint8_t *__restrict__ dst, int DH,
                         int DW) {
  const int ox = blockIdx.x * blockDim.x + threadIdx.x, oy = blockIdx.y;
  if (ox >= DW || oy >= DH) return;
  dst[(int64_t)oy * DW + ox] = (uint8_t)pyr_up_at(src, H, W, oy, ox);
}

// pyrUp(cr), pyrUp(cb) to 2h x 2w, crop y, cvtColor(YCrCb2RGB); output rows from
// 2 sb on (Y and rgb point at row 2 sb), chroma buffers starting at image row c_row0
__global__ void k_ycrcb420_rgb(const uint8_t *__restrict__ Y, int64_t ystride, const uint8_t *__restrict__ Cr,
                               const uint8_t *__restrict__ Cb, int h, int w, int sb, int c_row0,
                               uint8_t *__restrict__ rgb) {
  const int ox = blockIdx.x * blockDim.x + threadIdx.x, oy = blockIdx.y;  // oy: relative to 2 sb
  if (ox >= 2 * w) return;
  const int y = Y[(int64_t)oy * ystride + ox];
  const int cr = pyr_up_at(Cr, h, w, 2 * sb + oy, ox, c_row0) - 128;
  const int cb = pyr_up_at(Cb, h, w, 2 * sb + oy, ox, c_row0) - 128;
  uint8_t *o = rgb + ((int64_t)oy * 2 * w + ox) * 3;
  o[0] = (uint8_t)sat8(y + descale14(cr * kCR2R));
  o[1] = (uint8_t)sat8(y + descale14(cb * kCB2G + cr * kCR2G));
  o[2] = (uint8_t)sat8(y + descale14(cb * kCB2B));
}

// Fast form of k_ycrcb420_rgb for even w (4-byte aligned Y rows and RGB): a wave
// owns a strip of 64 output quads (4 pixels = 2 chroma columns per lane, 12 B of
// RGB: one dwordx3 store, 768 contiguous bytes per wave and row) and walks down
// kUpSeg chroma rows (2 * kUpSeg output rows).  Each chroma row is loaded once (2 B
// per lane and plane) and filtered horizontally ([1 6 1] at even, [4 4] at odd
// output columns); its neighbour columns 2q-1 / 2q+2 come from the adjacent lanes
// by DPP wave shifts (the strip-edge lanes load them).  The vertical taps run over
// a 3-row register window.  Edges as pyr_up_at: reflect-101 left / top, replicate
// right / bottom.
//
// Arithmetic (VALU-bound before: 37 ops and 2 quarter-rate multiplies per pixel):
// Cr and Cb travel as one packed pair (cr | cb << 16) through both filters
// (v_pk_mad_u16 / v_pk_add_u16, mod 2^16); every horizontal value carries a bias
// of -1020, so the vertical sum (weights 8 x 8) is v + 32 - 8192, in [-8160,
// 8160], and one v_pk_ashrrev_i16 by 6 gives both (cr - 128, cb - 128) exactly as
// sat8((v + 32) >> 6) - 128 (v <= 64 * 255, no saturation).  Each colour channel
// is then one v_dot2_i32_i16 of that pair with (kCR2x, kCB2x) accumulated onto
// y << 14 | 8192: y + descale14(...) == (y * 2^14 + 8192 + ...) >> 14 since
// y * 2^14 is a multiple of 2^14.  ~18 VALU per pixel.
constexpr int kUpSeg = 8;

// Row-range form (a tile shard's decode, sharding.ShardDecoder): chroma rows
// [sb, se) of an h-row image are produced, i.e. output rows [2 sb, 2 se); Y and rgb
// point at output row 2 sb; Cr / Cb hold chroma rows from c_row0 on (the shard's
// rows plus one halo row from each neighbour: rows sb - 1 and se are read when they
// exist).  The whole image is sb = 0, se = h, c_row0 = 0.
__global__ __launch_bounds__(256) void k_ycrcb420_rgb_walk(const uint8_t *__restrict__ Y, int64_t ystride,
                                                           const uint8_t *__restrict__ Cr,
                                                           const uint8_t *__restrict__ Cb, int h, int w,
                                                           int sb, int se, int c_row0,
                                                           uint8_t *__restrict__ rgb, int nstrips, int nwaves) {
  const int lane = threadIdx.x & 63;
  // wave-uniform (readfirstlane): row offsets and the loop count stay scalar
  const int wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (wid >= nwaves) return;
  const int seg = wid / nstrips, strip = wid - seg * nstrips;
  const int nq = w >> 1;
  const int q = strip * 64 + lane;
  const bool owner = q < nq;
  const int qc = owner ? q : nq - 1;
  const int s0 = sb + seg * kUpSeg;
  const int ns = se - s0 < kUpSeg ? se - s0 : kUpSeg;
  constexpr uint32_t K4 = 0x00040004u, K6 = 0x00060006u;
  constexpr uint32_t KB = 0xFC04FC04u;  // -1020 per half
  // (kCR2x | kCB2x << 16) in SGPRs: the three-operand v_dot2_i32_i16 then needs no
  // accumulator copies (its two-operand form with a literal does)
  const uint32_t kr = sreg((uint32_t)(uint16_t)kCR2R), kg = sreg((uint32_t)(uint16_t)kCR2G | (uint32_t)kCB2G << 16),
                 kb = sreg((uint32_t)kCB2B << 16);
  // row bases wave-uniform (scalar), lane offsets 32-bit.  Every lane also loads one
  // more chroma pair: lane 0 the pair left of its own (column 2q-1), lane 63 the pair
  // right of it (column 2q+2), the others a clamped dummy -- no divergent branch,
  // so the loads of row s+2 and of the next two Y rows are issued a whole
  // iteration before their use (software pipelining; each wave otherwise waits
  // out every load)
  const uint32_t qo = 2u * (uint32_t)qc;
  const uint32_t qe = lane == 0 ? (qo >= 2 ? qo - 2 : 0) : (qo + 2 <= (uint32_t)w - 2 ? qo + 2 : (uint32_t)w - 2);
  const uint32_t esel = lane == 0 ? 0x0C050C01u : 0x0C040C00u;
  struct Raw {
    uint32_t cr, cb, cre, cbe;
  };
  auto fetch = [&](int r) {
    const int64_t ro = (int64_t)(r - c_row0) * w;
    const uint8_t *crr = Cr + ro, *cbr = Cb + ro;
    Raw x;
    x.cr = *reinterpret_cast<const uint16_t *>(crr + qo);
    x.cb = *reinterpret_cast<const uint16_t *>(cbr + qo);
    x.cre = *reinterpret_cast<const uint16_t *>(crr + qe);
    x.cbe = *reinterpret_cast<const uint16_t *>(cbr + qe);
    return x;
  };
  // horizontally filtered chroma row, packed (cr | cb << 16) + bias, for output
  // columns 4q .. 4q+3 (x8 scale)
  auto filter = [&](const Raw &x, uint32_t (&hv)[4]) {
    const uint32_t p0 = __builtin_amdgcn_perm(x.cb, x.cr, 0x0C040C00u);  // column 2q:   cr | cb << 16
    const uint32_t p1 = __builtin_amdgcn_perm(x.cb, x.cr, 0x0C050C01u);  // column 2q+1
    const uint32_t e = __builtin_amdgcn_perm(x.cbe, x.cre, esel);        // 2q-1 (lane 0) / 2q+2 (lane 63)
    uint32_t l = shr1(p1), rr = shl1(p0);                                // columns 2q-1, 2q+2
    l = lane == 0 ? e : l;
    rr = lane == 63 ? e : rr;
    l = qc == 0 ? p1 : l;        // reflect-101: column -1 -> 1
    rr = qc == nq - 1 ? p1 : rr;  // replicate: column w -> w - 1
    hv[0] = pk_mad_u16(p0, K6, pk_add_u16(l, pk_add_u16(p1, KB)));
    hv[1] = pk_mad_u16(pk_add_u16(p0, p1), K4, KB);
    hv[2] = pk_mad_u16(p1, K6, pk_add_u16(rr, pk_add_u16(p0, KB)));
    hv[3] = pk_mad_u16(pk_add_u16(p1, rr), K4, KB);
  };
  auto yrow = [&](int oy) {  // output row oy (relative to 2 sb): 4 Y bytes
    return *reinterpret_cast<const uint32_t *>(Y + (int64_t)oy * ystride + 2 * qo);
  };
  uint32_t pv[4], cv[4], nv[4];
  filter(fetch(s0 > 0 ? s0 - 1 : (h > 1 ? 1 : 0)), pv);
  filter(fetch(s0), cv);
  Raw rn = fetch(s0 + 1 < h ? s0 + 1 : h - 1);
  uint32_t yq[2] = {yrow(2 * (s0 - sb)), yrow(2 * (s0 - sb) + 1)};
  for (int k = 0; k < ns; ++k) {
    const int s = s0 + k;
    filter(rn, nv);
    // prefetch for iteration k + 1 (rows inside the shard's halo: s + 2 <= se)
    uint32_t yn[2] = {yq[0], yq[1]};
    if (k + 1 < ns) {
      rn = fetch(s + 2 < h ? s + 2 : h - 1);
      yn[0] = yrow(2 * (s + 1 - sb));
      yn[1] = yrow(2 * (s + 1 - sb) + 1);
    }
#pragma unroll
    for (int odd = 0; odd < 2; ++odd) {
      const int oy = 2 * (s - sb) + odd;  // output row, relative to 2 sb
      int R[4], G[4], B[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t v = odd ? pk_mad_u16(pk_add_u16(cv[j], nv[j]), K4, 0) : pk_mad_u16(cv[j], K6, pk_add_u16(pv[j], nv[j]));
        const uint32_t crcb = pk_sra6(v);  // (cr - 128, cb - 128), signed
        const int acc = (int)(((yq[odd] >> (8 * j)) & 255) << 14 | 8192);
        R[j] = ycc_dot(crcb, kr, acc);
        G[j] = ycc_dot(crcb, kg, acc);
        B[j] = ycc_dot(crcb, kb, acc);
      }
      if (owner) {
        uint32_t *o = reinterpret_cast<uint32_t *>(rgb + (int64_t)oy * 6 * w + 12u * (uint32_t)q);
        // sat8(x >> 14) of channel pairs, two bytes per v_ashr_pk_u8_i32; its upper
        // half is not relied on (the halves are joined by v_perm)
        auto join = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x05040100u); };
        const uint3 v = make_uint3(join(sat_pk2(R[0], G[0]), sat_pk2(B[0], R[1])),
                                   join(sat_pk2(G[1], B[1]), sat_pk2(R[2], G[2])),
                                   join(sat_pk2(B[2], R[3]), sat_pk2(G[3], B[3])));
        *reinterpret_cast<uint3 *>(o) = v;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pv[j] = cv[j];
      cv[j] = nv[j];
    }
    yq[0] = yn[0];
    yq[1] = yn[1];
  }
}

bool dims_ok(int64_t H, int64_t W) { return H > 0 && W > 0 && H < (1 << 20) && W < (1 << 20); }

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" int hic_rgb_to_ycrcb420_rows(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H,
                                        int64_t W, int64_t out_row0, int64_t out_rows, uint8_t *y, uint8_t *cr,
                                        uint8_t *cb, void *stream) {
  if (!rgb_rows || !y || !cr || !cb) return arg_error("null pointer");
  if (!dims_ok(H, W) || H < 2 || W < 2) return arg_error("image shape (needs >= 2x2)");
  if (reinterpret_cast<uintptr_t>(rgb_rows) % 4 || reinterpret_cast<uintptr_t>(y) % 4)
    return arg_error("rgb / y must be 4-byte aligned");
  if (out_row0 < 0 || out_rows < 1 || out_row0 % 2 || out_row0 + out_rows > H) return arg_error("output row range");
  if (out_rows % 2 && out_row0 + out_rows != H) return arg_error("odd output row count before the last row");
  const int64_t dh = H / 2, dw = W / 2;
  const int64_t c0 = out_row0 / 2, c1 = (out_row0 + out_rows) / 2 < dh ? (out_row0 + out_rows) / 2 : dh;
  // rows the kernel reads: chroma rows [c0, c1) need image rows [2*c0 - 2, 2*c1 + 2) (reflected);
  // the Y rows are inside that span
  const int64_t need0 = 2 * c0 - 2 < 0 ? 0 : 2 * c0 - 2;
  const int64_t need1 = (2 * c1 + 2 > H ? H : 2 * c1 + 2) > out_row0 + out_rows ? (2 * c1 + 2 > H ? H : 2 * c1 + 2)
                                                                                : out_row0 + out_rows;
  if (in_row0 > need0 || in_row0 + in_rows < need1) return arg_error("input rows do not cover the pyrDown halo");
  if (c1 <= c0) return arg_error("no chroma rows in the output range");
  if (W % 4 == 0 && reinterpret_cast<uintptr_t>(cr) % 2 == 0 && reinterpret_cast<uintptr_t>(cb) % 2 == 0 &&
      knob(HIC_KNOB_COLOR_TILED) == 0) {
    const int nstrips = (int)((W / 4 + kStripQ - 1) / kStripQ);
    const int segc = knob(HIC_KNOB_COLOR_SEG) == 16 ? 16 : 8;
    const int nseg = (int)((c1 - c0 + segc - 1) / segc);
    const int nwaves = nstrips * nseg;
    const dim3 grid((unsigned)((nwaves + 3) / 4));
    if (segc == 16)
      hipLaunchKernelGGL(k_rgb_ycrcb420_walk<16>, grid, dim3(256), 0, as_stream(stream), rgb_rows, (int)in_row0,
                         (int)in_rows, (int)H, (int)W, (int)out_row0, (int)out_rows, y, cr, cb, (int)(c1 - c0),
                         nstrips, nwaves);
    else if (knob(HIC_KNOB_COLOR_NT) == 1)  // A/B: nontemporal plane stores
      hipLaunchKernelGGL((k_rgb_ycrcb420_walk<8, true>), grid, dim3(256), 0, as_stream(stream), rgb_rows,
                         (int)in_row0, (int)in_rows, (int)H, (int)W, (int)out_row0, (int)out_rows, y, cr, cb,
                         (int)(c1 - c0), nstrips, nwaves);
    else
      hipLaunchKernelGGL(k_rgb_ycrcb420_walk<8>, grid, dim3(256), 0, as_stream(stream), rgb_rows, (int)in_row0,
                         (int)in_rows, (int)H, (int)W, (int)out_row0, (int)out_rows, y, cr, cb, (int)(c1 - c0),
                         nstrips, nwaves);
    return check_launch("k_rgb_ycrcb420_walk");
  }
  const dim3 grid((unsigned)((dw + TX - 1) / TX), (unsigned)((c1 - c0 + TY - 1) / TY));
  hipLaunchKernelGGL(k_rgb_ycrcb420, grid, dim3(256), 0, as_stream(stream), rgb_rows, (int)in_row0, (int)in_rows, (int)H, (int)W,
                     (int)out_row0, (int)out_rows, y, cr, cb, (int)(c1 - c0), (int)dw);
  return check_launch("k_rgb_ycrcb420");
}

extern "C" int hic_rgb_to_ycrcb420(const uint8_t *rgb, int64_t H, int64_t W, uint8_t *y, uint8_t *cr, uint8_t *cb,
                                   void *stream) {
  return hic_rgb_to_ycrcb420_rows(rgb, 0, H, H, W, 0, H, y, cr, cb, stream);
}

extern "C" int hic_rgb_to_ycrcb(const uint8_t *rgb, int64_t H, int64_t W, uint8_t *y, uint8_t *cr, uint8_t *cb,
                                void *stream) {
  if (!rgb || !y || !cr || !cb) return arg_error("null pointer");
  if (!dims_ok(H, W)) return arg_error("image shape");
  const int64_t n = H * W;
  hipLaunchKernelGGL(k_rgb_ycrcb, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), rgb, n, y,
                     cr, cb);
  return check_launch("k_rgb_ycrcb");
}

extern "C" int hic_pyr_down_u8(const uint8_t *src, int64_t H, int64_t W, uint8_t *dst, int64_t DH, int64_t DW,
                               void *stream) {
  if (!src || !dst) return arg_error("null pointer");
  if (!dims_ok(H, W) || DH <= 0 || DW <= 0) return arg_error("shape");
  // OpenCV: |2*dsize - ssize| <= 2 in each dimension
  if (2 * DW - W > 2 || W - 2 * DW > 2 || 2 * DH - H > 2 || H - 2 * DH > 2) return arg_error("pyrDown dstsize");
  hipLaunchKernelGGL(k_pyr_down, dim3((unsigned)((DW + 255) / 256), (unsigned)DH), dim3(256), 0,
                     as_stream(stream), src, (int)H, (int)W, dst, (int)DH, (int)DW);
  return check_launch("k_pyr_down");
}

extern "C" int hic_pyr_up_u8(const uint8_t *src, int64_t H, int64_t W, uint8_t *dst, int64_t DH, int64_t DW,
                             void *stream) {
  if (!src || !dst) return arg_error("null pointer");
  if (!dims_ok(H, W) || DH <= 0 || DW <= 0) return arg_error("shape");
  // OpenCV: |dsize - 2*ssize| <= dsize % 2
  if (DW - 2 * W > DW % 2 || 2 * W - DW > DW % 2 || DH - 2 * H > DH % 2 || 2 * H - DH > DH % 2)
    return arg_error("pyrUp dstsize");
  hipLaunchKernelGGL(k_pyr_up, dim3((unsigned)((DW + 255) / 256), (unsigned)DH), dim3(256), 0, as_stream(stream),
                     src, (int)H, (int)W, dst, (int)DH, (int)DW);
  return check_launch("k_pyr_up");
}

extern "C" int hic_ycrcb420_to_rgb_rows(const uint8_t *y, int64_t y_stride, const uint8_t *cr, const uint8_t *cb,
                                        int64_t c_row0, int64_t c_rows, int64_t h, int64_t w, int64_t s0, int64_t s1,
                                        uint8_t *rgb, void *stream) {
  if (!y || !cr || !cb || !rgb) return arg_error("null pointer");
  if (!dims_ok(2 * h, 2 * w) || y_stride < 2 * w) return arg_error("shape");
  if (s0 < 0 || s1 > h || s1 <= s0) return arg_error("chroma row range");
  // pyrUp reads chroma rows s0 - 1 .. s1 (clamped to the image)
  const int64_t need0 = s0 > 0 ? s0 - 1 : 0, need1 = s1 < h ? s1 + 1 : h;
  if (c_row0 > need0 || c_row0 + c_rows < need1) return arg_error("chroma rows do not cover the pyrUp halo");
  if (w % 2 || y_stride % 4 || reinterpret_cast<uintptr_t>(y) % 4 || reinterpret_cast<uintptr_t>(rgb) % 4 ||
      reinterpret_cast<uintptr_t>(cr) % 2 || reinterpret_cast<uintptr_t>(cb) % 2 || knob(HIC_KNOB_COLOR_TILED)) {
    hipLaunchKernelGGL(k_ycrcb420_rgb, dim3((unsigned)((2 * w + 255) / 256), (unsigned)(2 * (s1 - s0))), dim3(256), 0,
                       as_stream(stream), y, y_stride, cr, cb, (int)h, (int)w, (int)s0, (int)c_row0, rgb);
    return check_launch("k_ycrcb420_rgb");
  }
  const int nstrips = (int)((w / 2 + 63) / 64), nseg = (int)((s1 - s0 + kUpSeg - 1) / kUpSeg);
  const int nwaves = nstrips * nseg;
  hipLaunchKernelGGL(k_ycrcb420_rgb_walk, dim3((unsigned)((nwaves + 3) / 4)), dim3(256), 0, as_stream(stream), y,
                     y_stride, cr, cb, (int)h, (int)w, (int)s0, (int)s1, (int)c_row0, rgb, nstrips, nwaves);
  return check_launch("k_ycrcb420_rgb_walk");
}

extern "C" int hic_ycrcb420_to_rgb(const uint8_t *y, int64_t y_stride, const uint8_t *cr, const uint8_t *cb,
                                   int64_t h, int64_t w, uint8_t *rgb, void *stream) {
  if (!y || !cr || !cb || !rgb) return arg_error("null pointer");
  if (!dims_ok(2 * h, 2 * w) || y_stride < 2 * w) return arg_error("shape");
  return hic_ycrcb420_to_rgb_rows(y, y_stride, cr, cb, 0, h, h, w, 0, h, rgb, stream);
}
