// dev: A/B of the colour walk kernel body (memory-only vs full) on 8K.
#include "../../hiccup_amd/csrc/color.hip"
#include "../../hiccup_amd/csrc/common.hip"
namespace hic { namespace {
template <int kSegC, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kSegC == 8 ? 4 : 3))) void k_walk_ab(const uint8_t *__restrict__ rgb, int in_row0, int in_rows,
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
  // halo of row `lane`: left = (cr, cr, cb, cb) of x0-2, x0-1; right = (cr, cb) of x0+256
  uint32_t hal_l = 0, hal_r = 0;
  if (lane < nr) {
    const uint8_t *row = src_row(lane);
    const int x0 = 4 * q0;
    if (x0 >= 2) {
      const uint8_t *p = row + 3 * (x0 - 2);
      const YCC a = rgb2ycc(p[0], p[1], p[2]), b = rgb2ycc(p[3], p[4], p[5]);
      hal_l = pack4(a.cr, b.cr, a.cb, b.cb);
    }
    if (x0 + 256 < W) {
      const uint8_t *p = row + 3 * (x0 + 256);
      const YCC c = rgb2ycc(p[0], p[1], p[2]);
      hal_r = c.cr | c.cb << 8;
    }
  }
  // Interior waves (a full segment clear of the image / shard top and bottom, a
  // full strip that is neither the first nor the last) run a variant with no
  // per-lane conditions: every row's Y store and every chroma store is decided at
  // compile time, and the strip-edge halo comes in by v_cndmask.
  const bool interior = ncr == kSegC && oyl0 + kSegC < dh_out && gy0 >= (in_row0 > 0 ? in_row0 : 0) &&
                        gy0 + nr <= (in_row1 < H ? in_row1 : H) && gy0 + nr <= out_row0 + out_rows &&
                        gy0 >= out_row0 && strip > 0 && q0 + 64 < nq;
  auto body = [&](auto edge_tag) {
    constexpr bool EDGE = decltype(edge_tag)::value;
    int hcr0[kSegR], hcr2[kSegR], hcb0[kSegR], hcb2[kSegR];
#pragma unroll
    for (int r = 0; r < kSegR; ++r) {
      if (EDGE && r >= nr) continue;
      const uint32_t w0 = raw[r][0], w1 = raw[r][1], w2 = raw[r][2];
      const int px[12] = {(int)(w0 & 255), (int)((w0 >> 8) & 255), (int)((w0 >> 16) & 255), (int)(w0 >> 24),
                          (int)(w1 & 255), (int)((w1 >> 8) & 255), (int)((w1 >> 16) & 255), (int)(w1 >> 24),
                          (int)(w2 & 255), (int)((w2 >> 8) & 255), (int)((w2 >> 16) & 255), (int)(w2 >> 24)};
      int cr[4], cb[4];
      uint32_t yq = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const YCC c = MODE == 0 ? YCC{(uint32_t)px[3 * k], (uint32_t)px[3 * k + 1], (uint32_t)px[3 * k + 2]}
                                : rgb2ycc(px[3 * k], px[3 * k + 1], px[3 * k + 2]);
        yq |= c.y << (8 * k);
        cr[k] = (int)c.cr;
        cb[k] = (int)c.cb;
      }
      const int gy = gy0 + r;
      if (EDGE) {
        if (owner && gy >= yw0 && gy < yw1)
          *reinterpret_cast<uint32_t *>(Y + (int64_t)(gy - out_row0) * W + 4 * q) = yq;
      } else if (r >= 2 && r < 2 + 2 * kSegC) {
        *reinterpret_cast<uint32_t *>(Y + (int64_t)(gy - out_row0) * W + 4 * q) = yq;
      }
      // neighbours: pixels x-2, x-1 from the left quad, x+4 from the right quad
      const uint32_t hl = (uint32_t)__builtin_amdgcn_readlane((int)hal_l, r);
      const uint32_t hr = (uint32_t)__builtin_amdgcn_readlane((int)hal_r, r);
      uint32_t lft = shr1(pack4(cr[2], cr[3], cb[2], cb[3]));
      uint32_t rgt = shl1((uint32_t)cr[0] | (uint32_t)cb[0] << 8);
      lft = lane == 0 ? hl : lft;
      rgt = lane == 63 ? hr : rgt;
      if (EDGE) {
        if (q == 0) lft = pack4(cr[2], cr[1], cb[2], cb[1]);
        if (q == nq - 1) rgt = (uint32_t)cr[2] | (uint32_t)cb[2] << 8;
      }
      hcr0[r] = (int)(lft & 255) + 4 * ((int)((lft >> 8) & 255) + cr[1]) + 6 * cr[0] + cr[2];
      hcb0[r] = (int)((lft >> 16) & 255) + 4 * ((int)(lft >> 24) + cb[1]) + 6 * cb[0] + cb[2];
      hcr2[r] = cr[0] + 4 * (cr[1] + cr[3]) + 6 * cr[2] + (int)(rgt & 255);
      hcb2[r] = cb[0] + 4 * (cb[1] + cb[3]) + 6 * cb[2] + (int)((rgt >> 8) & 255);
      if (r >= 4 && r % 2 == 0 && (!EDGE || owner)) {  // chroma row k = r/2 - 2 is complete
        const int a = r - 4, k = r / 2 - 2;
#define HIC_V(h) ((((h)[a] + 4 * ((h)[a + 1] + (h)[a + 3]) + 6 * (h)[a + 2] + (h)[a + 4]) + 128) >> 8)
        const int64_t o = (int64_t)(oyl0 + k) * dw + 2 * q;
        *reinterpret_cast<uint16_t *>(Cr + o) = (uint16_t)(sat8(HIC_V(hcr0)) | sat8(HIC_V(hcr2)) << 8);
        *reinterpret_cast<uint16_t *>(Cb + o) = (uint16_t)(sat8(HIC_V(hcb0)) | sat8(HIC_V(hcb2)) << 8);
#undef HIC_V
      }
    }
  };
  if (interior)
    body(std::false_type{});
  else
    body(std::true_type{});
}


} }
using namespace hic;
int main() {
  const int H = 4320, W = 7680, rot = 8;
  uint8_t *rgb[rot], *Y, *Cr, *Cb;
  for (int i = 0; i < rot; ++i) { hipMalloc(&rgb[i], (size_t)H * W * 3); hipMemset(rgb[i], 37 * i, (size_t)H * W * 3); }
  hipMalloc(&Y, (size_t)H * W); hipMalloc(&Cr, (size_t)H * W / 4); hipMalloc(&Cb, (size_t)H * W / 4);
  const int nstrips = (W / 4 + 63) / 64, nseg = (H / 2 + 7) / 8, nwaves = nstrips * nseg;
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  auto run = [&](const char *name, auto kern) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3((nwaves + 3) / 4), dim3(256), 0, 0, rgb[i % rot], 0, H, H, W, 0, H, Y, Cr, Cb, H / 2, nstrips, nwaves);
    hipEventRecord(s);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, dim3((nwaves + 3) / 4), dim3(256), 0, 0, rgb[i % rot], 0, H, H, W, 0, H, Y, Cr, Cb, H / 2, nstrips, nwaves);
    hipEventRecord(e); hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, s, e);
    printf("%-12s %.1f us\n", name, ms * 1e3 / 20);
  };
  run("memory-only", k_walk_ab<8, 0>);
  run("full", k_walk_ab<8, 1>);
  run("product", k_rgb_ycrcb420_walk<8>);
  return 0;
}
