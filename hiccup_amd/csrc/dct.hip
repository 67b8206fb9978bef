// dct.hip -- 8x8 block DCT-II + quantize (encode) and dequantize + DCT-III (decode)
// for MI355X (gfx950), bit-exact against hiccup's scipy/numpy path.
//
// Reference: transform.dct_channel / inv_dct_channel (transform.py:169-193),
// transform.dct2 / idct2 (transform.py:67-103) -> scipy.fftpack.dct / idct
// (pocketfft, scipy 1.15.3), quantization.jpeg_quantize / invert_jpeg_quantize
// (quantization.py:47-57,80-81).
//
// Design (DESIGN.md "forward kernel"):
//  * one 8x8 block per lane, 64 consecutive raster-order blocks per wave, so each
//    row load (8 B/lane) and each coefficient-row store (16 B/lane) of a wave is
//    one contiguous 512 B / 1 KiB segment of HBM; no LDS, no cross-lane traffic;
//  * float64 throughout, replicating pocketfft's length-8 operation order exactly
//    (built with -ffp-contract=off; the only FMAs are explicit ones whose product
//    is exact, e.g. y*2^-8);
//  * "half-scaled" DCT-II: pocketfft's x2 / x0.5 steps are exact power-of-two
//    scalings, so they are dropped and folded into the quantizer divisor
//    (DESIGN.md derives the bookkeeping: outputs 0 and 4 come out halved);
//  * the integer-exact prefix of each row transform (pixel sums/differences) runs
//    in int32, converting to float64 only where pocketfft first rounds;
//  * quantize = rint(b * (1/D)) with a near-tie guard: when the product lies
//    within 2^-30 of a half-integer (exact .5 ties occur at DC and at (4,4)), the
//    lane recomputes rint(b / D) with the IEEE-correct divide, which is what
//    numpy does.  The guard is > 10^3 x the reciprocal's error bound.
#include <stdlib.h>

#include "color_core.h"
#include "dct_core.h"
#include "rle_core.h"

namespace hic {
namespace {

template <int TABLE, int LAYOUT, bool FAST>
__global__ __launch_bounds__(256) void k_dct_quant(const uint8_t *__restrict__ plane, int H, int W,
                                                   int64_t stride, int nbx, int nblk,
                                                   void *__restrict__ out) {
  constexpr SlotOf<LAYOUT> kSlot{};
  const int blk = blockIdx.x * 256 + threadIdx.x;
  if (blk >= nblk) return;
  const int bi = blk / nbx, bj = blk - bi * nbx;
  const int y0 = bi * 8, x0 = bj * 8;

  // ---- row pass (rows of the 8x8 block) ----
  int col0[8];   // y'[r][0], exact integers
  double a[8][8];  // y'[r][1..7]  (a[r][0] unused)
  if (FAST) {
    const uint8_t *p = plane + (int64_t)y0 * stride + x0;
    uint2 w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + r * stride);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      int x[8];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        x[n] = (int)((w[r].x >> (8 * n)) & 0xFFu) - 128;
        x[n + 4] = (int)((w[r].y >> (8 * n)) & 0xFFu) - 128;
      }
      dct8h_int(x, col0[r], a[r]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      int x[8];
      const int yy = y0 + r;
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const int xx = x0 + n;
        // pad_matrix pads the (pixel - 128) plane with 0 (transform.py:17-30)
        x[n] = (yy < H && xx < W) ? (int)plane[(int64_t)yy * stride + xx] - 128 : 0;
      }
      dct8h_int(x, col0[r], a[r]);
    }
  }

  // ---- column pass + quantize, packed to int16 in the output order ----
  uint32_t pk[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) pk[k] = 0;
  {
    int b0;
    double b[8];
    dct8h_int(col0, b0, b);
    put16(pk, kSlot.s[0], quantize<TABLE>((double)b0, 0));
#pragma unroll
    for (int u = 1; u < 8; ++u) put16(pk, kSlot.s[u * 8], quantize<TABLE>(b[u], u * 8));
  }
#pragma unroll
  for (int v = 1; v < 8; ++v) {
    double xc[8], b[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) xc[r] = a[r][v];
    dct8h(xc, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) put16(pk, kSlot.s[u * 8 + v], quantize<TABLE>(b[u], u * 8 + v));
  }

  // ---- store ----
  if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
    if (!FAST && (y0 + 8 > H || x0 + 8 > W)) {
      // positions cropped by merge_blocks are 0 when jpeg_encode re-pads
#pragma unroll
      for (int z = 0; z < 64; ++z) {
        const int u = ZZ[z] / 8, v = ZZ[z] % 8;
        if (y0 + u >= H || x0 + v >= W) pk[z >> 1] &= (z & 1) ? 0x0000FFFFu : 0xFFFF0000u;
      }
    }
    uint4 *o = reinterpret_cast<uint4 *>(static_cast<int16_t *>(out) + (int64_t)blk * 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = make_uint4(pk[4 * k], pk[4 * k + 1], pk[4 * k + 2], pk[4 * k + 3]);
  } else if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
    int16_t *o = static_cast<int16_t *>(out);
    if (FAST) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        *reinterpret_cast<uint4 *>(o + (int64_t)(y0 + u) * W + x0) =
            make_uint4(pk[4 * u], pk[4 * u + 1], pk[4 * u + 2], pk[4 * u + 3]);
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int v = 0; v < 8; ++v)
          if (y0 + u < H && x0 + v < W)
            o[(int64_t)(y0 + u) * W + x0 + v] = (int16_t)(pk[(u * 8 + v) >> 1] >> (16 * (v & 1)));
    }
  } else {  // RASTER_I32
    int32_t *o = static_cast<int32_t *>(out);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int q[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) q[v] = (int)(int16_t)(pk[(u * 8 + v) >> 1] >> (16 * (v & 1)));
      if (FAST) {
        int4 *row = reinterpret_cast<int4 *>(o + (int64_t)(y0 + u) * W + x0);
        row[0] = make_int4(q[0], q[1], q[2], q[3]);
        row[1] = make_int4(q[4], q[5], q[6], q[7]);
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v)
          if (y0 + u < H && x0 + v < W) o[(int64_t)(y0 + u) * W + x0 + v] = q[v];
      }
    }
  }
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ double sreg_f64(double k) {  // opaque wave-uniform constant
  asm volatile("" : "+s"(k));
  return k;
}
__device__ __forceinline__ double vreg_f64(double k) {
  asm volatile("" : "+v"(k));
  return k;
}
__device__ __forceinline__ double fma_scale_add(double y, double k_s, double c_v) {  // fl(y * k + c), one rounding
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(y), "s"(k_s), "v"(c_v));
  return d;
}

// Dequantize (q * T, exact in int32), the 2-D DCT-III in pocketfft's float64
// operation order, /256 + 128, truncate, wrap, and store the 8x8 pixels of the
// block at (y0, x0) of the H x W plane (FAST: whole block inside, 8-byte rows).
template <int TABLE>
__device__ __forceinline__ void idct_block_px(const int (&q)[64], uint32_t (&px)[16]) {
  // dequantize (q * T, exact in int32) and row pass
  double a[8][8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    int c[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) c[v] = q[u * 8 + v] * QT[TABLE][u * 8 + v];
    idct8<int>(c, a[u]);
  }
  // column pass, /256 (exact) + 128, truncate toward zero, wrap mod 256.  The
  // constants live in registers (2^-8 an SGPR pair, 128 a VGPR pair) for a
  // three-address v_fma_f64: LLVM's v_fmac_f64 form overwrote its accumulator,
  // so it re-materialised 128.0 (two v_mov_b32) before each of the 64 fmas
  const double k2m8 = sreg_f64(0x1p-8), k128 = vreg_f64(128.0);
  // row r: bytes v = 0..3 in px[2r], 4..7 in px[2r+1].  A truncated value's low
  // byte is the wrapped pixel; bytes are packed by byte permutes, a pair of columns
  // per v_perm and two pairs per dword (3 instructions per 4 pixels)
  uint32_t even[8];  // row r's pixel of the even column of the pair being packed
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    double xc[8], yv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xc[u] = a[u][v];
    idct8<double>(xc, yv);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double p = fma_scale_add(yv[r], k2m8, k128);  // == fl(y/256 + 128): y*2^-8 exact
      const uint32_t b = (uint32_t)__double2int_rz(p);
      if (!(v & 1)) {
        even[r] = b;
      } else {
        const uint32_t pair = __builtin_amdgcn_perm(b, even[r], 0x0C0C0400u);  // even.b0 | b.b0 << 8
        uint32_t &d = px[2 * r + (v >> 2)];
        d = (v & 2) ? __builtin_amdgcn_perm(pair, d, 0x05040100u) : pair;
      }
    }
  }
}
template <int TABLE, bool FAST>
__device__ __forceinline__ void idct_block_store(const int (&q)[64], int H, int W, int y0, int x0,
                                                 uint8_t *__restrict__ out, int64_t ostride) {
  uint32_t px[16];
  idct_block_px<TABLE>(q, px);
  if (FAST) {
    uint8_t *o = out + (int64_t)y0 * ostride + x0;  // one 64-bit multiply; rows step by the uniform stride
#pragma unroll
    for (int r = 0; r < 8; ++r) *reinterpret_cast<uint2 *>(o + r * ostride) = make_uint2(px[2 * r], px[2 * r + 1]);
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int v = 0; v < 8; ++v)
        if (y0 + r < H && x0 + v < W)
          out[(int64_t)(y0 + r) * ostride + x0 + v] = (uint8_t)(px[2 * r + (v >> 2)] >> (8 * (v & 3)));
  }
}

template <int TABLE, int LAYOUT, bool FAST>
__global__ __launch_bounds__(256) void k_dequant_idct(const void *__restrict__ coef, int H, int W,
                                                      int nbx, int nblk, uint8_t *__restrict__ out,
                                                      int64_t ostride) {
  const int blk = blockIdx.x * 256 + threadIdx.x;
  if (blk >= nblk) return;
  const int bi = blk / nbx, bj = blk - bi * nbx;
  const int y0 = bi * 8, x0 = bj * 8;

  int q[64];  // raster [u][v]
  if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
    const uint4 *src = reinterpret_cast<const uint4 *>(static_cast<const int16_t *>(coef) + (int64_t)blk * 64);
    uint32_t w[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 t = src[k];
      w[4 * k] = t.x;
      w[4 * k + 1] = t.y;
      w[4 * k + 2] = t.z;
      w[4 * k + 3] = t.w;
    }
#pragma unroll
    for (int z = 0; z < 64; ++z) q[ZZ[z]] = (int)(int16_t)(w[z >> 1] >> (16 * (z & 1)));
    if (!FAST && (y0 + 8 > H || x0 + 8 > W)) {
#pragma unroll
      for (int i = 0; i < 64; ++i)
        if (y0 + i / 8 >= H || x0 + i % 8 >= W) q[i] = 0;
    }
  } else if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
    const int16_t *c = static_cast<const int16_t *>(coef);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (FAST) {
        const uint4 t = *reinterpret_cast<const uint4 *>(c + (int64_t)(y0 + u) * W + x0);
        const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int v = 0; v < 8; ++v) q[u * 8 + v] = (int)(int16_t)(w[v >> 1] >> (16 * (v & 1)));
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v)
          q[u * 8 + v] = (y0 + u < H && x0 + v < W) ? (int)c[(int64_t)(y0 + u) * W + x0 + v] : 0;
      }
    }
  } else {
    const int32_t *c = static_cast<const int32_t *>(coef);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (FAST) {
        const int4 *row = reinterpret_cast<const int4 *>(c + (int64_t)(y0 + u) * W + x0);
        const int4 t0 = row[0], t1 = row[1];
        q[u * 8 + 0] = t0.x; q[u * 8 + 1] = t0.y; q[u * 8 + 2] = t0.z; q[u * 8 + 3] = t0.w;
        q[u * 8 + 4] = t1.x; q[u * 8 + 5] = t1.y; q[u * 8 + 6] = t1.z; q[u * 8 + 7] = t1.w;
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v)
          q[u * 8 + v] = (y0 + u < H && x0 + v < W) ? c[(int64_t)(y0 + u) * W + x0 + v] : 0;
      }
    }
  }

  idct_block_store<TABLE, FAST>(q, H, W, y0, x0, out, ostride);
}

// Indexed decode fused with the inverse transform: one wave per 64-block tile
// assembles its blocks in LDS from the symbols the encoder's tile index points at
// (as k_rld_indexed16 in rle.hip), then every lane runs the dequantize + IDCT of
// its block straight from LDS and stores pixels: the zig-zag blocks never reach
// HBM (codec.jpeg_decode's RLE / DC half, codec.py:397-421, + inv_dct_channel,
// transform.py:169-179, for one plane).
constexpr int kRowI16 = 68;  // LDS block row: 64 slots + pad (136 B, conflict-free 8 B reads)
// waves per SIMD: 3 (138 VGPRs, no spills) measured 2-6 % faster than 4 (128 VGPRs,
// ~10 spilled) once the gather went branch-free (profiles/r05/decode_wpe/)
#ifndef HIC_DEC_WPE
#define HIC_DEC_WPE 3
#endif
// The RGB of one 8x8 luma block (pixels px as idct_block_px leaves them) at block
// (bi, bj) of an H x W image, H and W multiples of 8: pyrUp(Cr), pyrUp(Cb) of the
// H/2 x W/2 chroma planes at its 64 pixels, then cvtColor(YCrCb2RGB)
// (compression.jpeg_decompression, compression.py:48-56).  The arithmetic is
// color.hip k_ycrcb420_rgb_walk's (cr | cb << 16 pairs biased by -1020 through both
// pyrUp passes, one v_dot2_i32_i16 per channel), so the bytes equal that kernel's
// on the same planes.  The chroma columns 4bj-1 / 4bj+4 next to the block's four come
// from the neighbouring lanes' blocks (DPP) or, at the wave's ends, from one extra
// dword load per row; reflect-101 at the top / left border, replicate at the
// bottom / right, as pyr_up_at.  Every lane of the wave must take part (the DPP
// reads); `live` gates the stores.
__device__ __forceinline__ void colour_block(const uint32_t (&px)[16], int bi, int bj, int nbx, int nby, int lane,
                                             bool live, const uint8_t *__restrict__ cr, const uint8_t *__restrict__ cb,
                                             uint8_t *__restrict__ rgb, int64_t rgb_stride) {
  const int w = 4 * nbx, h = 4 * nby;
  // The packed pixels are opaque: otherwise the compiler forwards each truncated
  // pixel past its packing to the byte extracts below, and 64 live values instead
  // of 16 spill the IDCT.  bi, bj pass through the last of them, so no address
  // below is computed (and held) across the IDCT.
  uint32_t y[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    y[k] = px[k];
    asm volatile("" : "+v"(y[k]));
  }
  asm volatile("" : "+v"(bi), "+v"(bj) : "v"(y[15]));
  // chroma rows 4bi-1 .. 4bi+4: its own four columns, and the wave-end lanes' outer
  // neighbour column (lane 0: the dword left of its own, lane 63: the one right)
  const int ce = lane == 0 ? (bj > 0 ? 4 * bj - 4 : 4 * bj) : (bj < nbx - 1 ? 4 * bj + 4 : 4 * bj);
  uint32_t dcr[6], dcb[6], ecr[6], ecb[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    int s = 4 * bi - 1 + r;
    s = s < 0 ? 1 : (s >= h ? h - 1 : s);
    const int64_t ro = (int64_t)s * w;
    dcr[r] = *reinterpret_cast<const uint32_t *>(cr + ro + 4 * bj);
    dcb[r] = *reinterpret_cast<const uint32_t *>(cb + ro + 4 * bj);
    ecr[r] = *reinterpret_cast<const uint32_t *>(cr + ro + ce);
    ecb[r] = *reinterpret_cast<const uint32_t *>(cb + ro + ce);
  }
  // KB: -1020 per half; K4 opaque (a splat 4 is strength-reduced to a shift + add)
  const uint32_t K4 = sreg(0x00040004u), K6 = 0x00060006u, KB = 0xFC04FC04u;
  const uint32_t kr = sreg((uint32_t)(uint16_t)kCR2R), kg = sreg((uint32_t)(uint16_t)kCR2G | (uint32_t)kCB2G << 16),
                 kb = sreg((uint32_t)kCB2B << 16);
  auto join = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x05040100u); };
  // horizontal pass of chroma row r: output columns 8bj .. 8bj+7 (x8 scale, biased)
  auto horiz = [&](int r, uint32_t (&hv)[8]) {
    uint32_t q[6];  // chroma columns 4bj-1 .. 4bj+4, packed cr | cb << 16
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j + 1] = __builtin_amdgcn_perm(dcb[r], dcr[r], 0x0C040C00u + 0x00010001u * j);
    uint32_t l = shr1(q[4]), rr = shl1(q[1]);
    l = lane == 0 ? __builtin_amdgcn_perm(ecb[r], ecr[r], 0x0C070C03u) : l;
    rr = lane == 63 ? __builtin_amdgcn_perm(ecb[r], ecr[r], 0x0C040C00u) : rr;
    q[0] = bj == 0 ? q[2] : l;         // reflect-101: column -1 -> 1
    q[5] = bj == nbx - 1 ? q[4] : rr;  // replicate: column w -> w - 1
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      hv[2 * c] = pk_mad_u16(q[c + 1], K6, pk_add_u16(q[c], pk_add_u16(q[c + 2], KB)));
      hv[2 * c + 1] = pk_mad_u16(pk_add_u16(q[c + 1], q[c + 2]), K4, KB);
    }
  };
  // output row 8bi + r8 from its vertical taps' packed sums v[8]
  auto emit = [&](int r8, const uint32_t (&v)[8]) {
    uint32_t o[6];
    int pend = 0;  // channel bytes waiting for their pair partner
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const uint32_t crcb = pk_sra6(v[x]);  // (cr - 128, cb - 128)
      const int acc = (int)(((y[2 * r8 + (x >> 2)] >> (8 * (x & 3))) & 255u) << 14 | 8192u);
      const int c3[3] = {ycc_dot(crcb, kr, acc), ycc_dot(crcb, kg, acc), ycc_dot(crcb, kb, acc)};
      // bytes 3x .. 3x+2 of the row's 24: pairs (2m, 2m+1) -> one v_ashr_pk_u8_i32
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const int byte = 3 * x + ch;
        if (byte & 1) {
          const uint32_t pr = sat_pk2(pend, c3[ch]);  // bytes byte-1, byte
          if ((byte >> 1) & 1) o[byte >> 2] = join(o[byte >> 2], pr);
          else o[byte >> 2] = pr;
        } else {
          pend = c3[ch];
        }
      }
    }
    if (live) {
      uint2 *d = reinterpret_cast<uint2 *>(rgb + (int64_t)(8 * bi + r8) * rgb_stride + 24 * bj);
      d[0] = make_uint2(o[0], o[1]);
      d[1] = make_uint2(o[2], o[3]);
      d[2] = make_uint2(o[4], o[5]);
    }
  };
  // a three-row window down chroma rows 4bi-1 .. 4bi+4: rows k, k+1, k+2 of it give
  // output rows 8bi + 2k ([1 6 1]) and 8bi + 2k + 1 ([4 4])
  uint32_t ha[8], hb[8], hc[8];
  horiz(0, ha);
  horiz(1, hb);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    horiz(k + 2, hc);
    uint32_t v[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) v[x] = pk_mad_u16(hb[x], K6, pk_add_u16(ha[x], hc[x]));
    emit(2 * k, v);
#pragma unroll
    for (int x = 0; x < 8; ++x) v[x] = pk_mad_u16(pk_add_u16(hb[x], hc[x]), K4, 0);
    emit(2 * k + 1, v);
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      ha[x] = hb[x];
      hb[x] = hc[x];
    }
  }
}

// RGB (luma plane only, TABLE 0, FAST): the pixels go through colour_block into
// the RGB image instead of to a Y plane -- the Y plane never reaches HBM
// (jpeg_decompression's decode of the luma channel + pyrUp + cvtColor, with the
// chroma planes decoded before).
// A second plane of the same shape and table (Cb beside Cr): the launch covers both
// planes' tiles, so the two share one tail (hic_rle_decode_idct_u8_indexed_pair).
struct DecPlane {
  const uint8_t *sym_len;
  const int16_t *sym_val;
  const int64_t *d_nsym;
  const int32_t *dc_diff;
  const int64_t *index;
  uint8_t *out;
  int64_t *d_status;
};
// SLOTS: the symbols in the slot layout (slots.h), `index` the close's int32 record
// index, rsh = log2 records per 64-block tile.
template <int TABLE, bool FAST, bool RGB = false, bool SLOTS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HIC_DEC_WPE))) void k_rld_idct_indexed(const uint8_t *__restrict__ sym_len_a,
                                                          const int16_t *__restrict__ sym_val_a,
                                                          const int64_t *__restrict__ d_nsym_a,
                                                          const int32_t *__restrict__ dc_diff_a,
                                                          const int64_t *__restrict__ index_a, int H, int W, int nbx,
                                                          int64_t nblk, uint8_t *__restrict__ out_a, int64_t ostride,
                                                          int64_t *__restrict__ d_status_a,
                                                          const uint8_t *__restrict__ cr = nullptr,
                                                          const uint8_t *__restrict__ cb = nullptr,
                                                          DecPlane second = DecPlane{}, int rsh = 0) {
  static_assert(!RGB || (TABLE == 0 && FAST), "the RGB form decodes whole-block luma planes");
  __shared__ uint2 s_tile[4][64 * kRowI16 / 4];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ntiles = (nblk + 63) / 64;
  int64_t t = (int64_t)blockIdx.x * 4 + wv;
  const bool b = !RGB && t >= ntiles;  // wave-uniform: the second plane's tile t - ntiles
  if (b) {
    if (!second.sym_len || t >= 2 * ntiles) return;
    t -= ntiles;
  } else if (t >= ntiles) {
    return;
  }
  const uint8_t *__restrict__ sym_len = b ? second.sym_len : sym_len_a;
  const int16_t *__restrict__ sym_val = b ? second.sym_val : sym_val_a;
  const int64_t *__restrict__ d_nsym = b ? second.d_nsym : d_nsym_a;
  const int32_t *__restrict__ dc_diff = b ? second.dc_diff : dc_diff_a;
  const int64_t *__restrict__ index = b ? second.index : index_a;
  uint8_t *__restrict__ out = b ? second.out : out_a;
  int64_t *__restrict__ d_status = b ? second.d_status : d_status_a;
  uint2 *tile = s_tile[wv];
  int16_t *win = reinterpret_cast<int16_t *>(tile);
  const int64_t nsym_raw = *d_nsym, nsym = nsym_raw > 0 ? nsym_raw : 0;
  const int nvb = (int)(nblk - t * 64 < 64 ? nblk - t * 64 : 64);
  const int64_t blk = t * 64 + lane;
  // loads that depend on nothing else go out before the zero-fill: this lane's DC
  // difference and (slot layout) the tile's record index
  const int d = lane < nvb ? dc_diff[blk] : 0;
  // the gather (index, symbol loads, LDS scatter) at issue priority 1 over the
  // SIMD's waves in their IDCT / colour: 16K decode 0.713-0.766 vs 0.749-0.807 ms,
  // faster in 7 of 8 alternating rounds (profiles/r06/dec_prio/)
  __builtin_amdgcn_s_setprio(1);
  SlotTileIx six;
  if constexpr (SLOTS) six = slot_tile_ix(reinterpret_cast<const int32_t *>(index), t, rsh, nblk);
  for (int i = lane; i < 64 * kRowI16 / 4; i += 64) tile[i] = make_uint2(0, 0);
  __builtin_amdgcn_wave_barrier();
  const int64_t tb0 = t * 64 * 63;
  const int span = nvb * 63;
  // the symbols of the tile into its LDS rows (trash: the lane's row's first pad slot)
  int P, pdc;
  if constexpr (SLOTS) {
    P = slots_gather_tile<kRowI16>(sym_len, sym_val, six, t, rsh, span, win, lane * kRowI16 + 64, lane);
    pdc = six.r[0].z;
  } else {
    const int64_t o0 = index[3 * t] < nsym ? index[3 * t] : nsym;
    const int64_t o1 = t + 1 < ntiles ? (index[3 * (t + 1)] < nsym ? index[3 * (t + 1)] : nsym) : nsym;
    P = gather_tile<kRowI16, HIC_DEC_G, HIC_DEC_PF>(sym_len, sym_val, o0, o1, nsym, (int)(index[3 * t + 1] + 1 - tb0),
                                                    span, win, lane * kRowI16 + 64, lane);
    pdc = (int)index[3 * t + 2];
  }
  win[lane * kRowI16] = (int16_t)(pdc + wave_incl_sum_i32(d));
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_setprio(0);
  if (t == ntiles - 1 && lane == 0) {
    // (a slot-layout stream is whole by construction: its EOB zero-fills the rest)
    const int64_t total = tb0 + (int64_t)P, n_ac = nblk * 63;
    const bool eob = SLOTS || (nsym > 0 && sym_len[nsym - 1] == 0 && sym_val[nsym - 1] == 0);
    *d_status = nsym_raw < 1 ? -1 : ((eob && (SLOTS || total <= n_ac)) ? n_ac : total);
  }
  if (!RGB && lane >= nvb) return;
  int qv[64];  // raster [u][v]
  {
    const uint2 *row = tile + (lane < nvb ? lane : nvb - 1) * (kRowI16 / 4);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint2 x = row[k];
      qv[ZZ[4 * k]] = (int)(int16_t)(x.x & 0xFFFFu);
      qv[ZZ[4 * k + 1]] = (int)(int16_t)(x.x >> 16);
      qv[ZZ[4 * k + 2]] = (int)(int16_t)(x.y & 0xFFFFu);
      qv[ZZ[4 * k + 3]] = (int)(int16_t)(x.y >> 16);
    }
  }
  const int64_t blk_c = lane < nvb ? blk : t * 64 + nvb - 1;  // RGB: the dead lanes redo the last block
  const int bi = (int)(blk_c / nbx), bj = (int)(blk_c - (int64_t)bi * nbx);
  if (RGB) {
    uint32_t px[16];
    idct_block_px<TABLE>(qv, px);
    colour_block(px, bi, bj, nbx, H / 8, lane, lane < nvb, cr, cb, out, ostride);
  } else {
    idct_block_store<TABLE, FAST>(qv, H, W, bi * 8, bj * 8, out, ostride);
  }
}

// Production forward kernel for aligned planes: up to three planes per launch
// (Y, Cr, Cb of one image), one persistent grid over all their sets.  TABLE = -1:
// each plane's quantisation table is read at run time (its constants become scalar
// loads), so the three planes share one launch and one tail -- separate launches
// per table left a third of the waves idle in each tail.  TABLE = 0 / 1: a
// compile-time table (single-table callers).  One 8x8 block per lane, 64
// consecutive raster-order blocks ("a set" = one RLE tile) per wave iteration;
// persistent grid sized to the waves that fit at once.
// dct_block_aan (dct_core.h) writes the quantized coefficients straight to their
// slot in an LDS stage, which is copied out so that every store instruction writes
// one contiguous 1 KiB segment (zig-zag layout) or whole 16-byte row pieces
// (raster layouts).  TMF >= 0 (ZIGZAG_I16 only): the set's RLE tile record
// (rle_core.h) is written too -- the K1 pass of hic_rle_encode_i16 fused into the
// epilogue; TMF = 15 specialises max_len 15.
struct DctJob {
  const uint8_t *plane;
  int64_t stride;
  void *out;
  int64_t *tiles;
  int W, nbx, nblk, nsets, set0, table;
};
constexpr int kMaxPlaneJobs = 16;  // planes per launch (hic_dct_quant_rle_u8_batch)
struct DctJobs {
  DctJob j[kMaxPlaneJobs];
  int n, total_sets, M;
};

#ifndef HIC_DCT_WPE
#define HIC_DCT_WPE 3  // register budget: waves per SIMD (3: <= 168 VGPRs)
#endif
// (An LDS-DMA prefetch of the next set's pixels, round 6's dct_path 2, was bit-exact
// and within noise of these register loads: profiles/r06/glds_ab, commit "LDS-DMA
// prefetch form of the plane DCT"; removed.)
template <int TABLE, int LAYOUT, int TMF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HIC_DCT_WPE))) void k_dct_planes(DctJobs jobs,
                                                                                                       int path) {
  __shared__ uint2 s_stage[4 * 64 * kStageU2];
  // wv is wave-uniform: keep it (and the set / job indices derived from it) in
  // SGPRs, so the job fields are scalar loads, not vector loads on vmcnt
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  const int g0 = blockIdx.x * 4 + wv;
  uint2 *st2 = s_stage + wv * 64 * kStageU2;
  int16_t *st = reinterpret_cast<int16_t *>(st2 + lane * kStageU2);
  // 16 B of block b's stage row, at 8-byte granularity (ds_read_b64 pairs)
  auto st16 = [&](int b, int k) {
    const uint2 lo = st2[b * kStageU2 + 2 * k], hi = st2[b * kStageU2 + 2 * k + 1];
    return make_uint4(lo.x, lo.y, hi.x, hi.y);
  };
  const int M = jobs.M;

  // g is wave-uniform; readfirstlane keeps the job index in an SGPR (a VGPR index
  // into the by-value kernel argument copies it to scratch)
  auto job_of = [&](int g) {
    g = __builtin_amdgcn_readfirstlane(g);
    int k = 0;
    while (k + 1 < jobs.n && g >= jobs.j[k + 1].set0) ++k;
    return __builtin_amdgcn_readfirstlane(k);
  };
  auto load = [&](const DctJob &J, int set, uint2 (&w)[8]) {
    const int blk = set * 64 + lane;
    const int cblk = blk < J.nblk ? blk : J.nblk - 1;
    const int bi = cblk / J.nbx, bj = cblk - bi * J.nbx;
    const uint8_t *p = J.plane + (int64_t)bi * 8 * J.stride + bj * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = *reinterpret_cast<const uint2 *>(p + r * J.stride);
  };
  // stage -> output layout (+ the RLE tile record)
  auto store = [&](const DctJob &J, int set) {
    __builtin_amdgcn_wave_barrier();
    const int blk = set * 64 + lane;
    if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
      uint4 *o = reinterpret_cast<uint4 *>(static_cast<int16_t *>(J.out) + (int64_t)set * 64 * 64);
      auto sv = [&](int k) { return st16(8 * k + (lane >> 3), lane & 7); };
      if ((set + 1) * 64 <= J.nblk) {
        // nontemporal stores (the compiler's own nt encoding; an inline-asm sc1
        // store was faster but broke the sharded encode, see DESIGN)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint4 t = sv(k);
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 v = {t.x, t.y, t.z, t.w};
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(o + 64 * k + lane));
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (set * 64 + 8 * k + (lane >> 3) < J.nblk) o[64 * k + lane] = sv(k);
      }
      if (TMF >= 0) {
        uint32_t zw[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint4 t = st16(lane, k);
          zw[4 * k] = t.x; zw[4 * k + 1] = t.y; zw[4 * k + 2] = t.z; zw[4 * k + 3] = t.w;
        }
        tile_record16<TMF>(zw, blk < J.nblk, blk, M, J.tiles + (int64_t)set * 3);
      }
    } else if (blk < J.nblk) {
      const int bi = blk / J.nbx, bj = blk - bi * J.nbx;
      if (LAYOUT == HIC_LAYOUT_RASTER_I16) {
        int16_t *o = static_cast<int16_t *>(J.out) + (int64_t)bi * 8 * J.W + bj * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u) *reinterpret_cast<uint4 *>(o + (int64_t)u * J.W) = st16(lane, u);
      } else {
        int32_t *o = static_cast<int32_t *>(J.out) + (int64_t)bi * 8 * J.W + bj * 8;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint4 t = st16(lane, u);
          const uint32_t wd[4] = {t.x, t.y, t.z, t.w};
          int q[8];
#pragma unroll
          for (int v = 0; v < 8; ++v) q[v] = (int)(int16_t)(wd[v >> 1] >> (16 * (v & 1)));
          int4 *row = reinterpret_cast<int4 *>(o + (int64_t)u * J.W);
          row[0] = make_int4(q[0], q[1], q[2], q[3]);
          row[1] = make_int4(q[4], q[5], q[6], q[7]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  };

  // Main loop: the float64 AAN path.  A set with any coefficient inside the
  // quantiser's tie window is remembered (bit i of `redo` / `fix` = this wave's
  // i-th set; the launcher keeps every wave at <= 64 sets) and handled after the
  // loop -- a separate code region, so the paths do not share one register
  // allocation.  path 0 (A/B tests): exact replica only.
  uint64_t redo = 0, fix = 0;
  int i = 0;
  if (path != 0) {
    // the job's fields stay in SGPRs and are reloaded only when g enters the next
    // job (jobs are contiguous set ranges): no scalar loads on the per-set path
    int kj = g0 < jobs.total_sets ? job_of(g0) : 0;
    DctJob J = jobs.j[kj];
    int next0 = kj + 1 < jobs.n ? jobs.j[kj + 1].set0 : jobs.total_sets;
    // (a software-pipelined load of the next set's pixels into registers was measured
    // slower and removed: 160 vs 149 VGPRs, 8K luma 27.6-27.7 vs 25.6-26.2 us,
    // profiles/r03/s2/dct_pf/; the other waves of the SIMD hide the loads)
    for (int g = g0; g < jobs.total_sets; g += nwaves, ++i) {
      if (g >= next0) {
        kj = job_of(g);
        J = jobs.j[kj];
        next0 = kj + 1 < jobs.n ? jobs.j[kj + 1].set0 : jobs.total_sets;
      }
      const int set = g - J.set0;
      uint2 w[8];
      load(J, set, w);
      bool t26 = false;
      const bool f = dct_block_aan<TABLE, LAYOUT>(w, st, &t26, nullptr, J.table);
      if (__builtin_amdgcn_ballot_w64(f) != 0) redo |= 1ull << i;
      if (__builtin_amdgcn_ballot_w64(t26) != 0) fix |= 1ull << i;
      store(J, set);
    }
  } else {
    for (int g = g0; g < jobs.total_sets; g += nwaves, ++i) redo |= 1ull << i;
  }
  fix &= ~redo;
  // (2,2)-class exact ties: rewrite just those four coefficients of the set's
  // blocks in the output (and the set's RLE tile record)
  while (fix) {
    const int k = __builtin_ctzll(fix);
    fix &= fix - 1;
    const int g = g0 + k * nwaves;
    const DctJob &J = jobs.j[job_of(g)];
    const int set = g - J.set0;
    const int blk = set * 64 + lane;
    uint2 w[8];
    load(J, set, w);
    int q[4];
    dct_fix26<TABLE>(w, q, J.table);
    if (blk < J.nblk) {
      constexpr SlotOf<LAYOUT> kSlot{};
      constexpr int idx[4] = {18, 22, 50, 54};
      if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16) {
        int16_t *o = static_cast<int16_t *>(J.out) + (int64_t)blk * 64;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[kSlot.s[idx[j]]] = (int16_t)q[j];
      } else {
        const int bi = blk / J.nbx, bj = blk - bi * J.nbx;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t at = (int64_t)(bi * 8 + idx[j] / 8) * J.W + bj * 8 + idx[j] % 8;
          if (LAYOUT == HIC_LAYOUT_RASTER_I16)
            static_cast<int16_t *>(J.out)[at] = (int16_t)q[j];
          else
            static_cast<int32_t *>(J.out)[at] = q[j];
        }
      }
    }
    if (LAYOUT == HIC_LAYOUT_ZIGZAG_I16 && TMF >= 0) {
      uint32_t zw[32];
      if (blk < J.nblk) {
        const uint4 *b4 = reinterpret_cast<const uint4 *>(static_cast<const int16_t *>(J.out) + (int64_t)blk * 64);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint4 t = b4[j];
          zw[4 * j] = t.x; zw[4 * j + 1] = t.y; zw[4 * j + 2] = t.z; zw[4 * j + 3] = t.w;
        }
      }
      tile_record16<TMF>(zw, blk < J.nblk, blk, M, J.tiles + (int64_t)set * 3);
    }
  }
  // any other tie (rare): the whole set again on the exact pocketfft replica
  while (redo) {
    const int k = __builtin_ctzll(redo);
    redo &= redo - 1;
    const int g = g0 + k * nwaves;
    const DctJob &J = jobs.j[job_of(g)];
    const int set = g - J.set0;
    uint2 w[8];
    load(J, set, w);
    dct_block_2ph<TABLE, LAYOUT>(w, st, J.table);
    store(J, set);
  }
}

// ---------------------------------------------------------------------------
// Block-level helpers (transform.dct2 / idct2, quantization.jpeg_quantize /
// invert_jpeg_quantize on arbitrary float64 / int blocks): one block per lane.
__global__ __launch_bounds__(256) void k_dct2_f64(const double *__restrict__ in, int64_t nblk, double *__restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  const double *p = in + b * 64;
  double a[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    double x[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) x[n] = p[r * 8 + n];
    dct8h(x, a[r]);
  }
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    double xc[8], y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) xc[r] = a[r][v];
    dct8h(xc, y);
#pragma unroll
    for (int u = 0; u < 8; ++u) out[b * 64 + u * 8 + v] = y[u] / (rho(u) * rho(v));  // exact power-of-2 rescale
  }
}

__global__ __launch_bounds__(256) void k_idct2_f64(const double *__restrict__ in, int64_t nblk, double *__restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  const double *p = in + b * 64;
  double a[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    double x[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) x[n] = p[r * 8 + n];
    idct8<double>(x, a[r]);
  }
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    double xc[8], y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) xc[r] = a[r][v];
    idct8<double>(xc, y);
#pragma unroll
    for (int r = 0; r < 8; ++r) out[b * 64 + r * 8 + v] = y[r] * 0x1p-8;  // == y / 256
  }
}

__global__ void k_quantize_f64(const double *__restrict__ in, int64_t n, int table, int32_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (int32_t)__builtin_rint(in[i] / (double)QT[table][i & 63]);
}

__global__ void k_dequantize_i32(const int32_t *__restrict__ in, int64_t n, int table, int64_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (int64_t)in[i] * QT[table][i & 63];
}

inline bool aligned(const void *p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

// Forward-path selection (A/B tests only; every path is bit-exact): knob
// "dct_path" 1 = float64 AAN fast path (k_dct_planes, the default), 2 = the same
// (its prefetch variant is compiled out), 0 = the exact pocketfft replica for every
// block; "dct_waves_per_cu" = persistent grid size (0 = one wave per set).  Round 5
// measured and removed the packed-float32 (path 3) and two-lanes-per-block (path 4)
// kernels (commit ae5c500 holds them).  Set through
// hic_set_knob (common.hip); the library reads no environment variables.
inline int dct_path() { return knob(HIC_KNOB_DCT_PATH); }
inline int dct_waves_per_cu(int njobs) {
  const int v = knob(HIC_KNOB_DCT_WAVES_PER_CU);
  if (v >= 0) return v;
  // float64 path: one wave per set for a multi-plane launch (the hardware's dispatch
  // balances the planes' mixed tail: 8K Y + Cr + Cb 37.5 us vs 39.7 for 12
  // persistent waves per CU), 12 persistent waves per CU for one plane (4K luma
  // 13.4 vs 13.8 us, 8K luma 27.4 vs 27.8; scripts/gpu_r2aj.sh)
  return njobs > 1 ? 0 : 12;
}

inline bool fwd_fast(int H, int W, int64_t stride, const void *plane, const void *out) {
  return (H % 8 == 0) && (W % 8 == 0) && (stride % 8 == 0) && aligned(plane, 8) && aligned(out, 16);
}

// Persistent launch of k_dct_planes over the jobs' sets (all fast-path planes).
template <int TABLE, int LAYOUT, int TMF>
int launch_planes(DctJobs &jobs, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  int total = 0;
  for (int k = 0; k < jobs.n; ++k) {
    jobs.j[k].set0 = total;
    total += jobs.j[k].nsets;
  }
  jobs.total_sets = total;
  int cap = dct_waves_per_cu(jobs.n) * cu_count();
  if (cap > 0 && (total + cap - 1) / cap > 64) cap = (total + 63) / 64;  // <= 64 sets per wave (redo mask)
  const int waves = (cap == 0 || total < cap) ? total : cap;
  const dim3 grid((waves + 3) / 4), block(256);
  const int path = dct_path();
  if (e0 || e1)
    hipExtLaunchKernelGGL((k_dct_planes<TABLE, LAYOUT, TMF>), grid, block, 0, s, e0, e1, 0, jobs, path);
  else
    hipLaunchKernelGGL((k_dct_planes<TABLE, LAYOUT, TMF>), grid, block, 0, s, jobs, path);
  return check_launch("k_dct_planes");
}

inline DctJob make_job(const uint8_t *plane, int H, int W, int64_t stride, int table, void *out, int64_t *tiles) {
  const int nbx = (W + 7) / 8, nblk = nbx * ((H + 7) / 8);
  return DctJob{plane, stride, out, tiles, W, nbx, nblk, (nblk + 63) / 64, 0, table};
}

template <int TABLE, int LAYOUT>
int launch_fwd(const uint8_t *plane, int H, int W, int64_t stride, void *out, hipStream_t s, hipEvent_t e0,
               hipEvent_t e1) {
  const int nbx = (W + 7) / 8, nby = (H + 7) / 8, nblk = nbx * nby;
  const bool fast = fwd_fast(H, W, stride, plane, out);
  const dim3 grid((nblk + 255) / 256), block(256);
  if (fast) {
    DctJobs jobs{};
    jobs.n = 1;
    jobs.j[0] = make_job(plane, H, W, stride, TABLE, out, nullptr);
    return launch_planes<TABLE, LAYOUT, -1>(jobs, s, e0, e1);
  } else if (e0 || e1)
    hipExtLaunchKernelGGL((k_dct_quant<TABLE, LAYOUT, false>), grid, block, 0, s, e0, e1, 0, plane, H, W, stride, nbx,
                          nblk, out);
  else
    hipLaunchKernelGGL((k_dct_quant<TABLE, LAYOUT, false>), grid, block, 0, s, plane, H, W, stride, nbx, nblk, out);
  return check_launch("k_dct_quant");
}

template <int TABLE, int LAYOUT>
int launch_inv(const void *coef, int H, int W, uint8_t *out, int64_t ostride, hipStream_t s) {
  const int nbx = (W + 7) / 8, nby = (H + 7) / 8, nblk = nbx * nby;
  const bool fast = (H % 8 == 0) && (W % 8 == 0) && (ostride % 8 == 0) && aligned(out, 8) && aligned(coef, 16);
  const dim3 grid((nblk + 255) / 256), block(256);
  if (fast)
    hipLaunchKernelGGL((k_dequant_idct<TABLE, LAYOUT, true>), grid, block, 0, s, coef, H, W, nbx, nblk, out, ostride);
  else
    hipLaunchKernelGGL((k_dequant_idct<TABLE, LAYOUT, false>), grid, block, 0, s, coef, H, W, nbx, nblk, out, ostride);
  return check_launch("k_dequant_idct");
}

bool dims_ok(int64_t H, int64_t W) {
  // one lane per block, int32 block / element indices
  return H > 0 && W > 0 && H < (1 << 20) && W < (1 << 20) && ((H + 7) / 8) * ((W + 7) / 8) < (1LL << 31) / 256;
}

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" int hic_dct_quant_u8(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                                int layout, void *out, void *stream) {
  return hic_dct_quant_u8_timed(plane, H, W, stride, table_id, layout, out, stream, nullptr, nullptr);
}

extern "C" int hic_dct_quant_u8_timed(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                                      int layout, void *out, void *stream, void *ev_start, void *ev_stop) {
  if (!plane || !out) return arg_error("null pointer");
  if (!dims_ok(H, W) || stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  hipStream_t s = as_stream(stream);
  const int h = (int)H, w = (int)W;
#define HIC_FWD(T, L) \
  return launch_fwd<T, L>(plane, h, w, stride, out, s, (hipEvent_t)ev_start, (hipEvent_t)ev_stop)
  if (table_id == 0) {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_FWD(0, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_FWD(0, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_FWD(0, HIC_LAYOUT_ZIGZAG_I16);
  } else {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_FWD(1, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_FWD(1, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_FWD(1, HIC_LAYOUT_ZIGZAG_I16);
  }
#undef HIC_FWD
  return arg_error("layout");
}

extern "C" int hic_dct_quant_rle_u8(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                                    int max_len, int16_t *out, void *rle_workspace, void *stream, void *ev_start,
                                    void *ev_stop) {
  hic_dct_plane_job job{plane, H, W, stride, table_id, out, rle_workspace};
  return hic_dct_quant_rle_u8_batch(1, &job, max_len, stream, ev_start, ev_stop);
}

extern "C" int hic_dct_quant_rle_u8_batch(int n, const hic_dct_plane_job *jobs, int max_len, void *stream,
                                          void *ev_start, void *ev_stop) {
  if (n < 1 || n > kMaxPlaneJobs || !jobs) return arg_error("1 <= n <= %d planes", kMaxPlaneJobs);
  if (max_len < 1 || max_len > 256) return arg_error("max_len must be in [1, 256]");
  hipStream_t s = as_stream(stream);
  const hipEvent_t e0 = (hipEvent_t)ev_start, e1 = (hipEvent_t)ev_stop;
  // fast-path planes: one launch for all of them (the kernel reads each plane's
  // table at run time)
  const bool merge = true;
  DctJobs fastj[2] = {};
  // rle_workspace: every job's or none (NULL: the records-free pass, DCT + quantize +
  // zig-zag only)
  const bool recs = jobs[0].rle_workspace != nullptr;
  // every job is checked before anything is launched (an error on job k > 0
  // used to return after the ragged planes before it were queued)
  for (int k = 0; k < n; ++k) {
    const hic_dct_plane_job &a = jobs[k];
    if (!a.plane || !a.out) return arg_error("plane %d: null pointer", k);
    if ((a.rle_workspace != nullptr) != recs) return arg_error("plane %d: rle_workspace for every plane or none", k);
    if (!dims_ok(a.H, a.W) || a.stride < a.W) return arg_error("plane %d: shape / stride", k);
    if (a.table_id != HIC_TABLE_LUMINANCE && a.table_id != HIC_TABLE_CHROMINANCE) return arg_error("plane %d: table_id", k);
  }
  for (int k = 0; k < n; ++k) {
    const hic_dct_plane_job &a = jobs[k];
    const int h = (int)a.H, w = (int)a.W;
    int64_t *tiles = static_cast<int64_t *>(a.rle_workspace);
    if (fwd_fast(h, w, a.stride, a.plane, a.out)) {
      DctJobs &J = fastj[merge ? 0 : a.table_id];
      J.j[J.n++] = make_job(a.plane, h, w, a.stride, a.table_id, a.out, tiles);
      continue;
    }
    // ragged plane: pocketfft replica, then the stand-alone tile pass
    const int e = a.table_id == 0 ? launch_fwd<0, HIC_LAYOUT_ZIGZAG_I16>(a.plane, h, w, a.stride, a.out, s, e0, e1)
                                  : launch_fwd<1, HIC_LAYOUT_ZIGZAG_I16>(a.plane, h, w, a.stride, a.out, s, e0, e1);
    if (e) return e;
    if (recs)
      if (int e2 = rle_tile16_launch(a.out, (int64_t)((h + 7) / 8) * ((w + 7) / 8), max_len, tiles, s)) return e2;
  }
  // the events (if any) time the first launch
  bool timed = false;
  for (int t = 0; t < 2; ++t) {
    DctJobs &J = fastj[t];
    if (J.n == 0) continue;
    J.M = max_len;
    const hipEvent_t a0 = timed ? nullptr : e0, a1 = timed ? nullptr : e1;
    timed = true;
    // one table for every job (a batch of luminance planes, say): the kernel compiled
    // for it, whose quantiser constants are literals instead of scalar loads per set
    int uni = J.j[0].table;
    for (int k = 1; k < J.n; ++k)
      if (J.j[k].table != uni) uni = -1;
    if (!merge) uni = t;
    int e;
    if (!recs)
      e = uni == 0   ? launch_planes<0, HIC_LAYOUT_ZIGZAG_I16, -1>(J, s, a0, a1)
          : uni == 1 ? launch_planes<1, HIC_LAYOUT_ZIGZAG_I16, -1>(J, s, a0, a1)
                     : launch_planes<-1, HIC_LAYOUT_ZIGZAG_I16, -1>(J, s, a0, a1);
    else if (uni == 0)
      e = max_len == 15 ? launch_planes<0, HIC_LAYOUT_ZIGZAG_I16, 15>(J, s, a0, a1)
                        : launch_planes<0, HIC_LAYOUT_ZIGZAG_I16, 0>(J, s, a0, a1);
    else if (uni == 1)
      e = max_len == 15 ? launch_planes<1, HIC_LAYOUT_ZIGZAG_I16, 15>(J, s, a0, a1)
                        : launch_planes<1, HIC_LAYOUT_ZIGZAG_I16, 0>(J, s, a0, a1);
    else
      e = max_len == 15 ? launch_planes<-1, HIC_LAYOUT_ZIGZAG_I16, 15>(J, s, a0, a1)
                        : launch_planes<-1, HIC_LAYOUT_ZIGZAG_I16, 0>(J, s, a0, a1);
    if (e) return e;
  }
  return HIC_OK;
}

extern "C" int hic_dequant_idct_u8(const void *coef, int layout, int64_t H, int64_t W, int table_id,
                                   uint8_t *out, int64_t out_stride, void *stream) {
  if (!coef || !out) return arg_error("null pointer");
  if (!dims_ok(H, W) || out_stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  hipStream_t s = as_stream(stream);
  const int h = (int)H, w = (int)W;
#define HIC_INV(T, L) return launch_inv<T, L>(coef, h, w, out, out_stride, s)
  if (table_id == 0) {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_INV(0, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_INV(0, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_INV(0, HIC_LAYOUT_ZIGZAG_I16);
  } else {
    if (layout == HIC_LAYOUT_RASTER_I32) HIC_INV(1, HIC_LAYOUT_RASTER_I32);
    if (layout == HIC_LAYOUT_RASTER_I16) HIC_INV(1, HIC_LAYOUT_RASTER_I16);
    if (layout == HIC_LAYOUT_ZIGZAG_I16) HIC_INV(1, HIC_LAYOUT_ZIGZAG_I16);
  }
#undef HIC_INV
  return arg_error("layout");
}

extern "C" int hic_rle_decode_idct_u8_indexed(const uint8_t *sym_len, const int16_t *sym_val, const int64_t *d_nsym,
                                              const int32_t *dc_diff, const int64_t *d_index, int64_t H, int64_t W,
                                              int table_id, uint8_t *out, int64_t out_stride, int64_t *d_status,
                                              void *stream) {
  if (!sym_len || !sym_val || !d_nsym || !dc_diff || !d_index || !out || !d_status) return arg_error("null pointer");
  if (!dims_ok(H, W) || out_stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  if ((reinterpret_cast<uintptr_t>(sym_len) | reinterpret_cast<uintptr_t>(sym_val)) % 16)
    return arg_error("symbol arrays must be 16-byte aligned");
  const int nbx = (int)((W + 7) / 8);
  const int64_t nblk = (int64_t)nbx * ((H + 7) / 8);
  if (nblk * 63 >= ((int64_t)1 << 31)) return arg_error("plane too large (AC stream >= 2^31)");
  const bool fast = H % 8 == 0 && W % 8 == 0 && out_stride % 8 == 0 && aligned(out, 8);
  const int64_t ntiles = (nblk + 63) / 64;
  const dim3 grid((unsigned)((ntiles + 3) / 4)), block(256);
  hipStream_t s = as_stream(stream);
  const int h = (int)H, w = (int)W;
#define HIC_RI(T, F)                                                                                              \
  hipLaunchKernelGGL((k_rld_idct_indexed<T, F>), grid, block, 0, s, sym_len, sym_val, d_nsym, dc_diff, d_index, h, \
                     w, nbx, nblk, out, out_stride, d_status)
  if (table_id == 0 && fast) HIC_RI(0, true);
  else if (table_id == 0) HIC_RI(0, false);
  else if (fast) HIC_RI(1, true);
  else HIC_RI(1, false);
#undef HIC_RI
  return check_launch("k_rld_idct_indexed");
}

extern "C" int hic_rle_decode_idct_u8_indexed_pair(const uint8_t *const *h_sym_len, const int16_t *const *h_sym_val,
                                                   const int64_t *const *h_d_nsym, const int32_t *const *h_dc_diff,
                                                   const int64_t *const *h_d_index, int64_t H, int64_t W, int table_id,
                                                   uint8_t *const *h_out, int64_t out_stride, int64_t *const *h_d_status,
                                                   void *stream) {
  if (!h_sym_len || !h_sym_val || !h_d_nsym || !h_dc_diff || !h_d_index || !h_out || !h_d_status)
    return arg_error("null pointer");
  for (int k = 0; k < 2; ++k) {
    if (!h_sym_len[k] || !h_sym_val[k] || !h_d_nsym[k] || !h_dc_diff[k] || !h_d_index[k] || !h_out[k] ||
        !h_d_status[k])
      return arg_error("plane %d: null pointer", k);
    if ((reinterpret_cast<uintptr_t>(h_sym_len[k]) | reinterpret_cast<uintptr_t>(h_sym_val[k])) % 16)
      return arg_error("plane %d: symbol arrays must be 16-byte aligned", k);
  }
  if (!dims_ok(H, W) || out_stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  const int nbx = (int)((W + 7) / 8);
  const int64_t nblk = (int64_t)nbx * ((H + 7) / 8);
  if (nblk * 63 >= ((int64_t)1 << 31)) return arg_error("plane too large (AC stream >= 2^31)");
  const bool fast = H % 8 == 0 && W % 8 == 0 && out_stride % 8 == 0 && aligned(h_out[0], 8) && aligned(h_out[1], 8);
  const int64_t ntiles = (nblk + 63) / 64;
  const dim3 grid((unsigned)((2 * ntiles + 3) / 4)), block(256);
  hipStream_t s = as_stream(stream);
  const DecPlane p1{h_sym_len[1], h_sym_val[1], h_d_nsym[1], h_dc_diff[1], h_d_index[1], h_out[1], h_d_status[1]};
#define HIC_RI2(T, F)                                                                                              \
  hipLaunchKernelGGL((k_rld_idct_indexed<T, F>), grid, block, 0, s, h_sym_len[0], h_sym_val[0], h_d_nsym[0],     \
                     h_dc_diff[0], h_d_index[0], (int)H, (int)W, nbx, nblk, h_out[0], out_stride, h_d_status[0], \
                     nullptr, nullptr, p1)
  if (table_id == 0 && fast) HIC_RI2(0, true);
  else if (table_id == 0) HIC_RI2(0, false);
  else if (fast) HIC_RI2(1, true);
  else HIC_RI2(1, false);
#undef HIC_RI2
  return check_launch("k_rld_idct_indexed<pair>");
}

extern "C" int hic_rle_decode_idct_rgb_indexed(const uint8_t *sym_len, const int16_t *sym_val, const int64_t *d_nsym,
                                               const int32_t *dc_diff, const int64_t *d_index, int64_t H, int64_t W,
                                               const uint8_t *cr, const uint8_t *cb, uint8_t *rgb, int64_t rgb_stride,
                                               int64_t *d_status, void *stream) {
  if (!sym_len || !sym_val || !d_nsym || !dc_diff || !d_index || !cr || !cb || !rgb || !d_status)
    return arg_error("null pointer");
  if (!dims_ok(H, W) || H % 8 || W % 8) return arg_error("plane shape (H, W multiples of 8)");
  if (rgb_stride < 3 * W || rgb_stride % 8 || !aligned(rgb, 8)) return arg_error("rgb stride / alignment (8 B)");
  if (!aligned(cr, 4) || !aligned(cb, 4)) return arg_error("chroma planes must be 4-byte aligned");
  if ((reinterpret_cast<uintptr_t>(sym_len) | reinterpret_cast<uintptr_t>(sym_val)) % 16)
    return arg_error("symbol arrays must be 16-byte aligned");
  const int nbx = (int)(W / 8);
  const int64_t nblk = (int64_t)nbx * (H / 8);
  if (nblk * 63 >= ((int64_t)1 << 31)) return arg_error("plane too large (AC stream >= 2^31)");
  const int64_t ntiles = (nblk + 63) / 64;
  hipLaunchKernelGGL((k_rld_idct_indexed<0, true, true>), dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0,
                     as_stream(stream), sym_len, sym_val, d_nsym, dc_diff, d_index, (int)H, (int)W, nbx, nblk, rgb,
                     rgb_stride, d_status, cr, cb);
  return check_launch("k_rld_idct_indexed<rgb>");
}

// ---- the slot-layout decoders (slots.h): the *_indexed entry points above, reading
// the slots through the close's record index
static int slots_args(const void *slot_len, const void *slot_val, int records_per_tile, int64_t nblk) {
  if (records_per_tile != 1 && records_per_tile != 2) return arg_error("records_per_tile must be 1 or 2");
  if (nblk % (64 / records_per_tile)) return arg_error("the plane's blocks must form whole records");
  if ((reinterpret_cast<uintptr_t>(slot_len) | reinterpret_cast<uintptr_t>(slot_val)) % 16)
    return arg_error("slot arrays must be 16-byte aligned");
  return HIC_OK;
}

extern "C" int hic_rle_decode_idct_u8_slots(const uint8_t *slot_len, const int16_t *slot_val, const int64_t *d_nsym,
                                            const int32_t *dc_diff, const int32_t *d_index, int records_per_tile,
                                            int64_t H, int64_t W, int table_id, uint8_t *out, int64_t out_stride,
                                            int64_t *d_status, void *stream) {
  if (!slot_len || !slot_val || !d_nsym || !dc_diff || !d_index || !out || !d_status) return arg_error("null pointer");
  if (!dims_ok(H, W) || out_stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  const int nbx = (int)((W + 7) / 8);
  const int64_t nblk = (int64_t)nbx * ((H + 7) / 8);
  if (nblk * 63 >= ((int64_t)1 << 31)) return arg_error("plane too large (AC stream >= 2^31)");
  if (int e = slots_args(slot_len, slot_val, records_per_tile, nblk)) return e;
  const bool fast = H % 8 == 0 && W % 8 == 0 && out_stride % 8 == 0 && aligned(out, 8);
  const int64_t ntiles = (nblk + 63) / 64;
  const dim3 grid((unsigned)((ntiles + 3) / 4)), block(256);
  hipStream_t s = as_stream(stream);
  const int h = (int)H, w = (int)W, rsh = records_per_tile == 2 ? 1 : 0;
  const int64_t *ix = reinterpret_cast<const int64_t *>(d_index);
#define HIC_RS(T, F)                                                                                                \
  hipLaunchKernelGGL((k_rld_idct_indexed<T, F, false, true>), grid, block, 0, s, slot_len, slot_val, d_nsym, dc_diff, \
                     ix, h, w, nbx, nblk, out, out_stride, d_status, nullptr, nullptr, DecPlane{}, rsh)
  if (table_id == 0 && fast) HIC_RS(0, true);
  else if (table_id == 0) HIC_RS(0, false);
  else if (fast) HIC_RS(1, true);
  else HIC_RS(1, false);
#undef HIC_RS
  return check_launch("k_rld_idct_indexed<slots>");
}

extern "C" int hic_rle_decode_idct_u8_slots_pair(const uint8_t *const *h_slot_len, const int16_t *const *h_slot_val,
                                                 const int64_t *const *h_d_nsym, const int32_t *const *h_dc_diff,
                                                 const int32_t *const *h_d_index, int records_per_tile, int64_t H,
                                                 int64_t W, int table_id, uint8_t *const *h_out, int64_t out_stride,
                                                 int64_t *const *h_d_status, void *stream) {
  if (!h_slot_len || !h_slot_val || !h_d_nsym || !h_dc_diff || !h_d_index || !h_out || !h_d_status)
    return arg_error("null pointer");
  if (!dims_ok(H, W) || out_stride < W) return arg_error("plane shape / stride");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  const int nbx = (int)((W + 7) / 8);
  const int64_t nblk = (int64_t)nbx * ((H + 7) / 8);
  if (nblk * 63 >= ((int64_t)1 << 31)) return arg_error("plane too large (AC stream >= 2^31)");
  for (int k = 0; k < 2; ++k) {
    if (!h_slot_len[k] || !h_slot_val[k] || !h_d_nsym[k] || !h_dc_diff[k] || !h_d_index[k] || !h_out[k] ||
        !h_d_status[k])
      return arg_error("plane %d: null pointer", k);
    if (int e = slots_args(h_slot_len[k], h_slot_val[k], records_per_tile, nblk)) return e;
  }
  const bool fast = H % 8 == 0 && W % 8 == 0 && out_stride % 8 == 0 && aligned(h_out[0], 8) && aligned(h_out[1], 8);
  const int64_t ntiles = (nblk + 63) / 64;
  const dim3 grid((unsigned)((2 * ntiles + 3) / 4)), block(256);
  hipStream_t s = as_stream(stream);
  const int rsh = records_per_tile == 2 ? 1 : 0;
  const DecPlane p1{h_slot_len[1], h_slot_val[1], h_d_nsym[1], h_dc_diff[1],
                    reinterpret_cast<const int64_t *>(h_d_index[1]), h_out[1], h_d_status[1]};
#define HIC_RS2(T, F)                                                                                              \
  hipLaunchKernelGGL((k_rld_idct_indexed<T, F, false, true>), grid, block, 0, s, h_slot_len[0], h_slot_val[0],    \
                     h_d_nsym[0], h_dc_diff[0], reinterpret_cast<const int64_t *>(h_d_index[0]), (int)H, (int)W, nbx, \
                     nblk, h_out[0], out_stride, h_d_status[0], nullptr, nullptr, p1, rsh)
  if (table_id == 0 && fast) HIC_RS2(0, true);
  else if (table_id == 0) HIC_RS2(0, false);
  else if (fast) HIC_RS2(1, true);
  else HIC_RS2(1, false);
#undef HIC_RS2
  return check_launch("k_rld_idct_indexed<slots pair>");
}

extern "C" int hic_rle_decode_idct_rgb_slots(const uint8_t *slot_len, const int16_t *slot_val, const int64_t *d_nsym,
                                             const int32_t *dc_diff, const int32_t *d_index, int records_per_tile,
                                             int64_t H, int64_t W, const uint8_t *cr, const uint8_t *cb, uint8_t *rgb,
                                             int64_t rgb_stride, int64_t *d_status, void *stream) {
  if (!slot_len || !slot_val || !d_nsym || !dc_diff || !d_index || !cr || !cb || !rgb || !d_status)
    return arg_error("null pointer");
  if (!dims_ok(H, W) || H % 8 || W % 8) return arg_error("plane shape (H, W multiples of 8)");
  if (rgb_stride < 3 * W || rgb_stride % 8 || !aligned(rgb, 8)) return arg_error("rgb stride / alignment (8 B)");
  if (!aligned(cr, 4) || !aligned(cb, 4)) return arg_error("chroma planes must be 4-byte aligned");
  const int nbx = (int)(W / 8);
  const int64_t nblk = (int64_t)nbx * (H / 8);
  if (nblk * 63 >= ((int64_t)1 << 31)) return arg_error("plane too large (AC stream >= 2^31)");
  if (int e = slots_args(slot_len, slot_val, records_per_tile, nblk)) return e;
  const int64_t ntiles = (nblk + 63) / 64;
  hipLaunchKernelGGL((k_rld_idct_indexed<0, true, true, true>), dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0,
                     as_stream(stream), slot_len, slot_val, d_nsym, dc_diff, reinterpret_cast<const int64_t *>(d_index),
                     (int)H, (int)W, nbx, nblk, rgb, rgb_stride, d_status, cr, cb, DecPlane{},
                     records_per_tile == 2 ? 1 : 0);
  return check_launch("k_rld_idct_indexed<rgb slots>");
}

extern "C" int hic_dct2_f64(const double *in, int64_t nblk, double *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  hipLaunchKernelGGL(k_dct2_f64, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, as_stream(stream), in, nblk, out);
  return check_launch("k_dct2_f64");
}

extern "C" int hic_idct2_f64(const double *in, int64_t nblk, double *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  hipLaunchKernelGGL(k_idct2_f64, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, as_stream(stream), in, nblk, out);
  return check_launch("k_idct2_f64");
}

extern "C" int hic_quantize_f64(const double *in, int64_t nblk, int table_id, int32_t *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (table_id != 0 && table_id != 1) return arg_error("table_id");
  const int64_t n = nblk * 64;
  hipLaunchKernelGGL(k_quantize_f64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), in, n,
                     table_id, out);
  return check_launch("k_quantize_f64");
}

extern "C" int hic_dequantize_i32(const int32_t *in, int64_t nblk, int table_id, int64_t *out, void *stream) {
  if (!in || !out) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (table_id != 0 && table_id != 1) return arg_error("table_id");
  const int64_t n = nblk * 64;
  hipLaunchKernelGGL(k_dequantize_i32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), in, n,
                     table_id, out);
  return check_launch("k_dequantize_i32");
}
