// wire.hip -- the gather's lossless wire format for quantized zig-zag blocks
// (DESIGN.md section 6): slot z of a block is stored in kWireW[table][z] bits of
// two's complement, the per-slot widths proven sufficient by
// tools/check/wire_widths.py (hiccup's unnormalised DCT of pixels - 128 is
// bounded by 4 * 128 * S_u * S_v, divided by the table entry), so a luminance
// block is 637 bits and a chrominance block 597 (against 1024 as int16).  Blocks
// are packed back to back; a 64-block tile is 2 * bits-per-block 32-bit words
// (whole words for any width), stored at a stride rounded up to 16 bytes.  Bit i
// of a tile is bit (i & 31) of its word i >> 5 (LSB first).  The pack kernel
// checks every value against its width and raises *d_flag on a violation; the
// stream gather points d_flag at a trailer word of the sender's segment, so the
// flag travels with the data and the receiver turns it into the stream's count
// (HIC_COUNT_WIRE_OVERFLOW, sharding.ShardEncoder.finish).
//
//  hic_wire_pack_i16:   nblk blocks (64 int16, ZIGZAG_I16) -> ceil(nblk / 64) tiles
//  hic_wire_unpack_i16: the inverse (blocks past nblk in the last tile dropped)
//  hic_rle_records_rebase: a shard's RLE tile records moved into the whole
//                       image's record array (positions + pos_shift), so the
//                       gathering rank runs the scan + emit without a tile pass
#include "hic_common.h"
#include "wire_widths.h"

namespace hic {
namespace {

constexpr int kWPB = 4;  // waves per workgroup
template <int TABLE>
struct WireGeo {
  static constexpr int kBits = kWireBits[TABLE];                    // per block
  static constexpr int kWords = 2 * kBits;                          // per 64-block tile
  static constexpr int kStride = (kWords + 3) / 4 * 4;              // words per tile on the wire
};
static_assert(WireGeo<0>::kStride <= 1280 && WireGeo<1>::kStride <= 1280, "LDS tile");
constexpr int kTileLds = 1280;  // words of the LDS tile (>= every stride)

// pack: lane j = block j of the wave's tile; its bits are ORed into the LDS tile
// at bit kBits * j (the two words a lane shares with its neighbours need the OR)
template <int TABLE>
__global__ __launch_bounds__(64 * kWPB) void k_wire_pack(const int16_t *__restrict__ blocks, int64_t nblk,
                                                         uint32_t *__restrict__ out, int *__restrict__ flag) {
  using G = WireGeo<TABLE>;
  __shared__ uint32_t s_tile[kWPB][kTileLds];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t ntiles = (nblk + 63) / 64;
  const int64_t t = (int64_t)blockIdx.x * kWPB + wv;
  if (t >= ntiles) return;  // wave-uniform
  uint32_t *st = s_tile[wv];
  for (int i = lane; i < G::kStride; i += 64) st[i] = 0;
  __builtin_amdgcn_wave_barrier();
  const int64_t b = t * 64 + lane;
  uint32_t w[32];
  if (b < nblk) {
    const uint4 *q = reinterpret_cast<const uint4 *>(blocks + b * 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 v = q[k];
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 32; ++k) w[k] = 0;
  }
  // stream the fields into 32-bit words: acc holds `n` pending bits (LSB first)
  const int bit0 = lane * G::kBits;
  int wi = bit0 >> 5, n = bit0 & 31;
  uint64_t acc = 0;
  bool bad = false;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const int nb = kWireW[TABLE][i];
    const int v = (int)(int16_t)((w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
    bad |= v < -(1 << (nb - 1)) || v >= (1 << (nb - 1));
    acc |= (uint64_t)((uint32_t)v & ((1u << nb) - 1)) << n;
    n += nb;
    if (n >= 32) {
      atomicOr(&st[wi], (uint32_t)acc);  // first / last word: shared with a neighbour
      ++wi;
      acc >>= 32;
      n -= 32;
    }
  }
  if (n > 0) atomicOr(&st[wi], (uint32_t)acc);
  if (bad) *flag = 1;
  __builtin_amdgcn_wave_barrier();
  uint4 *o = reinterpret_cast<uint4 *>(out + t * G::kStride);
  for (int c = lane; c < G::kStride / 4; c += 64)
    o[c] = make_uint4(st[4 * c], st[4 * c + 1], st[4 * c + 2], st[4 * c + 3]);
}

// unpack: the tile into LDS (coalesced), lane j extracts block j into its stage
// row, the stage leaves as 1 KiB stores
constexpr int kRowU4 = 9;  // 144 B stage rows (128 B + pad)
template <int TABLE>
__global__ __launch_bounds__(64 * kWPB) void k_wire_unpack(const uint32_t *__restrict__ wire, int64_t nblk,
                                                           int16_t *__restrict__ blocks) {
  using G = WireGeo<TABLE>;
  __shared__ uint32_t s_tile[kWPB][kTileLds];
  __shared__ uint4 s_stage[kWPB][64 * kRowU4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t ntiles = (nblk + 63) / 64;
  const int64_t t = (int64_t)blockIdx.x * kWPB + wv;
  if (t >= ntiles) return;
  uint32_t *st = s_tile[wv];
  const uint4 *src = reinterpret_cast<const uint4 *>(wire + t * G::kStride);
  for (int c = lane; c < G::kStride / 4; c += 64) {
    const uint4 v = src[c];
    st[4 * c] = v.x; st[4 * c + 1] = v.y; st[4 * c + 2] = v.z; st[4 * c + 3] = v.w;
  }
  if (lane < 4) st[G::kStride + lane] = 0;  // a lane may read one word past its last field
  __builtin_amdgcn_wave_barrier();
  const int bit0 = lane * G::kBits;
  int wi = bit0 >> 5, n = 0;
  uint64_t acc = 0;
  {
    const int ph = bit0 & 31;
    acc = (uint64_t)st[wi++] >> ph;
    n = 32 - ph;
  }
  uint32_t w[32];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const int nb = kWireW[TABLE][i];
    if (n < nb) {
      acc |= (uint64_t)st[wi++] << n;
      n += 32;
    }
    const int h = 1 << (nb - 1);
    const int v = ((int)(acc & ((1u << nb) - 1)) ^ h) - h;  // sign-extend nb bits
    acc >>= nb;
    n -= nb;
    if (i & 1)
      w[i >> 1] |= ((uint32_t)v & 0xFFFFu) << 16;
    else
      w[i >> 1] = (uint32_t)v & 0xFFFFu;
  }
  uint4 *row = s_stage[wv] + lane * kRowU4;
#pragma unroll
  for (int k = 0; k < 8; ++k) row[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  __builtin_amdgcn_wave_barrier();
  // chunk c = 64 k + lane: block c / 8, 16-byte part c % 8
  uint4 *o = reinterpret_cast<uint4 *>(blocks + t * 64 * 64);
  const int64_t nvalid = nblk - t * 64;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = 64 * k + lane, bb = c >> 3;
    if (bb < nvalid) o[c] = s_stage[wv][bb * kRowU4 + (c & 7)];
  }
}

__global__ void k_records_rebase(const int64_t *__restrict__ src, int64_t nrec, int64_t shift,
                                 int64_t *__restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrec) return;
  const int64_t f = src[3 * i], l = src[3 * i + 1];
  dst[3 * i] = f >= 0 ? f + shift : f;
  dst[3 * i + 1] = l >= 0 ? l + shift : l;
  dst[3 * i + 2] = src[3 * i + 2];
}

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" size_t hic_wire_bytes(int64_t nblk, int table_id) {
  if (nblk <= 0 || (table_id != 0 && table_id != 1)) return 0;
  const int stride = table_id == 0 ? WireGeo<0>::kStride : WireGeo<1>::kStride;
  return (size_t)((nblk + 63) / 64) * stride * 4;
}

extern "C" int hic_wire_pack_i16(const int16_t *blocks, int64_t nblk, int table_id, uint8_t *wire, int *d_flag,
                                 void *stream) {
  if (!blocks || !wire || !d_flag) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  if ((reinterpret_cast<uintptr_t>(blocks) | reinterpret_cast<uintptr_t>(wire)) % 16)
    return arg_error("blocks and wire must be 16-byte aligned");
  const int64_t ntiles = (nblk + 63) / 64;
  const dim3 grid((unsigned)((ntiles + kWPB - 1) / kWPB)), block(64 * kWPB);
  uint32_t *w = reinterpret_cast<uint32_t *>(wire);
  if (table_id == 0)
    hipLaunchKernelGGL(k_wire_pack<0>, grid, block, 0, as_stream(stream), blocks, nblk, w, d_flag);
  else
    hipLaunchKernelGGL(k_wire_pack<1>, grid, block, 0, as_stream(stream), blocks, nblk, w, d_flag);
  return check_launch("k_wire_pack");
}

extern "C" int hic_wire_unpack_i16(const uint8_t *wire, int64_t nblk, int table_id, int16_t *blocks, void *stream) {
  if (!blocks || !wire) return arg_error("null pointer");
  if (nblk <= 0) return arg_error("nblk");
  if (table_id != HIC_TABLE_LUMINANCE && table_id != HIC_TABLE_CHROMINANCE) return arg_error("table_id");
  if ((reinterpret_cast<uintptr_t>(blocks) | reinterpret_cast<uintptr_t>(wire)) % 16)
    return arg_error("blocks and wire must be 16-byte aligned");
  const int64_t ntiles = (nblk + 63) / 64;
  const dim3 grid((unsigned)((ntiles + kWPB - 1) / kWPB)), block(64 * kWPB);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(wire);
  if (table_id == 0)
    hipLaunchKernelGGL(k_wire_unpack<0>, grid, block, 0, as_stream(stream), w, nblk, blocks);
  else
    hipLaunchKernelGGL(k_wire_unpack<1>, grid, block, 0, as_stream(stream), w, nblk, blocks);
  return check_launch("k_wire_unpack");
}

extern "C" int hic_rle_records_rebase(const int64_t *d_src, int64_t nrec, int64_t pos_shift, int64_t *d_dst,
                                      void *stream) {
  if (!d_src || !d_dst) return arg_error("null pointer");
  if (nrec < 0 || pos_shift < 0) return arg_error("nrec / pos_shift");
  if (nrec == 0) return HIC_OK;
  hipLaunchKernelGGL(k_records_rebase, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, as_stream(stream), d_src,
                     nrec, pos_shift, d_dst);
  return check_launch("k_records_rebase");
}
