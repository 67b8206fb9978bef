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
__device__ __forceinline__ void wire_pack_tile(const int16_t *__restrict__ blocks, int64_t nblk,
                                               uint32_t *__restrict__ out, int *__restrict__ flag, int64_t t,
                                               int lane, uint32_t *st) {
  using G = WireGeo<TABLE>;
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

template <int TABLE>
__global__ __launch_bounds__(64 * kWPB) void k_wire_pack(const int16_t *__restrict__ blocks, int64_t nblk,
                                                         uint32_t *__restrict__ out, int *__restrict__ flag) {
  __shared__ uint32_t s_tile[kWPB][kTileLds];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * kWPB + wv;
  if (t >= (nblk + 63) / 64) return;  // wave-uniform
  wire_pack_tile<TABLE>(blocks, nblk, out, flag, t, lane, s_tile[wv]);
}

// unpack: the tile into LDS (coalesced), lane j extracts block j into its stage
// row, the stage leaves as 1 KiB stores
constexpr int kRowU4 = 9;  // 144 B stage rows (128 B + pad)
template <int TABLE>
__device__ __forceinline__ void wire_unpack_tile(const uint32_t *__restrict__ wire, int64_t nblk,
                                                 int16_t *__restrict__ blocks, int64_t t, int lane, uint32_t *st,
                                                 uint4 *stage) {
  using G = WireGeo<TABLE>;
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
  uint4 *row = stage + lane * kRowU4;
#pragma unroll
  for (int k = 0; k < 8; ++k) row[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  __builtin_amdgcn_wave_barrier();
  // chunk c = 64 k + lane: block c / 8, 16-byte part c % 8
  uint4 *o = reinterpret_cast<uint4 *>(blocks + t * 64 * 64);
  const int64_t nvalid = nblk - t * 64;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = 64 * k + lane, bb = c >> 3;
    if (bb < nvalid) o[c] = stage[bb * kRowU4 + (c & 7)];
  }
}

template <int TABLE>
__global__ __launch_bounds__(64 * kWPB) void k_wire_unpack(const uint32_t *__restrict__ wire, int64_t nblk,
                                                           int16_t *__restrict__ blocks) {
  __shared__ uint32_t s_tile[kWPB][kTileLds];
  __shared__ uint4 s_stage[kWPB][64 * kRowU4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * kWPB + wv;
  if (t >= (nblk + 63) / 64) return;
  wire_unpack_tile<TABLE>(wire, nblk, blocks, t, lane, s_tile[wv], s_stage[wv]);
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

// Batches (hic_wire_pack_batch / _unpack_batch: a multi-GPU group's segments, 3
// channels x up to 7 peers, in 3 launches instead of ~3 each): the jobs of one table
// in a job table, wave t over their concatenated tiles.
constexpr int kWireJobsMax = 32;
struct WireJobD {
  int16_t *blocks;
  uint32_t *wire;
  int64_t nblk;
  int *flag;
  const int64_t *rec_src;
  int64_t *rec_dst;
  int64_t nrec, shift;
  int64_t *count;
};
struct WireBatch {
  WireJobD j[kWireJobsMax];
  int64_t tile0[kWireJobsMax + 1];
  int n;
};

__device__ __forceinline__ int wire_job_of(const WireBatch &B, int64_t t) {
  int k = 0;
  while (k + 1 < B.n && t >= B.tile0[k + 1]) ++k;  // wave-uniform
  return k;
}

template <int TABLE>
__global__ __launch_bounds__(64 * kWPB) void k_wire_pack_batch(WireBatch B) {
  __shared__ uint32_t s_tile[kWPB][kTileLds];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * kWPB + wv;
  if (t >= B.tile0[B.n]) return;
  const int k = wire_job_of(B, t);
  wire_pack_tile<TABLE>(B.j[k].blocks, B.j[k].nblk, B.j[k].wire, B.j[k].flag, t - B.tile0[k], lane, s_tile[wv]);
}

template <int TABLE>
__global__ __launch_bounds__(64 * kWPB) void k_wire_unpack_batch(WireBatch B) {
  __shared__ uint32_t s_tile[kWPB][kTileLds];
  __shared__ uint4 s_stage[kWPB][64 * kRowU4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * kWPB + wv;
  if (t >= B.tile0[B.n]) return;
  const int k = wire_job_of(B, t);
  wire_unpack_tile<TABLE>(B.j[k].wire, B.j[k].nblk, B.j[k].blocks, t - B.tile0[k], lane, s_tile[wv], s_stage[wv]);
}

// every job's records rebased (blockIdx.y = job) and, for a pack, its flag cleared
__global__ void k_wire_prep_batch(WireBatch B, int clear_flags) {
  const WireJobD &J = B.j[blockIdx.y];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (clear_flags && i == 0 && J.flag) *J.flag = 0;
  if (!J.rec_src || i >= J.nrec) return;
  const int64_t f = J.rec_src[3 * i], l = J.rec_src[3 * i + 1];
  J.rec_dst[3 * i] = f >= 0 ? f + J.shift : f;
  J.rec_dst[3 * i + 1] = l >= 0 ? l + J.shift : l;
  J.rec_dst[3 * i + 2] = J.rec_src[3 * i + 2];
}

// a job whose sender flag is raised overrides its stream's count
__global__ void k_wire_flags_apply(WireBatch B) {
  const int k = threadIdx.x;
  if (k >= B.n) return;
  const WireJobD &J = B.j[k];
  if (J.flag && J.count && *J.flag != 0) *J.count = HIC_COUNT_WIRE_OVERFLOW;
}

}  // namespace
}  // namespace hic

using namespace hic;

namespace {
// checks the jobs and sorts them into the all-jobs table and one table per
// quantisation table (tile prefix sums over their blocks)
int wire_tables(int n, const hic_wire_job *jobs, bool pack, WireBatch &all, WireBatch (&tb)[2], int64_t &maxrec) {
  if (n < 1 || n > kWireJobsMax || !jobs) return arg_error("1 <= n <= %d wire jobs", kWireJobsMax);
  all = WireBatch{};
  tb[0] = WireBatch{};
  tb[1] = WireBatch{};
  maxrec = 0;
  for (int i = 0; i < n; ++i) {
    const hic_wire_job &J = jobs[i];
    if (J.table_id != HIC_TABLE_LUMINANCE && J.table_id != HIC_TABLE_CHROMINANCE) return arg_error("job %d: table", i);
    if (J.nblk < 0 || J.nrec < 0 || J.pos_shift < 0) return arg_error("job %d: nblk / nrec / pos_shift", i);
    if (J.nblk > 0 && (!J.blocks || !J.wire || (pack && !J.d_flag))) return arg_error("job %d: null pointer", i);
    if (J.nblk > 0 && (reinterpret_cast<uintptr_t>(J.blocks) | reinterpret_cast<uintptr_t>(J.wire)) % 16)
      return arg_error("job %d: blocks and wire must be 16-byte aligned", i);
    if (J.nrec > 0 && (!J.rec_src || !J.rec_dst)) return arg_error("job %d: records need src and dst", i);
    const WireJobD d{J.blocks, reinterpret_cast<uint32_t *>(J.wire), J.nblk, J.d_flag, J.rec_src, J.rec_dst,
                     J.nrec, J.pos_shift, J.d_count};
    all.j[all.n++] = d;
    if (J.nrec > maxrec) maxrec = J.nrec;
    if (J.nblk > 0) {
      WireBatch &T = tb[J.table_id];
      T.tile0[T.n + 1] = T.tile0[T.n] + (J.nblk + 63) / 64;
      T.j[T.n++] = d;
    }
  }
  return HIC_OK;
}

int wire_batch(int n, const hic_wire_job *jobs, bool pack, void *stream) {
  WireBatch all, tb[2];
  int64_t maxrec;
  if (int e = wire_tables(n, jobs, pack, all, tb, maxrec)) return e;
  const hipStream_t s = as_stream(stream);
  const unsigned gx = (unsigned)((maxrec + 255) / 256 > 0 ? (maxrec + 255) / 256 : 1);
  hipLaunchKernelGGL(k_wire_prep_batch, dim3(gx, (unsigned)all.n), dim3(256), 0, s, all, pack ? 1 : 0);
  if (int e = check_launch("k_wire_prep_batch")) return e;
  for (int tbl = 0; tbl < 2; ++tbl) {
    const WireBatch &B = tb[tbl];
    if (B.n == 0) continue;
    const dim3 grid((unsigned)((B.tile0[B.n] + kWPB - 1) / kWPB)), block(64 * kWPB);
    if (pack)
      hipLaunchKernelGGL(tbl == 0 ? k_wire_pack_batch<0> : k_wire_pack_batch<1>, grid, block, 0, s, B);
    else
      hipLaunchKernelGGL(tbl == 0 ? k_wire_unpack_batch<0> : k_wire_unpack_batch<1>, grid, block, 0, s, B);
    if (int e = check_launch(pack ? "k_wire_pack_batch" : "k_wire_unpack_batch")) return e;
  }
  return HIC_OK;
}
}  // namespace

extern "C" int hic_wire_pack_batch(int n, const hic_wire_job *jobs, void *stream) {
  return wire_batch(n, jobs, true, stream);
}

extern "C" int hic_wire_unpack_batch(int n, const hic_wire_job *jobs, void *stream) {
  return wire_batch(n, jobs, false, stream);
}

extern "C" int hic_wire_flags_apply(int n, const hic_wire_job *jobs, void *stream) {
  WireBatch all, tb[2];
  int64_t maxrec;
  if (int e = wire_tables(n, jobs, false, all, tb, maxrec)) return e;
  hipLaunchKernelGGL(k_wire_flags_apply, dim3(1), dim3(64), 0, as_stream(stream), all);
  return check_launch("k_wire_flags_apply");
}

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
