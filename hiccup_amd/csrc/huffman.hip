// huffman.hip -- the device half of hiccup's Huffman back end:
// the key histograms codec.jpeg_encode builds its nine trees from, and the bit
// packing of the coded streams.  The trees themselves (a heapq over at most a few
// thousand leaves, hiccup/huffman.py:11-58) stay on the host.
//
// Reference: codec.jpeg_encode (codec.py:304-334): huffman.HuffmanTree.
// construct_from_data(stream) = utils.group_by (keys in FIRST-APPEARANCE order,
// huffman.py:20-28 / utils.py:31-39: the tree's tie order depends on it) + counts;
// encode_data = the concatenated '0'/'1' codes (huffman.py:131-142); the
// container stores them MSB-first behind a pad-length byte (iohelper.py:35-56).
//
//  hic_key_range      min / max of a key stream (int8/16/32)
//  hic_key_histogram  per key in [key_min, key_min + nbins): count and the index of
//                     its first appearance (LDS-privatised: 4 B count + 4 B index
//                     per bin, nbins <= 8192; global atomics beyond)
//  hic_huffman_pack   per symbol its code (host table, <= 64 bits); tiles of 4096
//                     symbols assemble their bits in LDS (atomic OR into 32-bit
//                     words, MSB-first), interior words are stored, the two edge
//                     words shared with neighbouring tiles OR-ed in; *d_nbits = total
//                     bits (words past out_bytes are not written: the caller sizes
//                     the buffer from the histogram, sum of count x code length)
#include "hic_common.h"

namespace hic {
namespace {

constexpr int kHT = 256;                  // threads per workgroup
constexpr int kHPT = 16;                  // symbols per thread
constexpr int kHTile = kHT * kHPT;        // symbols per tile
constexpr int kHistLds = 8192;            // bins held in LDS

__device__ __forceinline__ int key_at(const void *keys, int kb, int64_t i) {
  if (kb == 1) return (int)static_cast<const uint8_t *>(keys)[i];
  if (kb == 2) return (int)static_cast<const int16_t *>(keys)[i];
  return static_cast<const int32_t *>(keys)[i];
}

// min / max of the keys; keys at a 16-byte aligned address are read 16 bytes per
// load (the 8K jpeg_encode's nine streams: ~105 us per large stream read one key per
// load, 1- and 2-byte keys included)
template <int KB, bool VEC>
__global__ __launch_bounds__(kHT) void k_key_range(const void *__restrict__ keys, int64_t n, int *__restrict__ mm) {
  int lo = 2147483647, hi = -2147483647 - 1;
  const int64_t t0 = (int64_t)blockIdx.x * kHT + threadIdx.x, stride = (int64_t)gridDim.x * kHT;
  int64_t tail = 0;
  if constexpr (VEC) {
    constexpr int kPer = 16 / KB;  // keys per 16-byte load
    const uint4 *v = static_cast<const uint4 *>(keys);
    const int64_t nv = n / kPer;
    for (int64_t i = t0; i < nv; i += stride) {
      const uint4 q = v[i];
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if constexpr (KB == 4) {
          lo = min(lo, (int)w[c]);
          hi = max(hi, (int)w[c]);
        } else if constexpr (KB == 2) {
          const int a = (int)(int16_t)(w[c] & 0xFFFFu), b = (int)(int16_t)(w[c] >> 16);
          lo = min(lo, min(a, b));
          hi = max(hi, max(a, b));
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int a = (int)((w[c] >> (8 * k)) & 0xFFu);
            lo = min(lo, a);
            hi = max(hi, a);
          }
        }
      }
    }
    tail = nv * kPer;
  }
  for (int64_t i = tail + t0; i < n; i += stride) {
    const int k = key_at(keys, KB, i);
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int a = __shfl_xor(lo, d, 64), b = __shfl_xor(hi, d, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  // one atomic pair per workgroup: thousands on one address serialise in the L2
  // (~100 us per large stream with one pair per wave)
  __shared__ int s_lo[kHT / 64], s_hi[kHT / 64];
  if ((threadIdx.x & 63) == 0) {
    s_lo[threadIdx.x >> 6] = lo;
    s_hi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < kHT / 64; ++w) {
      lo = s_lo[w] < lo ? s_lo[w] : lo;
      hi = s_hi[w] > hi ? s_hi[w] : hi;
    }
    atomicMin(mm, lo);
    atomicMax(mm + 1, hi);
  }
}

// counts / first: nbins entries, zero / 0xFFFFFFFF initialised by the launcher
// LDS: privatised bins; with `part` each workgroup stores its bins (count, first) to
// part[blockIdx.x] and k_hist_reduce sums them -- per-workgroup global atomics on
// every bin (512 workgroups x thousands of bins) took ~55 us per large stream
template <bool LDS>
__global__ __launch_bounds__(kHT) void k_key_hist(const void *__restrict__ keys, int kb, int64_t n, int key_min,
                                                  int nbins, uint32_t *__restrict__ counts,
                                                  uint32_t *__restrict__ first, uint32_t *__restrict__ part = nullptr) {
  __shared__ uint32_t s_cnt[LDS ? kHistLds : 1], s_first[LDS ? kHistLds : 1];
  if (LDS) {
    for (int b = threadIdx.x; b < nbins; b += kHT) {
      s_cnt[b] = 0;
      s_first[b] = 0xFFFFFFFFu;
    }
    __syncthreads();
  }
  for (int64_t i = (int64_t)blockIdx.x * kHT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kHT) {
    const int b = key_at(keys, kb, i) - key_min;
    if ((unsigned)b >= (unsigned)nbins) continue;  // outside the caller's range: not counted
    if (LDS) {
      atomicAdd(&s_cnt[b], 1u);
      // a bin's first index is found early and a thread's i only grows: read before
      // the atomic (it may miss a smaller value in flight; the atomic then keeps the min)
      if ((uint32_t)i < s_first[b]) atomicMin(&s_first[b], (uint32_t)i);
    } else {
      atomicAdd(&counts[b], 1u);
      atomicMin(&first[b], (uint32_t)i);
    }
  }
  if (LDS) {
    __syncthreads();
    if (part) {
      uint32_t *pc = part + (int64_t)blockIdx.x * 2 * nbins;
      for (int b = threadIdx.x; b < nbins; b += kHT) {
        pc[b] = s_cnt[b];
        pc[nbins + b] = s_first[b];
      }
      return;
    }
    for (int b = threadIdx.x; b < nbins; b += kHT) {
      if (s_cnt[b]) {
        atomicAdd(&counts[b], s_cnt[b]);
        atomicMin(&first[b], s_first[b]);
      }
    }
  }
}

// counts[b] / first[b] = the sum / min of the nwg workgroups' partial bins
__global__ __launch_bounds__(kHT) void k_hist_reduce(const uint32_t *__restrict__ part, int nwg, int nbins,
                                                     uint32_t *__restrict__ counts, uint32_t *__restrict__ first) {
  const int b = blockIdx.x * kHT + threadIdx.x;
  if (b >= nbins) return;
  uint32_t c = 0, f = 0xFFFFFFFFu;
  for (int w = 0; w < nwg; ++w) {
    const uint32_t *pc = part + (int64_t)w * 2 * nbins;
    c += pc[b];
    f = pc[nbins + b] < f ? pc[nbins + b] : f;
  }
  counts[b] = c;
  first[b] = f;
}

// block-wide exclusive sum (256 threads = 4 waves)
__device__ __forceinline__ int64_t blk_excl_sum(int64_t v, int64_t *s_w, int64_t &total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = __shfl_up(x, d, 64);
    if (lane >= d) x += o;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  int64_t pre = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < kHT / 64; ++k) {
    pre += k < wv ? s_w[k] : 0;
    total += s_w[k];
  }
  __syncthreads();
  return pre + x - v;
}

// pass A: bits per tile
__global__ __launch_bounds__(kHT) void k_pack_sizes(const void *__restrict__ keys, int kb, int64_t n, int key_min,
                                                    int nbins, const uint8_t *__restrict__ code_len,
                                                    int64_t *__restrict__ tile_bits) {
  __shared__ int64_t s_w[kHT / 64];
  const int64_t s0 = (int64_t)blockIdx.x * kHTile + (int64_t)threadIdx.x * kHPT;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < kHPT; ++k)
    if (s0 + k < n) {
      const int b = key_at(keys, kb, s0 + k) - key_min;
      acc += (unsigned)b < (unsigned)nbins ? code_len[b] : 0;  // a key outside the table codes to nothing
    }
  int64_t total;
  blk_excl_sum(acc, s_w, total);
  if (threadIdx.x == 0) tile_bits[blockIdx.x] = total;
}

// in-place exclusive scan of n int64 by one workgroup; *total = the sum
__global__ __launch_bounds__(kHT) void k_pack_scan(int64_t *__restrict__ v, int64_t n, int64_t *__restrict__ total) {
  __shared__ int64_t s_w[kHT / 64];
  int64_t run = 0;
  for (int64_t c0 = 0; c0 < n; c0 += kHT) {
    const int64_t i = c0 + threadIdx.x;
    const int64_t x = i < n ? v[i] : 0;
    int64_t tot;
    const int64_t e = run + blk_excl_sum(x, s_w, tot);
    if (i < n) v[i] = e;
    run += tot;
  }
  if (threadIdx.x == 0) *total = run;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// pass B: each tile ORs its codes into an LDS word window (MSB-first), then writes
// the window: interior words stored (byte-swapped so memory is MSB-first bytes),
// the first / last word OR-ed atomically (shared with the neighbouring tiles).
// out must be zeroed; its words are big-endian bit runs.
constexpr int kPackWords = kHTile * 64 / 32 + 2;  // 64-bit codes at most
__global__ __launch_bounds__(kHT) void k_pack_bits(const void *__restrict__ keys, int kb, int64_t n, int key_min,
                                                   int nbins, const uint64_t *__restrict__ code_bits,
                                                   const uint8_t *__restrict__ code_len,
                                                   const int64_t *__restrict__ tile_off, uint32_t *__restrict__ out,
                                                   int64_t out_words) {
  extern __shared__ uint32_t s_words[];
  __shared__ int64_t s_w[kHT / 64];
  const int64_t s0 = (int64_t)blockIdx.x * kHTile + (int64_t)threadIdx.x * kHPT;
  int ks[kHPT];
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < kHPT; ++k) {
    ks[k] = s0 + k < n ? key_at(keys, kb, s0 + k) - key_min : -1;
    if ((unsigned)ks[k] >= (unsigned)nbins) ks[k] = -1;
    acc += ks[k] >= 0 ? code_len[ks[k]] : 0;
  }
  int64_t tile_total;
  const int64_t my = blk_excl_sum(acc, s_w, tile_total);
  const int64_t B0 = tile_off[blockIdx.x];      // the tile's first bit
  const int64_t w0 = B0 >> 5;                    // its first (global) word
  const int nwords = (int)(((B0 + tile_total + 31) >> 5) - w0);
  for (int i = threadIdx.x; i < nwords; i += kHT) s_words[i] = 0;
  __syncthreads();
  int64_t p = (B0 & 31) + my;  // bit position inside the window
#pragma unroll
  for (int k = 0; k < kHPT; ++k) {
    if (ks[k] < 0) continue;
    const int len = code_len[ks[k]];
    const uint64_t c = code_bits[ks[k]];
    // bits c[len-1 .. 0] go to window bits p .. p + len - 1 (MSB-first)
    int rem = len;
    int64_t q = p;
    while (rem > 0) {
      const int wi = (int)(q >> 5), off = (int)(q & 31);
      const int take = 32 - off < rem ? 32 - off : rem;
      const uint32_t piece = (uint32_t)((c >> (rem - take)) & ((take == 32) ? 0xFFFFFFFFull : ((1ull << take) - 1)));
      atomicOr(&s_words[wi], piece << (32 - off - take));
      rem -= take;
      q += take;
    }
    p += len;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nwords; i += kHT) {
    const uint32_t v = bswap32(s_words[i]);
    if (w0 + i >= out_words) break;  // buffer too small: *d_nbits tells the caller
    if ((i == 0 || i == nwords - 1)) {
      if (v) atomicOr(&out[w0 + i], v);
    } else {
      out[w0 + i] = v;
    }
  }
}

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" int hic_key_range(const void *keys, int key_bytes, int64_t n, int32_t *d_minmax, void *stream) {
  if (!keys || !d_minmax) return arg_error("null pointer");
  if (key_bytes != 1 && key_bytes != 2 && key_bytes != 4) return arg_error("key_bytes must be 1, 2 or 4");
  if (n <= 0) return arg_error("n");
  hipStream_t s = as_stream(stream);
  const int32_t init[2] = {2147483647, -2147483647 - 1};
  if (int e = hip_status(hipMemcpyAsync(d_minmax, init, sizeof init, hipMemcpyHostToDevice, s), "hipMemcpyAsync"))
    return e;
  const bool vec = reinterpret_cast<uintptr_t>(keys) % 16 == 0;
  const int per = vec ? 16 / key_bytes : 1;
  const int64_t want = (n + (int64_t)per * kHT - 1) / ((int64_t)per * kHT);
  const int grid = (int)(want < cu_count() ? want : cu_count());
  if (vec && key_bytes == 4)
    hipLaunchKernelGGL((k_key_range<4, true>), dim3(grid), dim3(kHT), 0, s, keys, n, d_minmax);
  else if (vec && key_bytes == 2)
    hipLaunchKernelGGL((k_key_range<2, true>), dim3(grid), dim3(kHT), 0, s, keys, n, d_minmax);
  else if (vec)
    hipLaunchKernelGGL((k_key_range<1, true>), dim3(grid), dim3(kHT), 0, s, keys, n, d_minmax);
  else if (key_bytes == 4)
    hipLaunchKernelGGL((k_key_range<4, false>), dim3(grid), dim3(kHT), 0, s, keys, n, d_minmax);
  else if (key_bytes == 2)
    hipLaunchKernelGGL((k_key_range<2, false>), dim3(grid), dim3(kHT), 0, s, keys, n, d_minmax);
  else
    hipLaunchKernelGGL((k_key_range<1, false>), dim3(grid), dim3(kHT), 0, s, keys, n, d_minmax);
  return check_launch("k_key_range");
}

extern "C" int hic_key_histogram(const void *keys, int key_bytes, int64_t n, int32_t key_min, int32_t nbins,
                                 uint32_t *d_counts, uint32_t *d_first, void *stream) {
  if (!keys || !d_counts || !d_first) return arg_error("null pointer");
  if (key_bytes != 1 && key_bytes != 2 && key_bytes != 4) return arg_error("key_bytes must be 1, 2 or 4");
  if (n <= 0 || n >= ((int64_t)1 << 32)) return arg_error("n");
  if (nbins < 1 || nbins > (1 << 24)) return arg_error("nbins");
  hipStream_t s = as_stream(stream);
  if (int e = hip_status(hipMemsetAsync(d_counts, 0, (size_t)nbins * 4, s), "hipMemsetAsync")) return e;
  if (int e = hip_status(hipMemsetAsync(d_first, 0xFF, (size_t)nbins * 4, s), "hipMemsetAsync")) return e;
  const int64_t want = (n + kHT * 8 - 1) / (kHT * 8);
  const int grid = (int)(want < 2 * cu_count() ? want : 2 * cu_count());
  if (nbins <= kHistLds && grid > 1) {
    // two phases: per-workgroup bins to a stream-ordered scratch, then one reduction
    void *part = nullptr;
    if (int e = hip_status(hipMallocAsync(&part, (size_t)grid * 2 * nbins * 4, s), "hipMallocAsync")) return e;
    hipLaunchKernelGGL(k_key_hist<true>, dim3(grid), dim3(kHT), 0, s, keys, key_bytes, n, key_min, nbins, d_counts,
                       d_first, static_cast<uint32_t *>(part));
    if (int e = check_launch("k_key_hist")) return e;
    hipLaunchKernelGGL(k_hist_reduce, dim3((unsigned)((nbins + kHT - 1) / kHT)), dim3(kHT), 0, s,
                       static_cast<const uint32_t *>(part), grid, nbins, d_counts, d_first);
    if (int e = check_launch("k_hist_reduce")) return e;
    return hip_status(hipFreeAsync(part, s), "hipFreeAsync");
  }
  if (nbins <= kHistLds)
    hipLaunchKernelGGL(k_key_hist<true>, dim3(grid), dim3(kHT), 0, s, keys, key_bytes, n, key_min, nbins, d_counts,
                       d_first);
  else
    hipLaunchKernelGGL(k_key_hist<false>, dim3(grid), dim3(kHT), 0, s, keys, key_bytes, n, key_min, nbins, d_counts,
                       d_first);
  return check_launch("k_key_hist");
}

extern "C" size_t hic_huffman_pack_workspace_bytes(int64_t n) {
  return (size_t)((n + kHTile - 1) / kHTile + 8) * sizeof(int64_t);
}

extern "C" int hic_huffman_pack(const void *keys, int key_bytes, int64_t n, int32_t key_min, int32_t nbins,
                                const uint64_t *d_code_bits, const uint8_t *d_code_len, uint8_t *out,
                                int64_t out_bytes, int64_t *d_nbits, void *workspace, void *stream) {
  if (!keys || !d_code_bits || !d_code_len || !out || !d_nbits || !workspace) return arg_error("null pointer");
  if (key_bytes != 1 && key_bytes != 2 && key_bytes != 4) return arg_error("key_bytes must be 1, 2 or 4");
  if (n <= 0) return arg_error("n");
  if (nbins < 1) return arg_error("nbins");
  if (reinterpret_cast<uintptr_t>(out) % 4 || out_bytes % 4 || out_bytes <= 0)
    return arg_error("out must be 4-byte aligned and sized");
  hipStream_t s = as_stream(stream);
  const int64_t nt = (n + kHTile - 1) / kHTile;
  int64_t *tile = static_cast<int64_t *>(workspace);
  if (int e = hip_status(hipMemsetAsync(out, 0, (size_t)out_bytes, s), "hipMemsetAsync")) return e;
  hipLaunchKernelGGL(k_pack_sizes, dim3((unsigned)nt), dim3(kHT), 0, s, keys, key_bytes, n, key_min, nbins,
                     d_code_len, tile);
  hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(kHT), 0, s, tile, nt, d_nbits);
  hipLaunchKernelGGL(k_pack_bits, dim3((unsigned)nt), dim3(kHT), kPackWords * sizeof(uint32_t), s, keys, key_bytes,
                     n, key_min, nbins, d_code_bits, d_code_len, tile, reinterpret_cast<uint32_t *>(out),
                     out_bytes / 4);
  return check_launch("k_pack_bits");
}
