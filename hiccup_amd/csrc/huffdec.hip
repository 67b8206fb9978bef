// huffdec.hip -- Huffman decode of a packed bit stream on the GPU: the inverse of
// hic_huffman_pack, i.e. HuffmanTree.decode_data (hiccup/huffman.py:149-178) over
// the bit strings codec.jpeg_decode reads from the .hic payloads (codec.py:372-388).
//
// The reference walks the tree one bit at a time ('1' = left, '0' = right), emits
// a leaf's value and restarts at the root; trailing bits that do not finish a code
// are dropped, and a step into a missing child (a one-leaf encoding tree's empty
// right side) raises.  The stream has no markers, so it is cut into fixed
// subsequences of g.sub bits (kSub = 256; with equal-length codes of L bits the
// multiple of L at or above it, so every subsequence starts on a codeword), one
// per thread, decoded speculatively from their nominal first bit; Huffman codes
// resynchronise within a few codewords, so after the exit bit of subsequence i is
// handed to i+1 and only changed subsequences re-decode (a handful of rounds,
// checked kRoundsPerSync at a time), every subsequence starts on a codeword boundary.
// A prefix sum over the per-subsequence symbol counts then places each one's
// output and a second decode writes the symbols.
//
//   tree:  child[2n] / child[2n+1] = node n's '1' / '0' child: >= 0 an internal
//          node, -1 missing, <= -2 leaf (-2 - leaf index); node 0 is the root
//   LUT:   the first kLutBits bits from the root: 4096 entries held in LDS,
//          [3:0] bits consumed - 1, [5:4] kind (0 leaf reached, 1 still internal
//          after kLutBits bits, 2 missing child), [31:8] leaf / node index
//   codes longer than kLutBits finish with a bit walk over child[] (global)
#include <vector>

#include "hic_common.h"

namespace hic {
namespace {

constexpr int kLutBits = 12, kLut = 1 << kLutBits;
// bits per subsequence (one thread each), at least.  256: the nine streams of an 8K
// jpeg_decode decode in 5.0-5.4 ms with the host upload, against 6.6 at 512 and 8.9
// at 1024 (more threads, shorter serial chains; 128 and 64 measured the same or
// slower: profiles/r06/huffdec/)
constexpr int kSub = 256;
constexpr int kDT = 256;        // threads per workgroup
constexpr int kMaxRounds = 24;  // resynchronisation rounds before the serial chain
constexpr int kRoundsPerSync = 4;  // rounds launched between two host reads of their flags
constexpr int64_t kEnd = INT64_MAX;  // exit of a subsequence that reached the stream end

enum : uint32_t { kLeaf = 0, kNode = 1, kMissing = 2 };

// 64-bit MSB-aligned window over big-endian 32-bit words (the stream's bytes are
// MSB-first); words past the buffer read as zero.
struct BitReader {
  const uint32_t *w;
  int64_t nwords, wi;
  uint64_t acc;
  int nacc;
  // the workgroup's words [lw0, lw0 + lwn), byte-swapped, in LDS (lwn = 0: none):
  // a thread's refills are then LDS reads, not a chain of dependent global loads
  const uint32_t *lw = nullptr;
  int64_t lw0 = 0, lwn = 0;
  __device__ uint32_t load(int64_t i) const {
    if ((uint64_t)(i - lw0) < (uint64_t)lwn) return lw[i - lw0];
    return i < nwords ? __builtin_bswap32(w[i]) : 0u;
  }
  __device__ void refill() {
    if (nacc <= 32) {
      acc |= (uint64_t)load(wi++) << (32 - nacc);
      nacc += 32;
    }
  }
  __device__ void init(const uint32_t *words, int64_t nw, int64_t p) {
    w = words;
    nwords = nw;
    wi = p >> 5;
    const int off = (int)(p & 31);
    acc = (uint64_t)load(wi++) << (32 + off);
    nacc = 32 - off;
    refill();
  }
  __device__ uint32_t peek(int k) const { return (uint32_t)(acc >> (64 - k)); }
  __device__ void skip(int k) {
    acc <<= k;
    nacc -= k;
    refill();
  }
};

// One symbol at bit p: 0 decoded (sym = leaf index), 1 stream end (no complete
// code before nbits), 2 missing child (the reference's AttributeError).
__device__ __forceinline__ int next_symbol(BitReader &br, int64_t &p, int64_t nbits, const uint32_t *lut,
                                           const int32_t *__restrict__ child, int &sym) {
  if (p >= nbits) return 1;
  const uint32_t e = lut[br.peek(kLutBits)];
  const int len = (int)(e & 15) + 1;
  const uint32_t kind = (e >> 4) & 3;
  if (kind == kLeaf) {
    if (p + len > nbits) return 1;
    br.skip(len);
    p += len;
    sym = (int)(e >> 8);
    return 0;
  }
  if (kind == kMissing) return p + len > nbits ? 1 : 2;
  if (p + kLutBits > nbits) return 1;
  br.skip(kLutBits);
  p += kLutBits;
  int node = (int)(e >> 8);
  for (;;) {
    if (p >= nbits) return 1;
    const int c = child[2 * node + 1 - (int)br.peek(1)];
    if (c == -1) return 2;
    br.skip(1);
    ++p;
    if (c < 0) {
      sym = -2 - c;
      return 0;
    }
    node = c;
  }
}

struct DecGeo {
  const uint32_t *words;
  int64_t nwords, nbits, nsub, sub;  // sub: bits per subsequence
  const uint32_t *lut;  // global copy (the kernels stage it in LDS)
  const int32_t *child;
};

// Symbols starting in [start, end): count and the first codeword start >= end
// (kEnd at the stream end or after a missing child: nothing follows).
struct LdsWords {  // a workgroup's staged words (n = 0: read global memory)
  const uint32_t *w;
  int64_t w0, n;
};

__device__ void count_sub(const DecGeo &g, const uint32_t *lut, int64_t start, int64_t end, int64_t &exit,
                          int32_t &count, LdsWords lw = LdsWords{nullptr, 0, 0}) {
  count = 0;
  exit = start;
  if (start >= end) return;
  BitReader br;
  br.lw = lw.w;
  br.lw0 = lw.w0;
  br.lwn = lw.n;
  br.init(g.words, g.nwords, start);
  int64_t p = start;
  int sym;
  while (p < end) {
    if (next_symbol(br, p, g.nbits, lut, g.child, sym) != 0) {
      exit = kEnd;
      return;
    }
    ++count;
  }
  exit = p;
}

__device__ void stage_lut(const uint32_t *__restrict__ lut, uint32_t *s_lut) {
  for (int i = threadIdx.x; i < kLut; i += kDT) s_lut[i] = lut[i];
  __syncthreads();
}

// The words this workgroup's subsequences read -- bits [b kDT sub, (b + 1) kDT sub)
// and a margin for the codes that run past the last one -- staged in LDS by
// coalesced loads (a subsequence is at most kSub + 23 bits: kSub, or a multiple of
// an equal code length L <= 24 at or above it); measured: 5.0-5.2 vs 5.5 ms for the
// nine 8K streams reading global memory directly (profiles/r06/huffdec/)
constexpr int kWinMargin = 64;  // words past the workgroup's bits (codes up to 2048 bits)
constexpr int kWinWords = kDT * (kSub + 23) / 32 + 2 + kWinMargin;
__device__ LdsWords stage_words(const DecGeo &g, uint32_t *s_w) {
  const int64_t b0 = (int64_t)blockIdx.x * kDT * g.sub;
  const int64_t w0 = b0 >> 5;
  int64_t n = ((b0 + (int64_t)kDT * g.sub + 31) >> 5) + kWinMargin - w0;
  if (n > kWinWords) n = kWinWords;
  for (int64_t k = threadIdx.x; k < n; k += kDT) s_w[k] = w0 + k < g.nwords ? __builtin_bswap32(g.words[w0 + k]) : 0u;
  __syncthreads();
  return LdsWords{s_w, w0, n};
}

// round 0: every subsequence from its nominal first bit
__global__ __launch_bounds__(kDT) void k_hd_count(DecGeo g, int64_t *__restrict__ start, int64_t *__restrict__ exit,
                                                  int32_t *__restrict__ cnt) {
  __shared__ uint32_t s_lut[kLut];
  __shared__ uint32_t s_win[kWinWords];
  stage_lut(g.lut, s_lut);
  const LdsWords lw = stage_words(g, s_win);
  const int64_t i = (int64_t)blockIdx.x * kDT + threadIdx.x;
  if (i >= g.nsub) return;
  int64_t e;
  int32_t c;
  count_sub(g, s_lut, i * g.sub, (i + 1) * g.sub, e, c, lw);
  start[i] = i * g.sub;
  exit[i] = e;
  cnt[i] = c;
}

// one resynchronisation round: subsequence i starts where i-1 exited last round
__global__ __launch_bounds__(kDT) void k_hd_sync(DecGeo g, int64_t *__restrict__ start,
                                                 const int64_t *__restrict__ exit_in, int64_t *__restrict__ exit_out,
                                                 int32_t *__restrict__ cnt, int32_t *__restrict__ changed) {
  __shared__ uint32_t s_lut[kLut];
  __shared__ uint32_t s_win[kWinWords];
  const int64_t i = (int64_t)blockIdx.x * kDT + threadIdx.x;
  int64_t s = 0;
  bool redo = false;
  if (i < g.nsub) {
    s = i == 0 ? 0 : exit_in[i - 1];
    redo = s != start[i];
    if (!redo) exit_out[i] = exit_in[i];
  }
  if (!__syncthreads_or(redo)) return;  // workgroup-uniform: nothing to re-decode here
  stage_lut(g.lut, s_lut);
  const LdsWords lw = stage_words(g, s_win);
  if (!redo) return;
  int64_t e;
  int32_t c;
  count_sub(g, s_lut, s, (i + 1) * g.sub, e, c, lw);
  start[i] = s;
  exit_out[i] = e;
  cnt[i] = c;
  *changed = 1;
}

// the serial chain for streams that do not resynchronise (e.g. equal-length codes
// whose length does not divide kSub): one thread walks the boundaries in order
__global__ void k_hd_chain(DecGeo g, int64_t *__restrict__ start, int64_t *__restrict__ exit,
                           int32_t *__restrict__ cnt) {
  for (int64_t i = 1; i < g.nsub; ++i) {
    const int64_t s = exit[i - 1];
    if (s == start[i]) continue;
    int64_t e;
    int32_t c;
    count_sub(g, g.lut, s, (i + 1) * g.sub, e, c);
    start[i] = s;
    exit[i] = e;
    cnt[i] = c;
  }
}

__device__ __forceinline__ int64_t blk_excl(int64_t v, int64_t *s_w, int64_t &total) {
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
  for (int k = 0; k < kDT / 64; ++k) {
    pre += k < wv ? s_w[k] : 0;
    total += s_w[k];
  }
  __syncthreads();
  return pre + x - v;
}

__global__ __launch_bounds__(kDT) void k_hd_bsum(const int32_t *__restrict__ cnt, int64_t nsub,
                                                 int64_t *__restrict__ bsum) {
  __shared__ int64_t s_w[kDT / 64];
  const int64_t i = (int64_t)blockIdx.x * kDT + threadIdx.x;
  int64_t tot;
  blk_excl(i < nsub ? cnt[i] : 0, s_w, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// in-place exclusive scan of n int64 by one workgroup; *total = the sum
__global__ __launch_bounds__(kDT) void k_hd_scan(int64_t *__restrict__ v, int64_t n, int64_t *__restrict__ total) {
  __shared__ int64_t s_w[kDT / 64];
  int64_t run = 0;
  for (int64_t c0 = 0; c0 < n; c0 += kDT) {
    const int64_t i = c0 + threadIdx.x;
    const int64_t x = i < n ? v[i] : 0;
    int64_t tot;
    const int64_t e = run + blk_excl(x, s_w, tot);
    if (i < n) v[i] = e;
    run += tot;
  }
  if (threadIdx.x == 0) *total = run;
}

// the output pass: symbols of subsequence i at its offset, as leaf values (or
// leaf indices when values is null); err = the first bit of a symbol that walks
// into a missing child (min over the stream)
__global__ __launch_bounds__(kDT) void k_hd_emit(DecGeo g, const int64_t *__restrict__ start,
                                                 const int32_t *__restrict__ cnt, const int64_t *__restrict__ boff,
                                                 const int32_t *__restrict__ values, int32_t *__restrict__ out,
                                                 int64_t out_cap, unsigned long long *__restrict__ err) {
  __shared__ uint32_t s_lut[kLut];
  __shared__ uint32_t s_win[kWinWords];
  __shared__ int64_t s_w[kDT / 64];
  stage_lut(g.lut, s_lut);
  const LdsWords lw = stage_words(g, s_win);
  const int64_t i = (int64_t)blockIdx.x * kDT + threadIdx.x;
  int64_t tot;
  const int64_t o = boff[blockIdx.x] + blk_excl(i < g.nsub ? cnt[i] : 0, s_w, tot);
  if (i >= g.nsub) return;
  const int64_t s = start[i], end = (i + 1) * g.sub;
  if (s >= end) return;
  BitReader br;
  br.lw = lw.w;
  br.lw0 = lw.w0;
  br.lwn = lw.n;
  br.init(g.words, g.nwords, s);
  int64_t p = s, k = o;
  int sym;
  while (p < end) {
    const int64_t at = p;
    const int r = next_symbol(br, p, g.nbits, s_lut, g.child, sym);
    if (r == 2) atomicMin(err, (unsigned long long)at);
    if (r != 0) break;
    if (k < out_cap) out[k] = values ? values[sym] : sym;
    ++k;
  }
}

struct DecWs {
  uint32_t *lut;
  int32_t *child, *values, *cnt, *changed;
  int64_t *start, *exit_a, *exit_b, *bsum, *total;
  unsigned long long *err;
};

DecWs carve(void *ws, int64_t nsub, int32_t nnodes, int32_t nleaves) {
  char *p = static_cast<char *>(ws);
  auto take = [&](size_t bytes) {
    char *q = p;
    p += round_up((int64_t)bytes, 256);
    return q;
  };
  DecWs w;
  const int64_t nblk = ceil_div(nsub, kDT);
  w.lut = reinterpret_cast<uint32_t *>(take(kLut * 4));
  w.child = reinterpret_cast<int32_t *>(take((size_t)2 * nnodes * 4));
  w.values = reinterpret_cast<int32_t *>(take((size_t)(nleaves > 0 ? nleaves : 1) * 4));
  w.start = reinterpret_cast<int64_t *>(take((size_t)nsub * 8));
  w.exit_a = reinterpret_cast<int64_t *>(take((size_t)nsub * 8));
  w.exit_b = reinterpret_cast<int64_t *>(take((size_t)nsub * 8));
  w.cnt = reinterpret_cast<int32_t *>(take((size_t)nsub * 4));
  w.bsum = reinterpret_cast<int64_t *>(take((size_t)(nblk + 1) * 8));
  w.total = reinterpret_cast<int64_t *>(take(16));  // {symbols, first error bit}: one read back
  w.err = reinterpret_cast<unsigned long long *>(w.total + 1);
  w.changed = reinterpret_cast<int32_t *>(take(4 * kRoundsPerSync));
  return w;
}

}  // namespace
}  // namespace hic

using namespace hic;

extern "C" size_t hic_huffman_decode_workspace_bytes(int64_t nbits, int32_t nnodes, int32_t nleaves) {
  if (nbits < 0 || nnodes < 0 || nleaves < 0) return 0;
  const int64_t nsub = ceil_div(nbits, kSub) > 0 ? ceil_div(nbits, kSub) : 1;
  const int64_t nblk = ceil_div(nsub, kDT);
  const int64_t r = 256;
  return (size_t)(round_up(kLut * 4, r) + round_up(2LL * nnodes * 4, r) + round_up((nleaves > 0 ? nleaves : 1) * 4LL, r) +
                  3 * round_up(nsub * 8, r) + round_up(nsub * 4, r) + round_up((nblk + 1) * 8, r) + 3 * r);
}

namespace {
// one stream's host-side state through the batch's phases
struct DecState {
  std::vector<uint32_t> lut;
  DecGeo g;
  DecWs w;
  dim3 grid;
  int64_t *ein, *eout;
  bool synced;
  int32_t changed[kRoundsPerSync];
  int64_t host[2];  // {symbols, first error bit} read back
};

// validation, the lookup table and the subsequence length of one job (no device work)
int decode_prepare(const hic_huffman_decode_job &j, DecState &st) {
  const int32_t nnodes = j.nnodes, nleaves = j.nleaves;
  const int32_t *h_child = j.h_child;
  if (!h_child || !j.workspace || (j.nbits > 0 && (!j.d_bits || !j.d_out))) return arg_error("null pointer");
  if (j.nbits < 0 || j.out_cap < 0) return arg_error("nbits / out_cap");
  if (reinterpret_cast<uintptr_t>(j.d_bits) % 4) return arg_error("d_bits must be 4-byte aligned");
  if (nnodes < 1 || nnodes >= (1 << 24) || nleaves < 1 || nleaves >= (1 << 24))
    return arg_error("tree size (1 <= nodes, leaves < 2^24)");
  // a tree: indices in range, every node but the root the child of exactly one node
  std::vector<uint8_t> seen((size_t)nnodes + nleaves, 0);
  for (int64_t k = 0; k < 2LL * nnodes; ++k) {
    const int32_t c = h_child[k];
    if (c == -1) continue;
    const int64_t slot = c >= 0 ? c : (int64_t)nnodes + (-2 - (int64_t)c);
    if ((c >= 0 && (c == 0 || c >= nnodes)) || (c < -1 && -2 - (int64_t)c >= nleaves) || seen[slot]++)
      return arg_error("child[%lld] = %d is not a tree edge", (long long)k, c);
  }
  // the kLutBits-bit lookup table from the root
  st.lut.assign(kLut, 0);
  for (int v = 0; v < kLut; ++v) {
    int node = 0;
    uint32_t e = ((uint32_t)(kLutBits - 1)) | (kNode << 4);
    for (int k = 0; k < kLutBits; ++k) {
      const int c = h_child[2 * node + 1 - ((v >> (kLutBits - 1 - k)) & 1)];
      if (c == -1) {
        e = (uint32_t)k | (kMissing << 4);
        break;
      }
      if (c < 0) {
        e = (uint32_t)k | (kLeaf << 4) | ((uint32_t)(-2 - c) << 8);
        break;
      }
      node = c;
      e = ((uint32_t)(kLutBits - 1)) | (kNode << 4) | ((uint32_t)node << 8);
    }
    st.lut[v] = e;
  }
  // equal-length codes (every leaf at one depth L, e.g. a near-uniform table): a
  // subsequence of a multiple of L bits starts on a codeword, so round 0 is already
  // synchronised (with kSub bits and L not dividing it the rounds may never converge)
  int64_t sub = kSub;
  {
    std::vector<int32_t> depth((size_t)nnodes, -1);
    depth[0] = 0;
    int leaf_depth = -1;
    bool equal = true;
    std::vector<int32_t> queue{0};
    for (size_t qi = 0; qi < queue.size() && equal; ++qi) {
      const int32_t n = queue[qi];
      for (int b = 0; b < 2; ++b) {
        const int32_t c = h_child[2 * n + b];
        if (c >= 0) {
          depth[c] = depth[n] + 1;
          queue.push_back(c);
        } else if (c <= -2) {
          if (leaf_depth < 0) leaf_depth = depth[n] + 1;
          equal = equal && leaf_depth == depth[n] + 1;
        }
      }
    }
    if (equal && leaf_depth > 0) sub = (int64_t)leaf_depth * ceil_div(kSub, leaf_depth);
  }
  const int64_t nsub = ceil_div(j.nbits, sub) > 0 ? ceil_div(j.nbits, sub) : 1;
  st.w = carve(j.workspace, nsub, nnodes, nleaves);
  st.g = DecGeo{reinterpret_cast<const uint32_t *>(j.d_bits), ceil_div(j.nbits, 32), j.nbits, nsub, sub, st.w.lut,
                st.w.child};
  st.grid = dim3((unsigned)ceil_div(nsub, kDT));
  st.ein = st.w.exit_a;
  st.eout = st.w.exit_b;
  st.synced = nsub == 1;
  return HIC_OK;
}
}  // namespace

// The streams of a batch go through each phase together on one HIP stream, so the
// host waits once per phase for all of them (3 waits when every stream
// resynchronises within kRoundsPerSync rounds) instead of once per phase per stream.
extern "C" int hic_huffman_decode_batch(int n, hic_huffman_decode_job *jobs, void *stream) {
  if (n < 0 || (n > 0 && !jobs)) return arg_error("jobs");
  std::vector<DecState> st((size_t)n);
  for (int i = 0; i < n; ++i) {  // every job checked before anything is queued
    jobs[i].count = 0;
    jobs[i].status = HIC_OK;
    if (int e = decode_prepare(jobs[i], st[i])) return e;
  }
  const hipStream_t s = as_stream(stream);
  bool any = false;
  for (int i = 0; i < n; ++i) {
    const hic_huffman_decode_job &j = jobs[i];
    if (j.nbits == 0) continue;
    any = true;
    DecWs &w = st[i].w;
    if (int e = hip_status(hipMemcpyAsync(w.lut, st[i].lut.data(), kLut * 4, hipMemcpyHostToDevice, s),
                           "hipMemcpyAsync"))
      return e;
    if (int e = hip_status(hipMemcpyAsync(w.child, j.h_child, (size_t)2 * j.nnodes * 4, hipMemcpyHostToDevice, s),
                           "hipMemcpyAsync"))
      return e;
    if (j.h_values)
      if (int e = hip_status(hipMemcpyAsync(w.values, j.h_values, (size_t)j.nleaves * 4, hipMemcpyHostToDevice, s),
                             "hipMemcpyAsync"))
        return e;
  }
  if (!any) return HIC_OK;
  // the host tables are locals / the caller's: wait for the uploads before anything can return
  if (int e = hip_status(hipStreamSynchronize(s), "hipStreamSynchronize")) return e;
  for (int i = 0; i < n; ++i) {
    if (jobs[i].nbits == 0) continue;
    DecState &x = st[i];
    if (int e = hip_status(hipMemsetAsync(x.w.err, 0xFF, 8, s), "hipMemsetAsync")) return e;
    hipLaunchKernelGGL(k_hd_count, x.grid, dim3(kDT), 0, s, x.g, x.w.start, x.ein, x.w.cnt);
    if (int e = check_launch("k_hd_count")) return e;
  }
  // rounds in batches of kRoundsPerSync, one host read of every stream's change flags
  // per batch: a round without a change means every later one has none either
  for (int round = 0; round < kMaxRounds; round += kRoundsPerSync) {
    bool pending = false;
    for (int i = 0; i < n; ++i) {
      DecState &x = st[i];
      if (jobs[i].nbits == 0 || x.synced) continue;
      pending = true;
      if (int e = hip_status(hipMemsetAsync(x.w.changed, 0, 4 * kRoundsPerSync, s), "hipMemsetAsync")) return e;
      for (int k = 0; k < kRoundsPerSync; ++k) {
        hipLaunchKernelGGL(k_hd_sync, x.grid, dim3(kDT), 0, s, x.g, x.w.start, x.ein, x.eout, x.w.cnt,
                           x.w.changed + k);
        if (int e = check_launch("k_hd_sync")) return e;
        std::swap(x.ein, x.eout);
      }
      if (int e = hip_status(hipMemcpyAsync(x.changed, x.w.changed, 4 * kRoundsPerSync, hipMemcpyDeviceToHost, s),
                             "hipMemcpyAsync"))
        return e;
    }
    if (!pending) break;
    if (int e = hip_status(hipStreamSynchronize(s), "hipStreamSynchronize")) return e;
    for (int i = 0; i < n; ++i) {
      DecState &x = st[i];
      if (jobs[i].nbits == 0 || x.synced) continue;
      for (int k = 0; k < kRoundsPerSync; ++k) x.synced = x.synced || x.changed[k] == 0;
    }
  }
  for (int i = 0; i < n; ++i) {
    const hic_huffman_decode_job &j = jobs[i];
    if (j.nbits == 0) continue;
    DecState &x = st[i];
    if (!x.synced) {
      hipLaunchKernelGGL(k_hd_chain, dim3(1), dim3(1), 0, s, x.g, x.w.start, x.ein, x.w.cnt);
      if (int e = check_launch("k_hd_chain")) return e;
    }
    hipLaunchKernelGGL(k_hd_bsum, x.grid, dim3(kDT), 0, s, x.w.cnt, x.g.nsub, x.w.bsum);
    hipLaunchKernelGGL(k_hd_scan, dim3(1), dim3(kDT), 0, s, x.w.bsum, (int64_t)x.grid.x, x.w.total);
    hipLaunchKernelGGL(k_hd_emit, x.grid, dim3(kDT), 0, s, x.g, x.w.start, x.w.cnt, x.w.bsum,
                       j.h_values ? x.w.values : nullptr, j.d_out, j.out_cap, x.w.err);
    if (int e = check_launch("k_hd_emit")) return e;
    if (int e = hip_status(hipMemcpyAsync(x.host, x.w.total, 16, hipMemcpyDeviceToHost, s), "hipMemcpyAsync"))
      return e;
  }
  if (int e = hip_status(hipStreamSynchronize(s), "hipStreamSynchronize")) return e;
  int first = HIC_OK;
  for (int i = 0; i < n; ++i) {
    hic_huffman_decode_job &j = jobs[i];
    if (j.nbits == 0) continue;
    const DecState &x = st[i];
    const unsigned long long err = (unsigned long long)x.host[1];
    j.count = x.host[0];  // on a missing child: the symbols before the failing one are in d_out
    if (err != ~0ULL) {
      j.status = HIC_ERR_ARG;
      if (first == HIC_OK) set_error("Huffman walk stepped into a missing child at bit %llu", err);
    } else if (x.host[0] > j.out_cap) {
      j.status = HIC_ERR_CAPACITY;
      if (first == HIC_OK) set_error("decoded %lld symbols, out_cap %lld", (long long)x.host[0], (long long)j.out_cap);
    }
    if (first == HIC_OK) first = j.status;
  }
  return first;
}

extern "C" int hic_huffman_decode(const uint8_t *d_bits, int64_t nbits, const int32_t *h_child, int32_t nnodes,
                                  const int32_t *h_values, int32_t nleaves, int32_t *d_out, int64_t out_cap,
                                  int64_t *h_count, void *workspace, void *stream) {
  if (!h_count) return arg_error("null pointer");
  hic_huffman_decode_job j{d_bits, nbits, h_child, nnodes, h_values, nleaves, d_out, out_cap, workspace, 0, 0};
  *h_count = 0;
  const int rc = hic_huffman_decode_batch(1, &j, stream);
  *h_count = j.count;
  return rc;
}
