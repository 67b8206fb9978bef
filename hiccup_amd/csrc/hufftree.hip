// hufftree.hip -- the Huffman trees of codec.jpeg_encode / jpeg_decode, built on
// the host in native code (no device code in this file).  The GPU side of the
// back end (histograms, bit packing, decoding) is huffman.hip / huffdec.hip; what
// remained in Python was the trees themselves: a heapq of node objects per key
// stream (~12 ms of the 8K jpeg_encode) and a recursive rebuild from the coding
// table plus its flattening (~14 ms of jpeg_decode).
//
// hic_huffman_build restates HuffmanTree._construct (hiccup/huffman.py:60-79): the
// leaves in first-appearance order go into a binary min-heap compared on frequency
// ONLY, by heapq's own algorithm (heapify = siftup of nodes n/2-1 .. 0; heappop =
// the last item to the top, then siftup; heappush = append + siftdown; siftup walks
// the smaller child down to a leaf -- the right one unless left < right -- then
// sifts the item back up), so equal frequencies tie exactly as the reference's
// heap order breaks them.  The first node popped is the LEFT child, a left edge
// reads "1" (translate_path, huffman.py:119-129); one leaf alone is the left child
// of a singleton root: code "1".
//
// hic_huffman_from_codes restates construct_from_coding (huffman.py:30-58) for a
// complete prefix code -- what every encoder table is -- and lays the tree out as
// hic_huffman_decode takes it (breadth first, huffman.HuffmanTree.flat).  Any other
// table (a code that is a prefix of another, unused code words, an empty code,
// characters other than '0' / '1') is refused with HIC_ERR_ARG and the caller keeps
// the reference's own construction, whose None leaves / unreachable codes then
// behave as the reference's do.
#include <string.h>

#include <vector>

#include "hic_common.h"

namespace {

struct Heap {  // heapq over node ids, ordered by freq[id] (a "<" compare only)
  std::vector<int32_t> a;
  const std::vector<int64_t> &f;
  explicit Heap(const std::vector<int64_t> &freq) : f(freq) {}
  bool lt(int32_t x, int32_t y) const { return f[x] < f[y]; }
  void siftdown(size_t start, size_t pos) {
    const int32_t item = a[pos];
    while (pos > start) {
      const size_t parent = (pos - 1) >> 1;
      if (!lt(item, a[parent])) break;
      a[pos] = a[parent];
      pos = parent;
    }
    a[pos] = item;
  }
  void siftup(size_t pos) {
    const size_t end = a.size(), start = pos;
    const int32_t item = a[pos];
    size_t child = 2 * pos + 1;
    while (child < end) {
      const size_t right = child + 1;
      if (right < end && !lt(a[child], a[right])) child = right;
      a[pos] = a[child];
      pos = child;
      child = 2 * pos + 1;
    }
    a[pos] = item;
    siftdown(start, pos);
  }
  void heapify() {
    for (size_t i = a.size() / 2; i-- > 0;) siftup(i);
  }
  int32_t pop() {
    const int32_t last = a.back();
    a.pop_back();
    if (a.empty()) return last;
    const int32_t top = a[0];
    a[0] = last;
    siftup(0);
    return top;
  }
  void push(int32_t x) {
    a.push_back(x);
    siftdown(0, a.size() - 1);
  }
};

}  // namespace

// leaf i's code as text ('1' / '0' from the root, then one space): the table
// payload's strings, split by one str.split on the Python side
static void code_text(const uint8_t *len, const uint64_t *code, int64_t n, char *text) {
  for (int64_t i = 0; i < n; ++i) {
    for (int b = len[i] - 1; b >= 0; --b) *text++ = (char)('0' + ((code[i] >> b) & 1));
    *text++ = ' ';
  }
}

extern "C" int hic_huffman_build(const int64_t *h_counts, int64_t n, uint8_t *h_len, uint64_t *h_code,
                                 char *h_text) {
  if (!h_counts || !h_len || !h_code) return hic::arg_error("null pointer");
  if (n < 1 || n > (int64_t)1 << 30) return hic::arg_error("leaf count %lld", (long long)n);
  if (n == 1) {  // Node.singleton: the leaf is the root's left child
    h_len[0] = 1;
    h_code[0] = 1;
    if (h_text) code_text(h_len, h_code, 1, h_text);
    return HIC_OK;
  }
  const int64_t nodes = 2 * n - 1;
  std::vector<int64_t> freq(nodes);
  std::vector<int32_t> kid(2 * (n - 1));  // internal node n + k: left kid[2k], right kid[2k + 1]
  for (int64_t i = 0; i < n; ++i) freq[i] = h_counts[i];
  Heap h(freq);
  h.a.resize(n);
  for (int64_t i = 0; i < n; ++i) h.a[i] = (int32_t)i;
  h.heapify();
  int32_t next = (int32_t)n;
  while (h.a.size() > 1) {
    const int32_t l = h.pop(), r = h.pop();
    freq[next] = freq[l] + freq[r];
    kid[2 * (next - n)] = l;
    kid[2 * (next - n) + 1] = r;
    h.push(next++);
  }
  // codes root -> leaf (left "1"), depth first with an explicit stack
  struct Item {
    int32_t node;
    int32_t len;
    uint64_t bits;
  };
  std::vector<Item> st;
  st.push_back({h.pop(), 0, 0});
  while (!st.empty()) {
    const Item it = st.back();
    st.pop_back();
    if (it.node < n) {
      h_len[it.node] = (uint8_t)it.len;
      h_code[it.node] = it.bits;
      continue;
    }
    if (it.len >= 64) return hic::arg_error("Huffman code longer than 64 bits");
    const int32_t k = it.node - (int32_t)n;
    st.push_back({kid[2 * k], it.len + 1, it.bits << 1 | 1});
    st.push_back({kid[2 * k + 1], it.len + 1, it.bits << 1});
  }
  if (h_text) code_text(h_len, h_code, n, h_text);
  return HIC_OK;
}

extern "C" int hic_huffman_from_codes(const char *h_chars, const int64_t *h_off, int64_t n, int32_t *h_child,
                                      int32_t *h_leaf_seg, int64_t *h_nodes, int32_t *h_minlen) {
  if (!h_chars || !h_off || !h_child || !h_leaf_seg || !h_nodes || !h_minlen) return hic::arg_error("null pointer");
  if (n < 2 || n > (int64_t)1 << 30) return hic::arg_error("irregular table: %lld codes", (long long)n);
  // the code trie: node 0 the root; kid[2 i] the '1' child, kid[2 i + 1] the '0'
  // child (0 = none); seg[i] the table entry ending there (the last one with that
  // code: the reference's dict keeps the last)
  std::vector<int32_t> kid(2, 0), seg(1, -1), depth(1, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = h_off[i], b = h_off[i + 1];
    if (b <= a) return hic::arg_error("irregular table: empty code");
    int32_t v = 0;
    for (int64_t j = a; j < b; ++j) {
      const char c = h_chars[j];
      if (c != '0' && c != '1') return hic::arg_error("irregular table: code character");
      const size_t e = 2 * (size_t)v + (c == '0');
      if (kid[e] == 0) {  // a new node (its slots appended after the edge is set)
        kid[e] = (int32_t)seg.size();
        kid.push_back(0);
        kid.push_back(0);
        seg.push_back(-1);
        depth.push_back(depth[v] + 1);
      }
      v = kid[e];
    }
    seg[v] = (int32_t)i;
  }
  // complete and prefix-free: a code ends exactly at every node without children
  for (size_t v = 0; v < seg.size(); ++v) {
    const bool inner = kid[2 * v] != 0 || kid[2 * v + 1] != 0;
    if (inner ? (seg[v] >= 0 || kid[2 * v] == 0 || kid[2 * v + 1] == 0) : seg[v] < 0)
      return hic::arg_error("irregular table: not a complete prefix code");
  }
  // breadth first over the internal nodes (HuffmanTree.flat's numbering)
  std::vector<int32_t> order(1, 0);
  int32_t nleaves = 0, minlen = 1 << 30;
  for (size_t q = 0; q < order.size(); ++q) {
    const int32_t v = order[q];
    for (int side = 0; side < 2; ++side) {
      const int32_t c = kid[2 * v + side];
      if (seg[c] >= 0) {
        h_child[2 * q + side] = -2 - nleaves;
        h_leaf_seg[nleaves++] = seg[c];
        if (depth[c] < minlen) minlen = depth[c];
      } else {
        h_child[2 * q + side] = (int32_t)order.size();
        order.push_back(c);
      }
    }
  }
  *h_nodes = (int64_t)order.size();
  *h_minlen = minlen;
  return HIC_OK;
}
