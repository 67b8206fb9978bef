"""Huffman entropy back end (mirrors hiccup/huffman.py:11-259).

Host-side: SURVEY.md section 8(f) ranks the Huffman stage as the first "next"
row after the GPU front end.  The tree is built exactly as the reference does
(a ``heapq`` of nodes ordered by frequency only, leaves in first-appearance
order of the keys, the first popped node becomes the LEFT child, codes read
root -> leaf with left = "1", right = "0"; a one-symbol alphabet gets the code
"1"), so tables and bit strings are identical to the reference's
(tests/test_codec_host.py pins them against golden payloads).

Encoding is vectorised (a code lookup per distinct key, then one join) instead
of the reference's per-symbol parent walk (huffman.py:131-142).

Device half (codec.jpeg_encode's hot loops, csrc/huffman.hip): the key histogram
in first-appearance order (``device_counts``) and the bit packing of a coded
stream (``encode_device``).  The trees of codec.jpeg_encode / jpeg_decode are built
in native host code (csrc/hufftree.hip): ``CodeBook`` (the codes of the heapq tree)
and ``FlatCodes`` (the decoding tree of a coding table, in the GPU decoder's
layout).  ``HuffmanTree`` is the reference's node-object tree, kept as the
reference-shaped API and for tables the native builder refuses.
"""
import ctypes
import heapq

import numpy as np
import torch

from . import _lib, device, utils


class _Packer:
    """encode_data of a device key stream through a tree's code table (the GPU
    packer): shared by HuffmanTree and the natively built CodeBook."""

    def encode_device(self, keys_dev, n, key_min, nbins, counts, stream=None):
        """encode_data of a device key stream (uint8 / int16 / int32 tensor of n keys
        in [key_min, key_min + nbins), with counts the per-bin histogram), packed on
        the GPU: returns (packed uint8 numpy array, number of bits), MSB-first --
        the bits io.padded_bs_2_bytes stores after its pad-length byte."""
        if n == 0:
            return np.zeros(0, np.uint8), 0
        with device.on_stream(stream):
            return self._encode_device(keys_dev, n, key_min, nbins, counts, stream)

    def _encode_device(self, keys_dev, n, key_min, nbins, counts, stream):
        bits, lens = self.code_table(key_min, nbins)
        total = int(np.sum(np.asarray(counts, dtype=np.int64) * lens.astype(np.int64)))
        nbytes = max(4, -(-total // 32) * 4)
        out = device.empty((nbytes,), torch.uint8)
        nbits = device.empty((1,), torch.int64)
        ws = device.workspace(_lib.load().hic_huffman_pack_workspace_bytes(n))
        cb, cl = device.to_device(bits.view(np.int64)), device.to_device(lens)
        _lib.call("hic_huffman_pack", device.ptr(keys_dev), keys_dev.element_size(), n, key_min, nbins, device.ptr(cb),
                  device.ptr(cl), device.ptr(out), nbytes, device.ptr(nbits), device.ptr(ws),
                  device.stream_ptr(stream))
        nb = int(nbits.cpu()[0])
        if nb != total:
            raise RuntimeError("packed %d bits, the histogram says %d" % (nb, total))
        return out[:-(-nb // 8)].cpu().numpy(), nb


class HuffmanTree(_Packer):
    class Node:
        GROUND = None
        ROOT = None

        def __init__(self, left, right, value, frequency):
            self.id = id(self)
            self.parent = self.ROOT
            self.left = left
            self.right = right
            self.value = value
            self.frequency = frequency

        @classmethod
        def leaf(cls, value, frequency):
            return cls(cls.GROUND, cls.GROUND, value, frequency)

        @classmethod
        def combine(cls, l, r):
            node = cls(l, r, None, l.frequency + r.frequency)
            l.parent = node
            r.parent = node
            return node

        @classmethod
        def singleton(cls, n):
            node = cls(n, cls.GROUND, None, n.frequency)
            n.parent = node
            return node

        def path(self, nodes=None):
            nodes = [] if nodes is None else nodes
            node = self
            while True:
                nodes.append(node)
                if node.is_root:
                    return nodes
                node = node.parent

        def inherit(self, child):
            child.parent = self
            return self

        def mass_adopt(self):
            self.inherit(self.left).inherit(self.right)

        @property
        def encoding(self):
            return self.value, self.path()

        @property
        def is_leaf(self):
            return self.left is self.GROUND and self.right is self.GROUND

        @property
        def is_root(self):
            return self.parent is self.ROOT

        @property
        def depth(self):
            if self.is_leaf:
                return 1
            return 1 + max(self.left.depth, self.right.depth)

        def __eq__(self, other):
            return type(self) == type(other) and self.id == other.id

        __hash__ = object.__hash__

        def __lt__(self, other):
            return self.frequency < other.frequency

        def __gt__(self, other):
            return self.frequency > other.frequency

        def __le__(self, other):
            return self < other or self == other

        def __ge__(self, other):
            return self > other or self == other

    # ------------------------------------------------------------ construction
    @classmethod
    def construct_from_data(cls, data, key_func=utils.identity):
        groups = utils.group_by(data, key_func=key_func)
        leaves = [cls.Node.leaf(k, len(v)) for k, v in groups.items()]
        return cls(cls._construct(leaves), leaves, data, key_func)

    @classmethod
    def construct_from_counts(cls, keys, counts, data=None, key_func=utils.identity):
        """Fast path: keys already in first-appearance order with their counts."""
        leaves = [cls.Node.leaf(k, int(c)) for k, c in zip(keys, counts)]
        return cls(cls._construct(leaves), leaves, data, key_func)

    @classmethod
    def construct_from_leaves(cls, segments, key_func=utils.identity):
        leaves = [cls.Node.leaf(*s) for s in segments]
        return cls(cls._construct(leaves), leaves, None, key_func)

    @classmethod
    def construct_from_coding(cls, segments, key_func=utils.identity):
        """Rebuild a decoding tree from (value, code) pairs (huffman.py:30-58)."""
        by_code = dict((code, value) for value, code in segments)
        levels = max(len(code) for _, code in segments)
        root = cls.Node(None, None, None, None)
        leaves = []
        stack = [(root, 0, "")]
        while stack:
            node, depth, code = stack.pop()
            if code in by_code:
                node.value = by_code[code]
                leaves.append(node)
                continue
            if depth != levels:
                node.left = cls.Node.leaf(None, None)
                node.right = cls.Node.leaf(None, None)
                node.mass_adopt()
                # visit left ("1") before right ("0"), as the reference's recursion does
                stack.append((node.right, depth + 1, code + "0"))
                stack.append((node.left, depth + 1, code + "1"))
        return cls(root, leaves, None, key_func)

    @classmethod
    def _construct(cls, leaves):
        if len(leaves) == 1:
            return cls.Node.singleton(leaves[0])
        heap = list(leaves)
        heapq.heapify(heap)
        while len(heap) > 1:
            a = heapq.heappop(heap)
            b = heapq.heappop(heap)
            heapq.heappush(heap, cls.Node.combine(a, b))
        return heapq.heappop(heap)

    def __init__(self, root, leaves, data, key_func):
        self.root = root
        self.leaves = leaves
        self.data = data
        self.key_func = key_func
        self._codes = None
        self._by_leaf = None

    # ------------------------------------------------------------ codes
    @staticmethod
    def _code_of(leaf):
        bits = []
        node = leaf
        while not node.is_root:
            parent = node.parent
            bits.append("1" if parent.left is node else "0")
            node = parent
        return "".join(reversed(bits))

    def _leaf_codes(self):
        """{id(leaf): code string}, every leaf's path in ONE walk down from the root
        ("1" = left child, as _code_of reads it bottom-up); cached."""
        if self._by_leaf is None:
            out = {}
            stack = [(self.root, "")]
            while stack:
                node, code = stack.pop()
                if node is None:  # a singleton root's empty right side
                    continue
                if node.is_leaf:
                    out[id(node)] = code
                    continue
                stack.append((node.left, code + "1"))
                stack.append((node.right, code + "0"))
            self._by_leaf = out
        return self._by_leaf

    def codes(self):
        """{key: code string} for every leaf."""
        if self._codes is None:
            by_leaf = self._leaf_codes()
            self._codes = dict((leaf.value, by_leaf[id(leaf)]) for leaf in self.leaves)
        return self._codes

    def get_leaf(self, value):
        return utils.first(self.leaves, lambda l: l.value == value)

    def translate_path(self, path, s=""):
        return s + self._code_of(path[0]) if path else s

    def encode_table(self):
        by_leaf = self._leaf_codes()
        return [(leaf.value, by_leaf[id(leaf)]) for leaf in self.leaves]

    def encode_data(self, data=None):
        data = self.data if data is None else data
        codes = self.codes()
        return "".join(codes[self.key_func(d)] for d in data)

    def encode_keys(self, keys):
        """Vectorised encode of an integer key array (the jpeg_encode fast path)."""
        keys = np.asarray(keys)
        if keys.size == 0:
            return ""
        uniq, inv = np.unique(keys, return_inverse=True)
        codes = self.codes()
        table = np.array([codes[int(k)] for k in uniq], dtype=object)
        return "".join(table[inv].tolist())

    def code_table(self, key_min, nbins):
        """(code bits uint64, code lengths uint8) for keys key_min .. key_min + nbins - 1
        (0 / 0 for keys not in the tree), the table hic_huffman_pack reads."""
        bits = np.zeros(nbins, dtype=np.uint64)
        lens = np.zeros(nbins, dtype=np.uint8)
        for k, code in self.codes().items():
            if len(code) > 64:
                raise ValueError("Huffman code longer than 64 bits")
            bits[int(k) - key_min] = int(code, 2)
            lens[int(k) - key_min] = len(code)
        return bits, lens

    def flat(self):
        """The tree as hic_huffman_decode takes it: (child int32[2 * nodes], leaf nodes
        in index order).  child[2n] / child[2n + 1] = node n's left ('1') / right ('0')
        child: >= 0 internal, -1 none, <= -2 the leaf -2 - c; node 0 is the root."""
        if getattr(self, "_flat", None) is None:
            if self.root.is_leaf:
                raise ValueError("a one-node tree decodes nothing")
            child, leaves, index = [], [], {id(self.root): 0}
            order = [self.root]
            for node in order:  # breadth first; order grows as internal nodes appear
                for c in (node.left, node.right):
                    if c is None:
                        child.append(-1)
                    elif c.is_leaf:
                        child.append(-2 - len(leaves))
                        leaves.append(c)
                    else:
                        index[id(c)] = len(order)
                        child.append(len(order))
                        order.append(c)
            self._flat = (np.asarray(child, dtype=np.int32), leaves)
        return self._flat

    def min_code_length(self):
        """Depth of the shallowest leaf (>= 1): the shortest code of the tree."""
        if getattr(self, "_minlen", None) is None:
            child, _ = self.flat()
            depth, frontier = 1, [0]
            found = None
            while frontier and found is None:
                nxt = []
                for node in frontier:
                    for c in child[2 * node:2 * node + 2]:
                        if c <= -2:
                            found = depth
                        elif c >= 0:
                            nxt.append(int(c))
                frontier, depth = nxt, depth + 1
            self._minlen = found or 1
        return self._minlen

    def decode_device(self, bits_dev, nbits, out=None, stream=None):
        """decode_data of a packed MSB-first stream on the device (hic_huffman_decode):
        bits_dev a 4-byte-aligned uint8 tensor, nbits the stream length.  Returns
        (int32 device tensor of the decoded values, count, ints); leaves whose value is
        not an int32 (None, from a table with unused codes) decode to their leaf index
        (ints False) and ``self.flat()[1]`` maps them back (see decode_packed)."""
        child, nnodes, h_vals, nleaves, minlen = self.decode_args()
        out, n = _decode_flat(child, nnodes, h_vals, nleaves, minlen, bits_dev, nbits, out, stream)
        return out, n, h_vals is not None

    def decode_args(self):
        """(child, nodes, int32 leaf values or None, leaves, minlen -- a callable) as
        hic_huffman_decode takes the tree; values None when a leaf is not an int32
        (the kernel then writes leaf indices)."""
        child, leaves = self.flat()
        vals = [l.value for l in leaves]
        ints = all(isinstance(v, (int, np.integer)) and -2 ** 31 <= int(v) < 2 ** 31 for v in vals)
        h_vals = np.asarray([int(v) for v in vals], dtype=np.int32) if ints else None
        return child, len(child) // 2, h_vals, len(leaves), self.min_code_length

    def decode_packed(self, packed, nbits, stream=None):
        """decode_data of a packed MSB-first stream (numpy uint8) through the GPU
        decoder: the list of leaf values."""
        if self.root.is_leaf:  # no edges: the reference fails on the first bit
            return self.decode_data("1" if nbits else "")
        buf = np.zeros(-(-max(int(nbits), 1) // 32) * 4, np.uint8)
        body = np.asarray(packed, dtype=np.uint8)[:-(-int(nbits) // 8)]
        buf[:body.size] = body
        out, n, ints = self.decode_device(device.to_device(buf), nbits, stream=stream)
        got = device.to_host(out[:n])
        if ints:
            return got.tolist()
        leaves = self.flat()[1]
        return [leaves[i].value for i in got.tolist()]

    def decode_data(self, bits):
        out = []
        node = self.root
        for ch in bits:
            if ch == "1":
                node = node.left
            elif ch == "0":
                node = node.right
            else:
                raise RuntimeError("Illegal state")
            if node.is_leaf:
                out.append(node.value)
                node = self.root
        return out


def _decode_flat(child, nnodes, h_vals, nleaves, minlen, bits_dev, nbits, out=None, stream=None):
    """hic_huffman_decode over a flat tree (HuffmanTree.flat's layout): (int32
    device tensor of the decoded values -- leaf indices when h_vals is None --,
    count).  minlen: the shortest code, or a callable giving it (only needed to size
    a missing `out`)."""
    lib = _lib.load()
    with device.on_stream(stream):
        if out is None:
            # every decoded symbol consumes at least the shallowest leaf's depth in
            # bits: the output needs nbits / that many slots, not one per bit
            ml = minlen() if callable(minlen) else minlen
            out = device.empty((max(int(nbits) // ml, 1),), torch.int32)
        ws = device.workspace(lib.hic_huffman_decode_workspace_bytes(int(nbits), nnodes, nleaves))
        count = ctypes.c_int64(0)
        st = lib.hic_huffman_decode(device.ptr(bits_dev) if nbits else None, int(nbits),
                                    child.ctypes.data_as(ctypes.c_void_p), nnodes,
                                    h_vals.ctypes.data_as(ctypes.c_void_p) if h_vals is not None else None, nleaves,
                                    device.ptr(out), out.numel(), ctypes.byref(count), device.ptr(ws),
                                    device.stream_ptr(stream))
        if st == _lib.HIC_ERR_ARG and "missing child" in _lib.last_error():
            # the reference's reduce steps into None: huffman.py:155-161
            raise AttributeError("'NoneType' object has no attribute 'is_leaf'")
        _lib.check(st, "hic_huffman_decode")
    return out, int(count.value)


class CodeBook(_Packer):
    """The codes of the reference's tree over keys in first-appearance order with
    their counts, built in native code (hic_huffman_build: HuffmanTree._construct's
    heapq order, huffman.py:60-79) -- all codec.jpeg_encode needs of a tree: the
    table payload (encode_table) and the code table the GPU packer reads.
    HuffmanTree.construct_from_counts builds the same codes from node objects
    (~12 ms of Python heap work per 8K image; tests/test_cpu_host.py pins the two
    against each other)."""

    def __init__(self, keys, counts):
        self.leaf_keys = [int(k) for k in keys]
        n = len(self.leaf_keys)
        if n == 0:
            raise ValueError("a Huffman tree needs at least one key")
        c = np.ascontiguousarray(counts, dtype=np.int64)
        if c.shape != (n,):
            raise ValueError("one count per key")
        self.lens = np.empty(n, np.uint8)
        self.bits = np.empty(n, np.uint64)
        text = ctypes.create_string_buffer(65 * n)
        _lib.call("hic_huffman_build", c.ctypes.data_as(ctypes.c_void_p), n,
                  self.lens.ctypes.data_as(ctypes.c_void_p), self.bits.ctypes.data_as(ctypes.c_void_p), text)
        self._strs = text.value.decode("ascii").split()

    def code_strings(self):
        """Every leaf's code string, in leaf order."""
        return self._strs

    def encode_table(self):
        """[(key, code string)] in leaf order -- HuffmanTree.encode_table's."""
        return list(zip(self.leaf_keys, self.code_strings()))

    def codes(self):
        return dict(self.encode_table())

    def code_table(self, key_min, nbins):
        """(code bits uint64, code lengths uint8) for keys key_min .. key_min + nbins - 1
        (0 / 0 for keys not in the tree), the table hic_huffman_pack reads."""
        bits = np.zeros(nbins, dtype=np.uint64)
        lens = np.zeros(nbins, dtype=np.uint8)
        idx = np.asarray(self.leaf_keys, dtype=np.int64) - int(key_min)
        bits[idx] = self.bits
        lens[idx] = self.lens
        return bits, lens


class FlatCodes:
    """construct_from_coding's decoding tree (huffman.py:30-58) for a table that is a
    complete prefix code with int32 values -- every table an encoder writes --, built
    natively straight into hic_huffman_decode's layout (hic_huffman_from_codes).
    ``from_table`` returns None for any other table; the caller then builds the
    reference's own tree (HuffmanTree.construct_from_coding), whose None leaves and
    unreachable codes behave as the reference's do."""

    def __init__(self, child, nnodes, values, minlen):
        self.child, self.nnodes, self.values, self.minlen = child, nnodes, values, minlen

    @classmethod
    def from_table(cls, segments):
        n = len(segments)
        if n < 2:
            return None
        try:
            codes = [c for _, c in segments]
            raw = "".join(codes).encode("ascii")
            lens = np.fromiter(map(len, codes), dtype=np.int64, count=n)
        except (TypeError, ValueError, UnicodeEncodeError):
            return None
        off = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        child = np.empty(2 * n, np.int32)
        seg = np.empty(n, np.int32)
        nodes, minlen = ctypes.c_int64(0), ctypes.c_int32(0)
        st = _lib.load().hic_huffman_from_codes(raw, off.ctypes.data_as(ctypes.c_void_p), n,
                                                child.ctypes.data_as(ctypes.c_void_p),
                                                seg.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nodes),
                                                ctypes.byref(minlen))
        if st != _lib.HIC_OK:
            return None
        nn = int(nodes.value)
        vals = [segments[i][0] for i in seg[:nn + 1].tolist()]  # a full binary tree: nodes + 1 leaves
        if set(map(type, vals)) <= {int}:  # the common case, checked without a Python loop
            v64 = np.asarray(vals, dtype=object).astype(np.int64) if vals else np.zeros(0, np.int64)
        elif all(isinstance(v, (int, np.integer)) for v in vals):
            v64 = np.asarray([int(v) for v in vals], dtype=object).astype(np.int64)
        else:
            return None
        if v64.size and (v64.min() < -2 ** 31 or v64.max() >= 2 ** 31):
            return None
        return cls(child[:2 * nn], nn, v64.astype(np.int32), int(minlen.value))

    def decode_args(self):
        return self.child, self.nnodes, self.values, self.values.size, self.minlen

    def decode_device(self, bits_dev, nbits, out=None, stream=None):
        """HuffmanTree.decode_device's (values, count, True)."""
        out, n = _decode_flat(self.child, self.nnodes, self.values, self.values.size, self.minlen, bits_dev, nbits,
                              out, stream)
        return out, n, True


def first_appearance_counts(keys):
    """(unique keys in first-appearance order, counts) -- utils.group_by order."""
    keys = np.asarray(keys)
    uniq, first, counts = np.unique(keys, return_index=True, return_counts=True)
    order = np.argsort(first, kind="stable")
    return [int(k) for k in uniq[order]], counts[order]


# ------------------------------------------------------------------ device half
def device_key_range(keys_dev, n=None, stream=None):
    """(min, max) of a device key stream (hic_key_range; syncs)."""
    n = keys_dev.numel() if n is None else n
    with device.on_stream(stream):
        mm = device.empty((2,), torch.int32)
        _lib.call("hic_key_range", device.ptr(keys_dev), keys_dev.element_size(), n, device.ptr(mm),
                  device.stream_ptr(stream))
        lo, hi = (int(x) for x in mm.cpu().tolist())
    return lo, hi


def device_counts_raw(keys_dev, n, key_min, nbins, stream=None):
    """Per-bin (counts, first index) host arrays of hic_key_histogram (syncs)."""
    with device.on_stream(stream):
        counts = device.empty((nbins,), torch.int32)
        first = device.empty((nbins,), torch.int32)
        _lib.call("hic_key_histogram", device.ptr(keys_dev), keys_dev.element_size(), n, key_min, nbins,
                  device.ptr(counts), device.ptr(first), device.stream_ptr(stream))
        return counts.cpu().numpy().view(np.uint32), first.cpu().numpy().view(np.uint32)


class DeviceStream:
    """One key stream on the device with its GPU histogram: the Huffman tree
    (construct_from_data's, huffman.py:20-28: leaves in first-appearance order) and
    the packed bits of encode_data (huffman.py:131-142)."""

    def __init__(self, keys_dev, n=None, stream=None):
        self.keys, self.n, self.stream = keys_dev, keys_dev.numel() if n is None else int(n), stream
        if self.n == 0:
            raise ValueError("empty key stream")
        self.lo, hi = device_key_range(keys_dev, self.n, stream)
        self.nbins = hi - self.lo + 1
        self.counts, first = device_counts_raw(keys_dev, self.n, self.lo, self.nbins, stream)
        present = np.flatnonzero(self.counts)
        order = present[np.argsort(first[present], kind="stable")]
        self.keys_in_order = [int(self.lo + b) for b in order]
        self.tree = CodeBook(self.keys_in_order, self.counts[order].astype(np.int64))

    def packed(self):
        return self.tree.encode_device(self.keys, self.n, self.lo, self.nbins, self.counts, self.stream)


def device_counts(keys_dev, n=None, stream=None):
    """first_appearance_counts of a device key stream: (keys in first-appearance
    order, counts) from the GPU histogram (utils.group_by's order, which the tree's
    ties follow: huffman.py:20-28)."""
    n = keys_dev.numel() if n is None else n
    if n == 0:
        return [], np.zeros(0, np.int64)
    lo, hi = device_key_range(keys_dev, n, stream)
    counts, first = device_counts_raw(keys_dev, n, lo, hi - lo + 1, stream)
    present = np.flatnonzero(counts)
    order = present[np.argsort(first[present], kind="stable")]
    return [int(lo + b) for b in order], counts[order].astype(np.int64)


_FAN = 3
_fan_streams = []


def _fan_out(calls, stream=None):
    """calls[i](stream pointer) on side stream i % _FAN, joined back into `stream`
    (None: the current one): the nine key streams' histograms and packings are small
    launches that fill the chip better side by side than in a row.  The buffers they
    use were allocated on `stream`, which waits for every side stream before anything
    can free them."""
    cur = stream if stream is not None else torch.cuda.current_stream()
    while len(_fan_streams) < _FAN:
        _fan_streams.append(torch.cuda.Stream())
    for st in _fan_streams:
        st.wait_stream(cur)
    for i, fn in enumerate(calls):
        fn(device.stream_ptr(_fan_streams[i % _FAN]))
    for st in _fan_streams:
        cur.wait_stream(st)


class DeviceStreams:
    """Several device key streams at once (the nine of codec.jpeg_encode): the same
    trees and packed bits as one DeviceStream each, with the host round trips
    batched -- one copy back for all key ranges, one for all histograms, one upload
    of all code tables, one copy back for every stream's bits -- instead of five
    synchronising copies per stream."""

    def __init__(self, keys_list, stream=None):
        """stream: the stream the keys were produced on (None: the current one); every
        launch, allocation and host read here runs on it."""
        self.keys = [k for k, _ in keys_list]
        self.n = [int(n) for _, n in keys_list]
        self.stream = stream
        if min(self.n) == 0:
            raise ValueError("empty key stream")
        with device.on_stream(stream):
            self._histograms()

    def _histograms(self):
        stream = self.stream
        lib = _lib.load()
        s = device.stream_ptr(stream)
        m = len(self.keys)
        mm = device.empty((m, 2), torch.int32)
        for i, (k, n) in enumerate(zip(self.keys, self.n)):
            _lib.call("hic_key_range", device.ptr(k), k.element_size(), n, device.ptr(mm[i]), s)
        rng = mm.cpu().numpy()
        self.lo = [int(a) for a, _ in rng]
        self.nbins = [int(b) - int(a) + 1 for a, b in rng]
        off = np.concatenate([[0], np.cumsum(self.nbins)]).astype(np.int64)
        counts = device.empty((int(off[-1]),), torch.int32)
        first = device.empty((int(off[-1]),), torch.int32)
        _fan_out([lambda sp, i=i, k=k, n=n: _lib.call(
            "hic_key_histogram", device.ptr(k), k.element_size(), n, self.lo[i], self.nbins[i],
            ctypes.c_void_p(counts.data_ptr() + 4 * int(off[i])), ctypes.c_void_p(first.data_ptr() + 4 * int(off[i])),
            sp) for i, (k, n) in enumerate(zip(self.keys, self.n))], stream)
        c_all = counts.cpu().numpy().view(np.uint32)
        f_all = first.cpu().numpy().view(np.uint32)
        self.counts, self.trees = [], []
        for i in range(m):
            c = c_all[off[i]:off[i + 1]]
            f = f_all[off[i]:off[i + 1]]
            present = np.flatnonzero(c)
            order = present[np.argsort(f[present], kind="stable")]
            self.counts.append(c)
            self.trees.append(CodeBook((order + self.lo[i]).tolist(), c[order].astype(np.int64)))
        self._lib = lib

    def packed(self):
        """[(packed uint8 numpy array, number of bits)] per stream (hic_huffman_pack)."""
        return self.packed_start()()

    def packed_start(self):
        """packed() in two halves: the packing and its copy back are queued now and
        the returned function waits for them, so host work in between (jpeg_encode's
        table payloads) overlaps the GPU."""
        with device.on_stream(self.stream):
            return self._packed()

    def _packed(self):
        m = len(self.keys)
        s = device.stream_ptr(self.stream)
        tabs = [t.code_table(lo, nb) for t, lo, nb in zip(self.trees, self.lo, self.nbins)]
        totals = [int(np.sum(np.asarray(c, dtype=np.int64) * l.astype(np.int64)))
                  for c, (_, l) in zip(self.counts, tabs)]
        nbytes = [max(4, -(-t // 32) * 4) for t in totals]
        boff = np.concatenate([[0], np.cumsum(nbytes)]).astype(np.int64)
        toff = np.concatenate([[0], np.cumsum(self.nbins)]).astype(np.int64)
        cb = device.to_device(np.concatenate([b for b, _ in tabs]).view(np.int64))
        cl = device.to_device(np.concatenate([l for _, l in tabs]))
        out = device.empty((int(boff[-1]),), torch.uint8)
        nbits = device.empty((m,), torch.int64)
        # one workspace per side stream: the launches of one stream run in order
        wss = [device.workspace(self._lib.hic_huffman_pack_workspace_bytes(max(self.n))) for _ in range(_FAN)]
        _fan_out([lambda sp, i=i, k=k, n=n: _lib.call(
            "hic_huffman_pack", device.ptr(k), k.element_size(), n, self.lo[i], self.nbins[i],
            ctypes.c_void_p(cb.data_ptr() + 8 * int(toff[i])), ctypes.c_void_p(cl.data_ptr() + int(toff[i])),
            ctypes.c_void_p(out.data_ptr() + int(boff[i])), nbytes[i], ctypes.c_void_p(nbits.data_ptr() + 8 * i),
            device.ptr(wss[i % _FAN]), sp) for i, (k, n) in enumerate(zip(self.keys, self.n))], self.stream)
        # the bits (~40 MB at 8K) and the bit counts copied back without waiting:
        # into a pinned pool buffer, on the stream after the packing
        cur = self.stream if self.stream is not None else torch.cuda.current_stream()
        host = device.host_empty((out.numel(),), np.uint8)
        nb_host = torch.empty((m,), dtype=torch.int64, pin_memory=True)
        with torch.cuda.stream(cur):
            nb_host.copy_(nbits, non_blocking=True)
            if device._is_pinned(host):
                torch.from_numpy(host).copy_(out, non_blocking=True)
            done = torch.cuda.Event()
            done.record(cur)

        def collect():
            done.synchronize()
            h = host if device._is_pinned(host) else device.to_host(out)
            nb = nb_host.numpy()
            res = []
            for i in range(m):
                if int(nb[i]) != totals[i]:
                    raise RuntimeError("stream %d: packed %d bits, the histogram says %d" % (i, int(nb[i]), totals[i]))
                res.append((h[boff[i]:boff[i] + -(-int(nb[i]) // 8)], int(nb[i])))
            return res
        return collect
