"""Entropy coding front end (mirrors hiccup/codec.py:23-426), JPEG flavour.

GPU (libhiccup_hip.so):
* ``run_length_coding``  -> hic_rle_stream_encode_i32 (codec.py:55-99)
* ``decode_run_length``  -> hic_rle_stream_decode_i32 (codec.py:102-113)
* ``jpeg_encode``: per channel, split + zig-zag (hic_zigzag_blocks_i32), DC DPCM
  and the channel-wide AC RLE (hic_rle_encode_i32) -- codec.py:286-301
* ``jpeg_decode``: AC RLE decode + group into blocks + DC integration
  (hic_rle_decode_i32) and izigzag + merge + crop (hic_izigzag_blocks_i32) --
  codec.py:397-425
Host ("next" row): the Huffman stage and payload assembly
(codec.py:242-272,304-334,354-394), byte-compatible with the reference.

Deliberate deviation: jpeg_decode does not print the luminance AC list to
stdout (the reference's debugging print at codec.py:406-408).
"""
import contextlib
import ctypes
import gc
import threading

import numpy as np
import torch

from . import _lib, device, hicimage as hic, huffman, model, settings, utils

MAX_LEN = 0xF
_OUT_OF_SCOPE = "the wavelet (HIC) scheme is out of scope (DESIGN.md)"


class RunLength:
    """(zeros-before, value) symbol (codec.py:23-44)."""

    @classmethod
    def from_dict(cls, d):
        return cls(d["value"], d["zeros"])

    def __init__(self, value=0, length=0):
        self.value = value
        self.length = length

    def __eq__(self, other):
        return type(self) == type(other) and self.value == other.value and self.length == other.length

    def __str__(self):
        return "(%d, %d)" % (self.length, self.value)

    __repr__ = __str__

    @property
    def segment(self):
        return [0] * self.length + [self.value]

    @property
    def is_trailing(self):
        return self.value == 0 and self.length == 0


def _i32(a, what):
    a = np.asarray(a)
    if a.size and not np.issubdtype(a.dtype, np.integer):
        if not np.all(np.mod(a, 1) == 0):
            raise ValueError("%s must be integer-valued" % what)
    a = a.astype(np.int64)
    if a.size and (a.min() < -(1 << 31) or a.max() >= (1 << 31)):
        raise ValueError("%s out of int32 range" % what)
    return a.astype(np.int32)


def _i32_device(a, what, wait=True):
    """_i32's checks and result as an int32 device tensor (large float planes are
    checked and cast on the GPU: device.to_device_i32)."""
    return device.to_device_i32(a, "%s must be integer-valued" % what, "%s out of int32 range" % what, wait=wait)


def differential_coding(blocks):
    """codec.py:47-52: [dc0, dc1 - dc0, ...] over the blocks' [0][0] entries."""
    return utils.differences([b[0][0] for b in blocks])


# ------------------------------------------------------------------ RLE on GPU
def rle_encode_device(arr_dev, n, max_len=MAX_LEN, stream=None):
    """run_length_coding of a device int32 array -> (lengths, values, count) device tensors."""
    cap = n + 1  # each element yields at most one symbol, plus the EOB
    L = device.empty((cap,), torch.int32)
    V = device.empty((cap,), torch.int32)
    cnt = device.empty((1,), torch.int64)
    lib = _lib.load()
    ws = device.workspace(lib.hic_rle_workspace_bytes(max(1, -(-n // 64)), 64))
    src = device.ptr(arr_dev) if n > 0 else ctypes.c_void_p(0)
    _lib.call("hic_rle_stream_encode_i32", src, n, max_len, device.ptr(L), device.ptr(V), cap, device.ptr(cnt),
              device.ptr(ws), device.stream_ptr(stream))
    return L, V, cnt


def run_length_coding(arr, max_len=MAX_LEN):
    """codec.py:55-99 -> list of RunLength."""
    if max_len is not None:
        if max_len == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
        if max_len < 0:
            raise ValueError("max_len must be positive")
    a = _i32(np.asarray(arr).reshape(-1), "run_length_coding input")
    utils.debug_msg("Going to determine RLE for %d size array" % len(a))
    n = len(a)
    dev = device.to_device(a) if n else device.empty((1,), torch.int32)
    L, V, cnt = rle_encode_device(dev, n, max_len or 0)
    count = int(device.to_host(cnt)[0])
    assert count > 0
    Lh = L[:count].cpu().numpy()
    Vh = V[:count].cpu().numpy()
    return [RunLength(int(v), int(l)) for l, v in zip(Lh, Vh)]


def decode_run_length(rles, length):
    """codec.py:102-113 -> list of ints (EOB zero-fills up to `length`)."""
    if len(rles) == 0:
        # the reference flattens an empty list with functools.reduce
        raise TypeError("reduce() of empty iterable with no initial value")
    Lh = _i32([r.length for r in rles], "run lengths")
    Vh = _i32([r.value for r in rles], "run values")
    total = int(np.sum(Lh.astype(np.int64) + 1))
    cap = -(-max(total, int(length), 1) // 64) * 64
    out = device.empty((cap,), torch.int32)
    status = device.empty((1,), torch.int64)
    lib = _lib.load()
    ws = device.workspace(lib.hic_rld_workspace_bytes(len(Lh), cap // 64))
    Ld, Vd = device.to_device(Lh), device.to_device(Vh)
    _lib.call("hic_rle_stream_decode_i32", device.ptr(Ld), device.ptr(Vd), len(Lh), int(length), device.ptr(out),
              cap, device.ptr(status), device.ptr(ws), device.stream_ptr())
    n = int(device.to_host(status)[0])
    return out[:n].cpu().numpy().tolist()


# ------------------------------------------------------------------ jpeg_encode
def encode_channel_device(raster_dev, H, W, bs, stream=None):
    """Front half of jpeg_encode for one int32 coefficient plane on the device:
    split + zig-zag (block size bs), DC DPCM, AC RLE.  Returns device tensors
    (dc_diff int32[nblk], lengths int32, values int32, count int64[1])."""
    nbx, nby = -(-W // bs), -(-H // bs)
    nblk, L = nbx * nby, bs * bs
    blocks = device.empty((nblk, L), torch.int32)
    _lib.call("hic_zigzag_blocks_i32", device.ptr(raster_dev), H, W, bs, device.ptr(blocks),
              device.stream_ptr(stream))
    if L == 1:
        # no AC coefficients: the AC stream is empty -> [EOB]
        dc = blocks.view(-1).clone()
        dc[1:] = blocks.view(-1)[1:] - blocks.view(-1)[:-1]
        Ls, Vs, cnt = rle_encode_device(dc, 0, MAX_LEN, stream)
        return dc, Ls, Vs, cnt
    cap = nblk * (L - 1) + 1
    dc = device.empty((nblk,), torch.int32)
    Ls = device.empty((cap,), torch.int32)
    Vs = device.empty((cap,), torch.int32)
    cnt = device.empty((1,), torch.int64)
    ws = device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, L))
    _lib.call("hic_rle_encode_i32", device.ptr(blocks), nblk, L, MAX_LEN, ctypes.c_void_p(0), device.ptr(dc),
              device.ptr(Ls), device.ptr(Vs), cap, device.ptr(cnt), device.ptr(ws), device.stream_ptr(stream))
    return dc, Ls, Vs, cnt


def encode_channel_device8(raster_dev, H, W, stream=None):
    """encode_channel_device for 8x8 blocks through int16: the zig-zag writes int16
    blocks (hic_zigzag8_blocks_i16) and the hot path's 16-bit RLE codes them
    (hic_rle_encode_i16: uint8 lengths, int16 values).  Returns (dc_diff, lengths,
    values, count, wide): wide (device int32[1]) is 1 when a coefficient did not fit
    int16, and the plane must then go through encode_channel_device instead."""
    nbx, nby = -(-W // 8), -(-H // 8)
    nblk = nbx * nby
    s = device.stream_ptr(stream)
    blocks = device.empty((nblk, 64), torch.int16)
    wide = device.empty((1,), torch.int32)
    _lib.call("hic_zigzag8_blocks_i16", device.ptr(raster_dev), H, W, device.ptr(blocks), device.ptr(wide), s)
    cap = nblk * 63 + 1
    dc = device.empty((nblk,), torch.int32)
    Ls = device.empty((cap,), torch.uint8)
    Vs = device.empty((cap,), torch.int16)
    cnt = device.empty((1,), torch.int64)
    ws = device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64))
    _lib.call("hic_rle_encode_i16", device.ptr(blocks), nblk, 64, MAX_LEN, ctypes.c_void_p(0), device.ptr(dc),
              device.ptr(Ls), device.ptr(Vs), cap, device.ptr(cnt), device.ptr(ws), s)
    return dc, Ls, Vs, cnt, wide


def encode_channel(plane, bs=None):
    """(dc_diffs, ac_lengths, ac_values) numpy arrays for one coefficient plane."""
    bs = settings.JPEG_BLOCK_SIZE if bs is None else bs
    p = _i32_device(plane, "coefficient plane")
    if p.ndim != 2:
        raise ValueError("expected a 2-D coefficient plane")
    H, W = p.shape
    dc, Ls, Vs, cnt = encode_channel_device(p, H, W, bs)
    count = int(device.to_host(cnt)[0])
    return dc.cpu().numpy(), Ls[:count].cpu().numpy(), Vs[:count].cpu().numpy()


def huffman_encode(huff, key_type=None):
    """A tree's table payload; key_type: the scalar type its keys have in the
    reference (numpy integers of the plane's dtype for the DC trees, whose keys come
    from the plane itself; Python ints for the RLE trees) -- it shows in the bytes."""
    kt = key_type or (lambda v: v)
    return hic.PayloadStringP(hic.TupP, [hic.TupP(kt(v), c) for v, c in huff.encode_table()])


def huffman_decode(data):
    return huffman.HuffmanTree.construct_from_coding([p.numbers for p in data.payloads])


def huffman_data_encode(huff):
    return hic.BitStringP(huff.encode_data())


def huffman_data_decode(data, tree):
    return tree.decode_data(data.payload)


def jpeg_encode(compressed):
    """codec.py:275-334: CompressedImage -> HicImage (9 tables, 9 bit strings, 2 shapes).
    Everything but the nine trees runs on the GPU: split + zig-zag, DC DPCM, AC RLE
    (encode_channel_device), the key histograms in first-appearance order and the
    bit packing of the coded streams (huffman.DeviceStreams, csrc/huffman.hip).  The
    trees' node objects pause Python's cyclic collector as in jpeg_decode."""
    with _gc_paused():
        return _jpeg_encode(compressed)


def _jpeg_encode(compressed):
    utils.debug_msg("Starting JPEG encoding")
    bs = settings.JPEG_BLOCK_SIZE
    chans = ("lum", "cr", "cb")
    enc, dc_type, planes = {}, {}, {}
    for k, v in compressed.as_dict.items():
        # the reference's DC keys are elements of the plane (utils.differences over
        # block[0][0]): numpy scalars of its dtype
        dc_type[k] = np.asarray(v).dtype.type
        # wait=False: `compressed` holds the planes unchanged until the count read
        # below synchronises, so the uploads queue back to back
        p = _i32_device(v, "coefficient plane", wait=False)
        if p.ndim != 2:
            raise ValueError("expected a 2-D coefficient plane")
        planes[k] = p
        # no host read here: the next plane's upload overlaps this plane's RLE.  8x8
        # blocks go through int16 (the hot path's RLE); a plane with a coefficient
        # outside int16 is redone below through int32
        enc[k] = (encode_channel_device8(p, p.shape[0], p.shape[1]) if bs == 8 else
                  encode_channel_device(p, p.shape[0], p.shape[1], bs) + (None,))
    flags = torch.cat([torch.cat([e[3], e[4].to(torch.int64)]) if e[4] is not None else
                       torch.cat([e[3], torch.zeros(1, dtype=torch.int64, device=e[3].device)])
                       for e in enc.values()]).cpu().tolist()
    counts = []
    for i, k in enumerate(list(enc)):
        cnt, wide = flags[2 * i], flags[2 * i + 1]
        if wide:
            p = planes[k]
            enc[k] = encode_channel_device(p, p.shape[0], p.shape[1], bs) + (None,)
            cnt = int(enc[k][3].cpu()[0])
        counts.append(cnt)
    del planes
    keys = {}
    for (k, (dc, Ls, Vs, _, _)), count in zip(enc.items(), counts):
        # trees per channel: DC differences, AC values, AC lengths (codec.py:304-313)
        keys[k] = ((dc, dc.numel()), (Vs, count), (Ls, count))
    # the nine streams in payload order (codec.py:310-330); each tree codes the
    # stream it was built from
    order = [(k, j) for j in range(3) for k in chans]
    ds = huffman.DeviceStreams([keys[k][j] for k, j in order])
    collect = ds.packed_start()  # the GPU packs while the host builds the table payloads
    tables = [huffman_encode(ds.trees[i], dc_type[k] if j == 0 else int) for i, (k, j) in enumerate(order)]
    data = [hic.BitStringP.from_packed(*pk) for pk in collect()]
    shape = compressed.shape
    payloads = tables + data + [hic.TupP(shape[0][0], shape[0][1]), hic.TupP(shape[1][0], shape[1][1])]
    return hic.HicImage.jpeg_image(payloads)


def jpeg_decode(hic_image):
    """codec.py:337-426: HicImage -> CompressedImage (float64 planes).  The nine
    coded streams are decoded on the GPU (hic_huffman_decode, in the reference's
    order: DC, AC values, AC lengths, codec.py:372-388) and stay there for the RLE
    decode, DC integration and izigzag (hic_rle_decode_i32, hic_izigzag_blocks_i32);
    only the nine trees (from the tables) are built on the host.  Python's cyclic
    collector (a process-wide switch) is paused while any jpeg_decode call runs: the
    trees' many small nodes set off full collections that cost 15-60 ms at 8K
    (tools/prof_jdec.py).  Concurrent calls share one pause (_gc_paused counts
    them), so a call ending never re-enables it under another still running, and
    the collector's state from before the first call is restored after the last."""
    with _gc_paused():
        return _jpeg_decode(hic_image)


_gc_lock = threading.Lock()
_gc_users = 0
_gc_was = True


@contextlib.contextmanager
def _gc_paused():
    global _gc_users, _gc_was
    with _gc_lock:
        if _gc_users == 0:
            _gc_was = gc.isenabled()
            gc.disable()
        _gc_users += 1
    try:
        yield
    finally:
        with _gc_lock:
            _gc_users -= 1
            if _gc_users == 0 and _gc_was:
                gc.enable()


def _jpeg_decode(hic_image):
    utils.debug_msg("JPEG decode")
    assert hic_image.hic_type == model.Compression.JPEG
    p = hic_image.payloads
    chans = ("lum", "cr", "cb")
    trees = [_decoding_tree(p[i]) for i in range(9)]
    streams = _huffman_streams_device([p[9 + i] for i in range(9)], trees)
    shapes = {"lum": p[18].numbers, "cr": p[19].numbers, "cb": p[19].numbers}
    bs = settings.JPEG_BLOCK_SIZE
    sub_length = bs * bs - 1
    # the three channels' RLE decodes and izigzags are queued before any status is
    # read (codec.py:418's checks then run in channel order), and the three planes
    # come back in one wait: chroma's kernels run beside luma's copy
    pending = []
    for c, k in enumerate(chans):
        dc, vals, lens = streams[c], streams[3 + c], streams[6 + c]
        n = min(vals[1], lens[1])  # zip() in codec.py:399-400
        if n == 0:
            raise TypeError("reduce() of empty iterable with no initial value")
        if sub_length == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
        pending.append(_decode_channel_start(dc, lens, vals, n, shapes[k], bs))
    for raster, check in pending:
        check()
    planes = device.to_host_f64_many([raster for raster, _ in pending])
    return model.CompressedImage.from_dict(dict(zip(chans, planes)))


def _decoding_tree(data):
    """huffman_decode's tree, built natively when the table is a complete prefix code
    of int32 values (huffman.FlatCodes: every table an encoder writes), else the
    reference's own construction."""
    flat = huffman.FlatCodes.from_table([p.numbers for p in data.payloads])
    return flat if flat is not None else huffman_decode(data)


def _huffman_streams_device(payloads, trees):
    """_huffman_stream_device of every (payload, tree) -- codec.jpeg_decode's nine
    huffman_data_decode calls (codec.py:372-388) -- in ONE hic_huffman_decode_batch:
    the bits go up in one copy, the streams share each phase's host wait.  Errors as
    the reference's sequential decode raises them: the first failing stream in
    payload order."""
    n = len(payloads)
    lib = _lib.load()
    res, errs, jobs_at = [None] * n, [None] * n, []
    bufs, offs, tot = [], [], 0
    for i, (pl, tree) in enumerate(zip(payloads, trees)):
        packed, nbits = pl.packed_bits()
        nbits = int(nbits)
        if isinstance(tree, huffman.HuffmanTree) and tree.root.is_leaf:
            try:  # no edges: the reference's walk fails on the first bit
                tree.decode_data("1" if nbits else "")
                res[i] = (device.to_device(np.zeros(1, np.int32)), 0, True)
            except Exception as e:  # noqa: BLE001 -- raised below, in payload order
                errs[i] = e
            continue
        words = -(-max(nbits, 1) // 32) * 4
        body = np.asarray(packed, dtype=np.uint8)[:-(-nbits // 8)]
        bufs.append((body, words))
        offs.append(tot)
        tot += words
        jobs_at.append((i, nbits, tree.decode_args()))
    if jobs_at:
        dbits = device.to_device_parts([body for body, _ in bufs], offs, tot)
        jobs = (_lib.HuffDecodeJob * len(jobs_at))()
        keep = []
        for k, ((i, nbits, (child, nnodes, h_vals, nleaves, minlen)), o) in enumerate(zip(jobs_at, offs)):
            ml = minlen() if callable(minlen) else minlen
            out = device.empty((max(nbits // ml, 1),), torch.int32)
            ws = device.workspace(lib.hic_huffman_decode_workspace_bytes(nbits, nnodes, nleaves))
            keep.append((out, ws, child, h_vals))
            jobs[k] = _lib.HuffDecodeJob(dbits.data_ptr() + o, nbits, child.ctypes.data, nnodes,
                                         h_vals.ctypes.data if h_vals is not None else None, nleaves, out.data_ptr(),
                                         out.numel(), ws.data_ptr(), 0, 0)
        st = lib.hic_huffman_decode_batch(len(jobs_at), jobs, device.stream_ptr())
        if st != _lib.HIC_OK and all(j.status == _lib.HIC_OK for j in jobs):
            _lib.check(st, "hic_huffman_decode_batch")  # refused before anything ran
        for k, (i, _, (_, _, h_vals, _, _)) in enumerate(jobs_at):
            j = jobs[k]
            if j.status == _lib.HIC_ERR_ARG:
                # the reference's reduce steps into None: huffman.py:155-161
                errs[i] = AttributeError("'NoneType' object has no attribute 'is_leaf'")
            elif j.status != _lib.HIC_OK:
                errs[i] = MemoryError("hic_huffman_decode_batch: stream %d decoded %d symbols" % (i, j.count))
            else:
                res[i] = (keep[k][0], int(j.count), h_vals is not None)
    for i in range(n):
        if errs[i] is not None:
            raise errs[i]
        d, cnt, ints = res[i]
        if not ints:  # a table with non-int32 leaves: the leaf indices map back on the host
            leaves = trees[i].flat()[1]
            vals = _i32([leaves[x].value for x in device.to_host(d[:cnt]).tolist()], "decoded values")
            res[i] = (device.to_device(vals if cnt else np.zeros(1, np.int32)), cnt, True)
    return [(d, cnt) for d, cnt, _ in res]


def _decode_channel_start(dc, lens, vals, n, shape, bs):
    """The RLE decode + DC integration + izigzag of one channel from its decoded
    streams (device int32 tensors with counts), queued: (the int32 raster on the
    device, a function that runs codec.py:418's assertions on the decode's status)."""
    (Dd, nblk), (Ld, _), (Vd, _) = dc, lens, vals
    L, sub = bs * bs, bs * bs - 1
    H, W = int(shape[0]), int(shape[1])
    if nblk == 0:  # decoded // sub_length == 0 needs decoded == 0; n > 0 symbols cover >= 1
        raise AssertionError()
    if H * W != nblk * L:
        # ac_length (codec.py:403) differs from nblk * sub: evaluate the assertion
        # on the symbols themselves (a malformed file; never the encoder's output)
        lh, vh = device.to_host(Ld[:n]).astype(np.int64), device.to_host(Vd[:n])
        total = int(np.sum(lh + 1))
        decoded = max(total, H * W - nblk) if (lh[-1] == 0 and vh[-1] == 0) else total
        assert decoded % sub == 0
        assert decoded // sub == nblk
    blocks = device.empty((nblk, L), torch.int32)
    status = device.empty((1,), torch.int64)
    ws = device.workspace(_lib.load().hic_rld_workspace_bytes(n, nblk))
    _lib.call("hic_rle_decode_i32", device.ptr(Ld), device.ptr(Vd), n, device.ptr(Dd), nblk, L,
              device.ptr(blocks), device.ptr(status), device.ptr(ws), device.stream_ptr())
    raster = device.zeros((H, W), torch.int32)
    _lib.call("hic_izigzag_blocks_i32", device.ptr(blocks), H, W, bs, device.ptr(raster), device.stream_ptr())

    def check():
        if H * W == nblk * L:
            # status = max(total, nblk * sub) after an EOB, else total (k_rld_status):
            # codec.py:418's two assertions hold exactly when it is nblk * sub
            assert int(status.cpu()[0]) == nblk * sub
    return raster, check


# ------------------------------------------------------------------ out of scope
def wavelet_encode(compressed):
    raise NotImplementedError(_OUT_OF_SCOPE)


def wavelet_decode(hic_image):
    raise NotImplementedError(_OUT_OF_SCOPE)


def wavelet_decode_pull_subbands(data, shapes):
    raise NotImplementedError(_OUT_OF_SCOPE)


def wavelet_decoded_subbands_shapes(min_shape, max_shape):
    raise NotImplementedError(_OUT_OF_SCOPE)


def wavelet_decoded_length(min_shape, max_shape):
    raise NotImplementedError(_OUT_OF_SCOPE)
