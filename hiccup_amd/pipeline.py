"""Device-resident JPEG-style encode / decode pipeline (the hot path, no host hops).

``Encoder.encode(rgb)`` = compression.jpeg_compression + the zig-zag / DC / RLE
half of codec.jpeg_encode (compression.py:16-39, codec.py:286-301) for one
H x W x 3 uint8 image that already lives in HBM:

  1+2. hic_encode420_u8       (W % 512 == 0 by default, any W % 16 on request;
                              H % 16 == 0) colour + 4:2:0 pyrDown +
                              8x8 DCT + quantize + zig-zag of the three planes + the
                              RLE tile records in ONE launch; the planes never reach
                              HBM.  Otherwise two launches:
  1. hic_rgb_to_ycrcb420      RGB -> Y (H x W) + pyrDown'd Cr, Cb (H/2 x W/2)
  2. hic_dct_quant_rle_u8_batch  8x8 DCT + quantize + zig-zag of the three planes in
                              one launch -> int16 blocks (ZIGZAG_I16), with the RLE
                              tile pass fused into the epilogue
  3. hic_rle_encode_i16_tiles_batch  DC DPCM + channel-wide AC RLE of all three
                              channels (one scan + one emit launch) -> (uint8 len, int16 val)

Slot layout (round 6, the default for a whole image with W % 512 == 0, H % 16 ==
0 and max_len 15): hic_encode420_slots_u8 writes every RLE record's symbols and DC
differences itself (slots.h), and hic_rle_slots_close (one scan launch) closes
the records' carried runs and writes the record index: two launches per image, no
int16 coefficients in HBM.  compact() / materialize() give the contiguous stream
and the zig-zag blocks when a caller asks (result(), hic_image()).

All launches are asynchronous on one stream; buffers are allocated once.
``Decoder.decode`` runs the inverse chain (codec.jpeg_decode's RLE/DC/izigzag
half + compression.jpeg_decompression).  The optional ``stitch`` tensors make
an encoder one tile-shard of a larger image (see sharding.py).
"""
import ctypes

import numpy as np
import torch

from . import _lib, device

CHANNELS = ("lum", "cr", "cb")
TABLES = {"lum": _lib.TABLE_LUMINANCE, "cr": _lib.TABLE_CHROMINANCE, "cb": _lib.TABLE_CHROMINANCE}


def _nblk(h, w):
    return -(-h // 8) * -(-w // 8)


def input_span(H, r0, r1):
    """Rows of an H-row image that hic_rgb_to_ycrcb420_rows needs for output rows [r0, r1)."""
    c0, c1 = r0 // 2, min(H // 2, r1 // 2)
    return max(0, 2 * c0 - 2), max(r1, min(H, 2 * c1 + 2))


# hic_rle_encode_* report failures through the count (include/hiccup_hip.h):
# -(symbols needed) when the buffer is too small, HIC_COUNT_SCAN_TIMEOUT when a
# cross-workgroup scan hand-off timed out (never expected; the stream is invalid)
COUNT_SCAN_TIMEOUT = -(2 ** 63)
COUNT_WIRE_OVERFLOW = -(2 ** 63) + 1  # a gathered segment's sender flagged an out-of-width value


def check_count(c, channel=""):
    """Raise the error a negative symbol count stands for."""
    if c >= 0:
        return
    if c == COUNT_SCAN_TIMEOUT:
        raise _lib.HipError("RLE scan hand-off timed out (channel %s): the stream is invalid" % channel)
    if c == COUNT_WIRE_OVERFLOW:
        raise _lib.HipError("a gathered shard flagged a coefficient outside its wire width (channel %s): the "
                            "stream is invalid" % channel)
    raise MemoryError("symbol buffer too small for channel %s: %d symbols needed" % (channel, -c))


def encoder_layout(H, W, rows=None, fused=None, index=False):
    """(fused, rpt) of an Encoder of rows `rows` of an H x W image (None: the whole
    image, its own encoder): whether it runs the fused kernel (None = the measured
    default: fusable, and for row shards or an encoder with a tile index W % 512 ==
    0 too), and its RLE records per 64-block tile per channel (the fused kernel's
    chroma: one per 32-block half tile; a whole image's ragged last strip: one per
    strip segment, see Encoder.seg)."""
    r0, r1 = rows if rows is not None else (0, H)
    a, b = input_span(H, r0, r1)
    # (hic_encode420_u8 reads the input rows through 32-bit buffer offsets)
    can_fuse = (W % 16 == 0 and H % 16 == 0 and r0 % 16 == 0 and r1 % 16 == 0
                and (b - a) * W * 3 <= 2**31 - 1)
    if fused and not can_fuse:
        raise ValueError("the fused encoder needs W, H and rows multiples of 16, "
                         "and < 2 GiB of input rows")
    seg = rows is None and not index  # a whole image's own encoder: records per strip segment
    f = (can_fuse and (W % 512 == 0 or seg)) if fused is None else bool(fused)
    half = f and (W % 512 == 0 or seg)
    return f, {"lum": 1, "cr": 2 if half else 1, "cb": 2 if half else 1}


def slots_eligible(H, W, max_len=15, rows=None, out=None, fused=None, landing_rpt=None):
    """Whether an Encoder of this shape can take the slot layout (hic_encode420_slots_u8:
    a whole image, W % 512 == 0, H % 16 == 0, max_len 15, < 2 GiB of RGB)."""
    return (rows is None and out is None and landing_rpt is None and fused is not False and max_len == 15
            and W % 512 == 0 and H % 16 == 0 and H >= 16 and H * W * 3 <= 2**31 - 1)


class SlotIndex:
    """The slot-layout stream of an Encoder for Decoder.decode(index=...): per channel
    the slot arrays, the close's record index and the records per 64-block tile."""

    def __init__(self, enc):
        self.slot_len, self.slot_val, self.sidx, self.rpt = enc.slot_len, enc.slot_val, enc.sidx, enc.rpt

    def __getitem__(self, k):
        return self.sidx[k]


class Encoder:
    """rows=(r0, r1) makes this encoder one row-shard of an H x W image (r0 even;
    shards of one image split at multiples of 16 rows so chroma blocks align)."""

    def __init__(self, H, W, max_len=15, rows=None, out=None, fused=None, index=False, landing_rpt=None, slots=None):
        """out: optional {channel: (coef (n, 64) int16, dc (n,) int32)} device views the
        encoder writes into (a gathering rank points them at its slice of the whole
        image's buffers, so its own shard needs no copy).
        fused: colour + 4:2:0 + DCT in one kernel (hic_encode420_u8, the planes never
        reach HBM; W, H and the row range multiples of 16); None = the faster path
        as measured (encoder_layout): fused for a whole image with W % 16 == 0 (a
        ragged last strip gets one RLE record per strip segment: 3840x2160 38.1-40.1
        vs 40.5-41.4 us per image for the chain), and for a row
        shard or an encoder with a tile index when W % 512 == 0; False = the chain.
        landing_rpt: a landing zone only (the gathering rank of a stream gather): no
        transform, no plane buffers, and the RLE record layout of the shards that
        fill it (their encoder_layout rpt), whatever this shape alone would pick.
        slots: the slot layout (module docstring); None = whenever slots_eligible,
        False = the coefficient + emit chain."""
        if H < 2 or W < 2:
            raise ValueError("image must be at least 2 x 2")
        device.require_gpu()
        self.H, self.W, self.max_len = H, W, max_len
        r0, r1 = rows if rows is not None else (0, H)
        if r0 % 2 or not (0 <= r0 < r1 <= H):
            raise ValueError("bad row range %r" % ((r0, r1),))
        self.rows = (r0, r1)
        self.want_index = bool(index)
        self.landing = landing_rpt is not None
        ok = slots_eligible(H, W, max_len, rows, out, fused, landing_rpt)
        if slots and not ok:
            raise ValueError("the slot layout needs a whole image with W % 512 == 0, H % 16 == 0 and max_len 15")
        self.slots = ok if slots is None else bool(slots)
        if self.landing:
            self.fused, self.rpt = False, dict(landing_rpt)
        elif self.slots:
            self.fused, self.rpt = True, {"lum": 1, "cr": 2, "cb": 2}
        else:
            self.fused, self.rpt = encoder_layout(H, W, rows, fused, index)
        # a whole image's ragged last strip (W % 512 != 0): the fused kernel writes one
        # RLE record per strip segment (hic_encode420_seg_u8) and the scan / emit walk
        # row segments (hic_rle_encode_i16_rows_batch): no tile pass
        self.seg = (not self.landing and not self.slots and self.fused and rows is None and W % 512 != 0
                    and not self.want_index)
        c0, c1 = r0 // 2, min(H // 2, r1 // 2)
        self.shapes = {"lum": (r1 - r0, W), "cr": (c1 - c0, W // 2), "cb": (c1 - c0, W // 2)}
        ys, cs = self.shapes["lum"], self.shapes["cr"]
        lib = _lib.load()
        # the planes exist only on the two-kernel path
        self.y = self.cr = self.cb = None
        if not self.fused and not self.landing:
            self.y = device.empty(ys, torch.uint8)
            self.cr = device.empty(cs, torch.uint8)
            self.cb = device.empty(cs, torch.uint8)
        self.planes = {"lum": self.y, "cr": self.cr, "cb": self.cb}
        self.coef, self.dc, self.sym_len, self.sym_val, self.ws, self.ws_bytes = {}, {}, {}, {}, {}, {}
        self.cap = {}
        self.counts = device.zeros((3,), torch.int64)
        self.summaries = device.zeros((3, 4), torch.int64)
        for k in CHANNELS:
            n = _nblk(*self.shapes[k])
            if out is not None:
                self.coef[k], self.dc[k] = out[k]
                if tuple(self.coef[k].shape) != (n, 64) or tuple(self.dc[k].shape) != (n,):
                    raise ValueError("out[%s]: expected (%d, 64) / (%d,) views" % (k, n, n))
            else:
                self.coef[k] = device.empty((n, 64), torch.int16)
                self.dc[k] = device.empty((n,), torch.int32)
            # a shard's stream can open with the fillers of a zero run carried from every
            # block before it (a flat previous shard): room for those too
            lead = (r0 // (8 if k == "lum" else 16)) * -(-self.shapes[k][1] // 8)
            self.cap[k] = n * 63 + 1 + (lead * 63 // max_len if max_len > 0 else 1)
            self.sym_len[k] = device.empty((self.cap[k],), torch.uint8)
            self.sym_val[k] = device.empty((self.cap[k],), torch.int16)
            # a whole image's row-segment records outnumber its 64-block tiles when the
            # image is narrow (W <= ~350): size by the records
            rowb = -(-self.shapes[k][1] // 8)
            self.ws_bytes[k] = (lib.hic_rle_rows_workspace_bytes(n, rowb, self.rpt[k]) if self.seg
                                else lib.hic_rle_workspace_bytes(n, 64))
            self.ws[k] = device.workspace(self.ws_bytes[k])
        if self.slots:
            # the slot layout: slots of 63 symbols per block, the close's record index
            # (4 int32 per record), the records + their last DCs in the workspace
            self.slot_len, self.slot_val, self.sidx = {}, {}, {}
            for k in CHANNELS:
                n = self.coef[k].shape[0]
                self.slot_len[k] = device.empty((n * 63,), torch.uint8)
                self.slot_val[k] = device.empty((n * 63,), torch.int16)
                self.sidx[k] = device.empty((4 * (n * self.rpt[k] // 64),), torch.int32)
                self.ws_bytes[k] = lib.hic_rle_slots_workspace_bytes(n, self.rpt[k])
                self.ws[k] = device.workspace(self.ws_bytes[k])
            self._mat_status = device.zeros((3,), torch.int64)
            self.index = SlotIndex(self)
            return
        # index=True: the encoder-side tile index a device decoder reads
        # (Decoder.decode(..., index=enc.index)): 3 int64 per 64-block tile
        self.index = ({k: device.empty((3 * -(-self.coef[k].shape[0] // 64),), torch.int64) for k in CHANNELS}
                      if self.want_index else None)

    @property
    def pixels(self):
        return (self.rows[1] - self.rows[0]) * self.W

    def input_span(self):
        """Image rows [in0, in1) this encoder reads: its rows plus the pyrDown halo."""
        return input_span(self.H, *self.rows)

    def transform(self, rgb, stream=None, in_row0=None, dct_events=None):
        """Steps 1-2: colour + 4:2:0 + DCT/quantize/zig-zag of the three planes.
        rgb holds image rows [in_row0, in_row0 + rgb.shape[0]) (default: the
        whole image for an unsharded encoder, input_span() for a shard)."""
        if self.landing:
            raise RuntimeError("a landing-zone Encoder does not transform")
        s = device.stream_ptr(stream)
        if in_row0 is None:
            in_row0 = 0 if self.rows == (0, self.H) else self.input_span()[0]
        r0, r1 = self.rows
        ev = (dct_events.start, dct_events.stop) if dct_events is not None else (None, None)
        if self.slots:
            # colour + pyrDown + DCT/quantize/zig-zag + the records' symbols and DC
            # differences, in ONE launch (slots.h): no coefficients reach HBM
            if in_row0 != 0 or rgb.shape[0] != self.H:
                raise ValueError("a slot-layout encoder takes the whole image")
            _lib.call("hic_encode420_slots_u8", device.ptr(rgb), self.H, self.W, self._slot_jobs(), self.max_len, s,
                      *ev)
            return
        if self.fused:
            # colour + pyrDown + DCT/quantize/zig-zag of the three planes + RLE tile
            # records in ONE launch (dct_events time it)
            rgb, in_row0 = self._fused_input(rgb, in_row0)
            coefs = [device.ptr(self.coef[k]) for k in CHANNELS]
            wss = [device.ptr(self.ws[k]) for k in CHANNELS]
            if self.seg:
                _lib.call("hic_encode420_seg_u8", device.ptr(rgb), in_row0, rgb.shape[0], self.H, self.W, r0, r1 - r0,
                          *coefs, *wss, self.ws_bytes["lum"], min(self.ws_bytes["cr"], self.ws_bytes["cb"]),
                          self.max_len, s, *ev)
            else:
                _lib.call("hic_encode420_u8", device.ptr(rgb), in_row0, rgb.shape[0], self.H, self.W, r0, r1 - r0,
                          *coefs, *wss, self.max_len, s, *ev)
            return
        _lib.call("hic_rgb_to_ycrcb420_rows", device.ptr(rgb), in_row0, rgb.shape[0], self.H, self.W, r0, r1 - r0,
                  device.ptr(self.y), device.ptr(self.cr), device.ptr(self.cb), s)
        # DCT + quantize + zig-zag of the three planes in ONE launch (each plane with
        # its own table), with the RLE tile pass fused into its epilogue; dct_events
        # (device.KernelEvents) receive the launch's own begin / end timestamps
        jobs = (_lib.DctPlaneJob * 3)()
        for i, k in enumerate(CHANNELS):
            h, w = self.shapes[k]
            p = self.planes[k]
            jobs[i] = _lib.DctPlaneJob(p.data_ptr(), h, w, p.stride(0), TABLES[k], self.coef[k].data_ptr(),
                                       self.ws[k].data_ptr())
        _lib.call("hic_dct_quant_rle_u8_batch", 3, jobs, self.max_len, s, *ev)

    def _fused_input(self, rgb, in_row0):
        """The fused kernel addresses its input rows with 32-bit offsets: hand it the
        span it reads (< 2 GiB by can_fuse) when the caller passes more rows."""
        a, b = self.input_span()
        if rgb.shape[0] * self.W * 3 > 2**31 - 1 and in_row0 <= a and in_row0 + rgb.shape[0] >= b:
            rgb, in_row0 = rgb[a - in_row0:b - in_row0], a
        return rgb, in_row0

    def batchable(self):
        """Whether transform_batch can take this encoder into a batched launch."""
        return (self.fused and not self.slots and not self.seg and not self.landing and self.W % 512 == 0)

    def _slot_jobs(self):
        jobs = (_lib.SlotJob * 3)()
        for i, k in enumerate(CHANNELS):
            jobs[i] = _lib.SlotJob(self.coef[k].shape[0], self.rpt[k], self.slot_len[k].data_ptr(),
                                   self.slot_val[k].data_ptr(), self.dc[k].data_ptr(), self.sidx[k].data_ptr(),
                                   self.ws[k].data_ptr(), self.ws_bytes[k], self.counts[i:i + 1].data_ptr(),
                                   self.sym_len[k].data_ptr(), self.sym_val[k].data_ptr(), self.cap[k])
        return jobs

    def compact(self, stream=None):
        """Slot layout: the contiguous symbol stream into sym_len / sym_val (what the
        emit writes; hic_rle_slots_compact).  A no-op for the coefficient chain."""
        if self.slots:
            _lib.call("hic_rle_slots_compact", 3, self._slot_jobs(), self.max_len, device.stream_ptr(stream))

    def materialize(self, stream=None):
        """Slot layout: the contiguous stream and the zig-zag blocks (self.coef,
        decoded from the slots: hic_rle_decode_i16_slots), as the coefficient chain
        leaves them.  A no-op for the coefficient chain."""
        if not self.slots:
            return
        self.compact(stream)
        s = device.stream_ptr(stream)
        for i, k in enumerate(CHANNELS):
            _lib.call("hic_rle_decode_i16_slots", device.ptr(self.slot_len[k]), device.ptr(self.slot_val[k]),
                      ctypes.c_void_p(self.counts.data_ptr() + 8 * i), device.ptr(self.dc[k]), self.coef[k].shape[0],
                      self.rpt[k], device.ptr(self.sidx[k]), device.ptr(self.coef[k]),
                      device.ptr(self._mat_status[i:i + 1]), s)

    def shard_summaries(self, stream=None):
        """Per-channel {trailing zeros, has nonzero, first DC, last DC} (sharded encode)."""
        if self.slots:
            raise ValueError("shard summaries are for row shards (a slot-layout encoder is a whole image)")
        if self.seg:
            raise ValueError("shard summaries read 64-block tile records (a row shard's); this whole-image "
                             "encoder keeps one per strip segment")
        s = device.stream_ptr(stream)
        for i, k in enumerate(CHANNELS):
            n = self.coef[k].shape[0]
            _lib.call("hic_rle_shard_summary_records", device.ptr(self.coef[k]), n, self.rpt[k], device.ptr(self.ws[k]),
                      device.ptr(self.summaries[i]), s)
        return self.summaries

    def entropy(self, stream=None, stitch=None):
        """Step 3: DC DPCM + AC RLE of the three channels (one scan launch and one
        emit launch for all three).  stitch: None or a (3, 4) int64 device tensor of
        per-channel {carry_zeros, emit_eob, has_prev_dc, prev_dc}."""
        s = device.stream_ptr(stream)
        if self.slots:
            if stitch is not None:
                raise ValueError("a slot-layout encoder is a whole image (no stitch)")
            _lib.call("hic_rle_slots_close", 3, self._slot_jobs(), self.max_len, s)
            return
        if self.seg:
            rowb = (ctypes.c_int64 * 3)(self.W // 8, self.W // 16, self.W // 16)
            _lib.call("hic_rle_encode_i16_rows_batch", 3, self._rle_jobs(stitch), rowb, self.max_len, s)
        else:
            # with a tile index wanted, the emit writes it too (hic_rle_job16.d_index:
            # hic_rle_tile_index_i16's words, no launch of its own)
            _lib.call("hic_rle_encode_i16_tiles_batch", 3, self._rle_jobs(stitch, index=True), self.max_len, s)

    def encode(self, rgb, stream=None, dct_events=None):
        self.transform(rgb, stream, dct_events=dct_events)
        self.entropy(stream)

    def _rle_jobs(self, stitch, index=False):
        jobs = (_lib.RleJob16 * 3)()
        for i, k in enumerate(CHANNELS):
            ix = self.index[k].data_ptr() if index and self.index is not None and stitch is None else None
            jobs[i] = _lib.RleJob16(self.coef[k].data_ptr(), self.coef[k].shape[0],
                                    stitch[i].data_ptr() if stitch is not None else None, self.dc[k].data_ptr(),
                                    self.sym_len[k].data_ptr(), self.sym_val[k].data_ptr(), self.cap[k],
                                    self.counts[i:i + 1].data_ptr(), self.ws[k].data_ptr(), self.rpt[k],
                                    self.ws_bytes[k], ix)
        return jobs

    def hic_image(self, stream=None):
        """codec.jpeg_encode of this encode, from the device streams: the nine Huffman
        trees from GPU key histograms, the nine bit strings packed on the GPU
        (huffman.DeviceStreams); == codec.jpeg_encode(the encoded CompressedImage)
        for an unsharded encoder (syncs)."""
        from . import hicimage as hic
        from . import huffman
        if self.rows != (0, self.H):
            raise ValueError("hic_image needs the whole image (an unsharded encoder)")
        self.compact(stream)
        with device.on_stream(stream):  # the counts and histograms are read after the stream's kernels
            return self._hic_image(stream)

    def _hic_image(self, stream):
        from . import hicimage as hic
        from . import huffman
        counts = self.counts.cpu().tolist()
        keys = {}
        for i, k in enumerate(CHANNELS):
            check_count(int(counts[i]), k)
            c = int(counts[i])
            keys[k] = ((self.dc[k], self.dc[k].numel()), (self.sym_val[k], c), (self.sym_len[k], c))
        # the nine streams in payload order, their host round trips batched
        order = [(k, j) for j in range(3) for k in CHANNELS]
        ds = huffman.DeviceStreams([keys[k][j] for k, j in order], stream=stream)
        # DC keys as the reference holds them (numpy int32: dct_channel's dtype)
        tables = [hic.PayloadStringP(hic.TupP, [hic.TupP(np.int32(v) if j == 0 else int(v), c)
                                                for v, c in ds.trees[i].encode_table()])
                  for i, (k, j) in enumerate(order)]
        data = [hic.BitStringP.from_packed(*pk) for pk in ds.packed()]
        (h, w), (hc, wc) = self.shapes["lum"], self.shapes["cr"]
        return hic.HicImage.jpeg_image(tables + data + [hic.TupP(h, w), hic.TupP(hc, wc)])

    def result(self):
        """Host copies: {channel: (zigzag blocks, dc_diff, sym_len, sym_val)} (syncs;
        a slot-layout encoder materializes its stream and blocks first)."""
        self.materialize()
        device.sync()
        counts = self.counts.cpu().numpy()
        out = {}
        for i, k in enumerate(CHANNELS):
            c = int(counts[i])
            check_count(c, k)
            out[k] = (self.coef[k].cpu().numpy(), self.dc[k].cpu().numpy(), self.sym_len[k][:c].cpu().numpy(),
                      self.sym_val[k][:c].cpu().numpy())
        return out


def transform_batch(encoders, inputs, stream=None, in_row0s=None, dct_events=None):
    """Encoder.transform of several encoders -- the row shards of a multi-GPU group,
    one per image -- in ONE launch (hic_encode420_batch_u8) when every one is a fused
    coefficient encoder whose records its kernel writes (Encoder.batchable) and at
    most 8 share one max_len; else one transform each.  A shard is 1/N of an image,
    too few waves to fill the chip alone: at N = 8 eight launches in a row took 2.4x
    one whole-image launch.  dct_events (per encoder, None or device.KernelEvents):
    each pair spans the batched launch."""
    n = len(encoders)
    in_row0s = in_row0s if in_row0s is not None else [None] * n
    dct_events = dct_events if dct_events is not None else [None] * n
    if not (2 <= n <= 8 and all(e.batchable() for e in encoders)
            and len(set(e.max_len for e in encoders)) == 1):
        for e, x, r, ev in zip(encoders, inputs, in_row0s, dct_events):
            e.transform(x, stream, in_row0=r, dct_events=ev)
        return
    jobs = (_lib.Encode420Job * n)()
    for i, (e, x, r) in enumerate(zip(encoders, inputs, in_row0s)):
        if r is None:
            r = 0 if e.rows == (0, e.H) else e.input_span()[0]
        x, r = e._fused_input(x, r)
        r0, r1 = e.rows
        jobs[i] = _lib.Encode420Job(x.data_ptr(), r, x.shape[0], e.H, e.W, r0, r1 - r0,
                                    *(e.coef[k].data_ptr() for k in CHANNELS), *(e.ws[k].data_ptr() for k in CHANNELS))
    s = device.stream_ptr(stream)
    evs = [ev for ev in dct_events if ev is not None]
    for ev in evs[1:]:
        _lib.call("hic_event_record", ev.start, s)
    first = (evs[0].start, evs[0].stop) if evs else (None, None)
    _lib.call("hic_encode420_batch_u8", n, jobs, encoders[0].max_len, s, *first)
    for ev in evs[1:]:
        _lib.call("hic_event_record", ev.stop, s)


class Decoder:
    """Inverse chain: symbols -> zig-zag blocks -> pixels -> RGB (2h x 2w x 3)."""

    def __init__(self, H, W, chroma_pair=True):
        """chroma_pair: the indexed decode's Cr and Cb in one launch
        (hic_rle_decode_idct_u8_indexed_pair); False: one launch each."""
        device.require_gpu()
        self.H, self.W = H, W
        self.chroma_pair = chroma_pair
        self.shapes = {"lum": (H, W), "cr": (H // 2, W // 2), "cb": (H // 2, W // 2)}
        self.blocks, self.pix, self.status = {}, {}, device.zeros((3,), torch.int64)
        for k in CHANNELS:
            h, w = self.shapes[k]
            self.blocks[k] = device.empty((_nblk(h, w), 64), torch.int16)
            self.pix[k] = device.empty((h, w), torch.uint8)
        self.rgb = device.empty((2 * (H // 2), 2 * (W // 2), 3), torch.uint8)
        self._ws = {}

    def decode(self, sym_len, sym_val, counts, dc, stream=None, index=None, keep_blocks=False, planes=False):
        """sym_len/sym_val/dc: {channel: device tensor}; counts: host ints per channel.
        index: an Encoder(index=True)'s tile index ({channel: device tensor}); then
        counts is the encoder's device count tensor (3,), nothing crosses to the
        host, and each plane is decoded and inverse-transformed by ONE kernel
        (hic_rle_decode_idct_u8_indexed: no tile pass, scans, DC chain or zig-zag
        blocks in HBM); keep_blocks=True writes self.blocks too (the block-level
        indexed decode, then the IDCT).  With the index and whole 8x8 blocks (H, W
        multiples of 8) the chroma planes decode first and the luminance plane goes
        straight to RGB (hic_rle_decode_idct_rgb_indexed: self.pix["lum"] is not
        written); planes=True keeps the Y plane and the separate colour kernel."""
        s = device.stream_ptr(stream)
        lib = _lib.load()
        if isinstance(index, SlotIndex):
            return self._decode_slots(index, counts, dc, s, keep_blocks, planes)
        if index is not None and not keep_blocks and not planes and self.H % 8 == 0 and self.W % 8 == 0:
            # Cr and Cb in one launch (one tail), then Y straight to RGB
            h, w = self.shapes["cr"]
            if self.chroma_pair:
                pair = lambda f: (ctypes.c_void_p * 2)(*(f(i, k) for i, k in ((1, "cr"), (2, "cb"))))
                _lib.call("hic_rle_decode_idct_u8_indexed_pair", pair(lambda i, k: sym_len[k].data_ptr()),
                          pair(lambda i, k: sym_val[k].data_ptr()), pair(lambda i, k: counts.data_ptr() + 8 * i),
                          pair(lambda i, k: dc[k].data_ptr()), pair(lambda i, k: index[k].data_ptr()), h, w,
                          TABLES["cr"], pair(lambda i, k: self.pix[k].data_ptr()), self.pix["cr"].stride(0),
                          pair(lambda i, k: self.status[i:i + 1].data_ptr()), s)
            else:
                for i, k in ((1, "cr"), (2, "cb")):
                    _lib.call("hic_rle_decode_idct_u8_indexed", device.ptr(sym_len[k]), device.ptr(sym_val[k]),
                              ctypes.c_void_p(counts.data_ptr() + 8 * i), device.ptr(dc[k]), device.ptr(index[k]),
                              h, w, TABLES[k], device.ptr(self.pix[k]), self.pix[k].stride(0),
                              device.ptr(self.status[i:i + 1]), s)
            _lib.call("hic_rle_decode_idct_rgb_indexed", device.ptr(sym_len["lum"]), device.ptr(sym_val["lum"]),
                      ctypes.c_void_p(counts.data_ptr()), device.ptr(dc["lum"]), device.ptr(index["lum"]), self.H,
                      self.W, device.ptr(self.pix["cr"]), device.ptr(self.pix["cb"]), device.ptr(self.rgb),
                      self.rgb.stride(0), device.ptr(self.status[0:1]), s)
            return self.rgb
        for i, k in enumerate(CHANNELS):
            h, w = self.shapes[k]
            n = self.blocks[k].shape[0]
            if index is not None and not keep_blocks:
                _lib.call("hic_rle_decode_idct_u8_indexed", device.ptr(sym_len[k]), device.ptr(sym_val[k]),
                          ctypes.c_void_p(counts.data_ptr() + 8 * i), device.ptr(dc[k]), device.ptr(index[k]), h, w,
                          TABLES[k], device.ptr(self.pix[k]), self.pix[k].stride(0),
                          device.ptr(self.status[i:i + 1]), s)
                continue
            if index is not None:
                _lib.call("hic_rle_decode_i16_indexed", device.ptr(sym_len[k]), device.ptr(sym_val[k]),
                          ctypes.c_void_p(counts.data_ptr() + 8 * i), device.ptr(dc[k]), n, device.ptr(index[k]),
                          device.ptr(self.blocks[k]), device.ptr(self.status[i:i + 1]), s)
            else:
                nsym = int(counts[i])
                need = lib.hic_rld_workspace_bytes(nsym, n)
                if k not in self._ws or self._ws[k].numel() * 8 < need:
                    self._ws[k] = device.workspace(need)
                _lib.call("hic_rle_decode_i16", device.ptr(sym_len[k]), device.ptr(sym_val[k]), nsym,
                          device.ptr(dc[k]), n, 64, device.ptr(self.blocks[k]), device.ptr(self.status[i:i + 1]),
                          device.ptr(self._ws[k]), s)
            _lib.call("hic_dequant_idct_u8", device.ptr(self.blocks[k]), _lib.LAYOUT_ZIGZAG_I16, h, w, TABLES[k],
                      device.ptr(self.pix[k]), self.pix[k].stride(0), s)
        h, w = self.shapes["cr"]
        _lib.call("hic_ycrcb420_to_rgb", device.ptr(self.pix["lum"]), self.pix["lum"].stride(0),
                  device.ptr(self.pix["cr"]), device.ptr(self.pix["cb"]), h, w, device.ptr(self.rgb), s)
        return self.rgb

    def _decode_slots(self, ix, counts, dc, s, keep_blocks, planes):
        """decode() from a slot-layout encoder's stream (SlotIndex): the *_slots forms of
        the indexed decoders."""
        cnt = lambda i: ctypes.c_void_p(counts.data_ptr() + 8 * i)  # noqa: E731
        if not keep_blocks and not planes and self.H % 8 == 0 and self.W % 8 == 0:
            h, w = self.shapes["cr"]
            if self.chroma_pair:
                pair = lambda f: (ctypes.c_void_p * 2)(*(f(i, k) for i, k in ((1, "cr"), (2, "cb"))))  # noqa: E731
                _lib.call("hic_rle_decode_idct_u8_slots_pair", pair(lambda i, k: ix.slot_len[k].data_ptr()),
                          pair(lambda i, k: ix.slot_val[k].data_ptr()), pair(lambda i, k: counts.data_ptr() + 8 * i),
                          pair(lambda i, k: dc[k].data_ptr()), pair(lambda i, k: ix.sidx[k].data_ptr()), ix.rpt["cr"],
                          h, w, TABLES["cr"], pair(lambda i, k: self.pix[k].data_ptr()), self.pix["cr"].stride(0),
                          pair(lambda i, k: self.status[i:i + 1].data_ptr()), s)
            else:
                for i, k in ((1, "cr"), (2, "cb")):
                    _lib.call("hic_rle_decode_idct_u8_slots", device.ptr(ix.slot_len[k]), device.ptr(ix.slot_val[k]),
                              cnt(i), device.ptr(dc[k]), device.ptr(ix.sidx[k]), ix.rpt[k], h, w, TABLES[k],
                              device.ptr(self.pix[k]), self.pix[k].stride(0), device.ptr(self.status[i:i + 1]), s)
            _lib.call("hic_rle_decode_idct_rgb_slots", device.ptr(ix.slot_len["lum"]), device.ptr(ix.slot_val["lum"]),
                      cnt(0), device.ptr(dc["lum"]), device.ptr(ix.sidx["lum"]), ix.rpt["lum"], self.H, self.W,
                      device.ptr(self.pix["cr"]), device.ptr(self.pix["cb"]), device.ptr(self.rgb),
                      self.rgb.stride(0), device.ptr(self.status[0:1]), s)
            return self.rgb
        for i, k in enumerate(CHANNELS):
            h, w = self.shapes[k]
            if keep_blocks:
                _lib.call("hic_rle_decode_i16_slots", device.ptr(ix.slot_len[k]), device.ptr(ix.slot_val[k]), cnt(i),
                          device.ptr(dc[k]), self.blocks[k].shape[0], ix.rpt[k], device.ptr(ix.sidx[k]),
                          device.ptr(self.blocks[k]), device.ptr(self.status[i:i + 1]), s)
                _lib.call("hic_dequant_idct_u8", device.ptr(self.blocks[k]), _lib.LAYOUT_ZIGZAG_I16, h, w, TABLES[k],
                          device.ptr(self.pix[k]), self.pix[k].stride(0), s)
            else:
                _lib.call("hic_rle_decode_idct_u8_slots", device.ptr(ix.slot_len[k]), device.ptr(ix.slot_val[k]),
                          cnt(i), device.ptr(dc[k]), device.ptr(ix.sidx[k]), ix.rpt[k], h, w, TABLES[k],
                          device.ptr(self.pix[k]), self.pix[k].stride(0), device.ptr(self.status[i:i + 1]), s)
        h, w = self.shapes["cr"]
        _lib.call("hic_ycrcb420_to_rgb", device.ptr(self.pix["lum"]), self.pix["lum"].stride(0),
                  device.ptr(self.pix["cr"]), device.ptr(self.pix["cb"]), h, w, device.ptr(self.rgb), s)
        return self.rgb

    def check_status(self):
        """Raise unless every channel's stream decoded to exactly its blocks' AC
        positions (codec.jpeg_decode's length check, codec.py:418-419; syncs)."""
        st = self.status.cpu().tolist()
        for i, k in enumerate(CHANNELS):
            want = self.blocks[k].shape[0] * 63
            if st[i] != want:
                raise ValueError("channel %s: stream covers %d AC positions, expected %d" % (k, st[i], want))
