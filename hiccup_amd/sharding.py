"""Tile-sharded multi-GPU encode: one process per GPU, RCCL over xGMI.

The image is split into contiguous row ranges (multiples of 16 rows, so Y and
4:2:0 chroma block rows align).  Every 8x8 block is independent through colour
conversion, DCT, quantisation and zig-zag, so each rank transforms its shard with
no communication (its input carries the 2-row pyrDown halo).  The reference's
entropy front end is ONE sequential pass over each channel's stream
(codec.py:47-99): the DC DPCM chain and the AC run-length state cross shard
boundaries and only the last shard emits the EOB.  That is the one real exchange
step, and it is tiny: each rank all-gathers a 4-word summary per channel
{trailing zeros, has-nonzero, first DC, last DC}, derives its stitch record
{carry zeros, emits EOB, has previous DC, previous DC} (hic_rle_stitch, on the
device), and then emits exactly the symbols of its slice of the single-GPU
stream.  A second all-gather of the per-channel symbol counts gives every rank its
global offsets.

Reassembly on one rank (north_star's "single RCCL gather"): every rank's
zig-zag coefficient blocks and DC differences are a contiguous slice of the whole
image's (block-row shards, raster block order), and their sizes follow from the
shard plan alone.  ``ShardEncoder.gather_coefficients`` therefore moves them with
ONE grouped point-to-point batch (``dist.batch_isend_irecv``: an RCCL group of
sends / receives on the encode stream) straight into the gathering rank's
whole-image buffers -- no host synchronisation, no sizes exchanged first.  The
gathering rank's own encoder writes into its slice of those buffers in place.
``gather_streams`` (tests, tools) also collects the variable-length symbol
streams; it needs the counts on the host.
"""
import ctypes
import weakref

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, device, pipeline

CHANNELS = pipeline.CHANNELS


def plan(H, world, align=16):
    """Row ranges [(r0, r1)] per rank: contiguous, multiples of `align` rows except
    the image's ragged end, as even as possible."""
    units = -(-H // align)
    if units < world:
        raise ValueError("image too small: %d rows for %d ranks" % (H, world))
    out = []
    for r in range(world):
        u0, u1 = units * r // world, units * (r + 1) // world
        out.append((u0 * align, min(H, u1 * align)))
    return out


def stitch_host(summaries, rank):
    """Host restatement of hic_rle_stitch: summaries (world, 4) per channel."""
    s = np.asarray(summaries, dtype=np.int64)
    world = len(s)
    carry = 0
    for r in range(rank - 1, -1, -1):
        carry += int(s[r, 0])
        if s[r, 1]:
            break
    return np.array([carry, int(rank == world - 1), int(rank > 0), int(s[rank - 1, 3]) if rank > 0 else 0],
                    dtype=np.int64)


def _all_gather(out_flat, inp, group=None):
    """all_gather_into_tensor; gloo (CPU rehearsal of the multi-GPU path) cannot
    gather device tensors, so there they are staged through host memory."""
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(out_flat.shape, dtype=out_flat.dtype)
        dist.all_gather_into_tensor(host, inp.detach().cpu().contiguous(), group=group)
        out_flat.copy_(host)
    else:
        dist.all_gather_into_tensor(out_flat, inp.contiguous(), group=group)


def exchange(summ_local, world, group=None):
    """All-gather every rank's (3, 4) channel summaries -> (world, 3, 4): the one
    collective of the sharded encode (RCCL on GPU tensors, gloo on CPU ones)."""
    shape = tuple(summ_local.shape)
    out = torch.empty((world * shape[0],) + shape[1:], dtype=summ_local.dtype, device=summ_local.device)
    _all_gather(out, summ_local, group=group)
    return out.view((world,) + shape)


def block_ranges(H, W, world):
    """{channel: [(b0, b1)] per rank}: each rank's blocks in the whole image's
    raster block order (4:2:0 chroma planes are (H/2) x (W/2))."""
    out = {}
    for k in CHANNELS:
        h, w = (H, W) if k == "lum" else (H // 2, W // 2)
        nbx = -(-w // 8)
        rr = []
        for r0, r1 in plan(H, world):
            if k == "lum":
                a, b = r0, r1
            else:
                a, b = r0 // 2, min(h, r1 // 2)
            rr.append(((a // 8) * nbx, -(-b // 8) * nbx))
        out[k] = rr
    return out


REC_BYTES = 24  # one RLE tile record: 3 int64
TRAILER_BYTES = 16  # a stream-gather segment's trailer: the sender's int32 out-of-width flag, padded
TABLE_OF = {"lum": 0, "cr": 1, "cb": 1}  # the plane's quantisation table (the wire widths follow it)


def wire_ranges(ranges, rpt, records):
    """{channel: [(o0, o1)]}: rank r's byte segment of the whole image's wire buffer
    -- its blocks in the wire format (hic_wire_bytes) followed, when `records`, by
    its RLE tile records already rebased to whole-image positions (REC_BYTES each,
    rpt records per 64 blocks, padded to a multiple of 16 bytes), then a
    TRAILER_BYTES trailer whose first int32 is the sender's out-of-width flag."""
    lib = _lib.load()
    out = {}
    for k in CHANNELS:
        o, rr = 0, []
        for b0, b1 in ranges[k]:
            n = b1 - b0
            # (the records padded to 16 bytes: every segment starts 16-byte aligned)
            size = lib.hic_wire_bytes(n, TABLE_OF[k]) + (-(-(-(-n * rpt[k] // 64) * REC_BYTES) // 16) * 16
                                                            if records else 0) + TRAILER_BYTES
            rr.append((o, o + size))
            o += size
        out[k] = rr
    return out


def records_aligned(ranges, rpt):
    """Every shard starts on a record boundary of the whole image (its records can
    be rebased instead of recomputed): W % 512 == 0 on the fused path."""
    return all((b0 * rpt[k]) % 64 == 0 for k in CHANNELS for b0, _ in ranges[k])


class ShardEncoder:
    """One rank's part of a tile-sharded encode of an H x W RGB image.

    gather_to: the rank that reassembles the image; None = no reassembly buffers.
    gather_kind "blocks": every rank entropy-codes its slice of the stream
    (summaries, stitch, scan + emit) and gather_to collects the whole image's
    coefficient blocks and DC differences (gather_coefficients).
    gather_kind "stream": the ranks only transform; each ships its blocks in the
    lossless wire format (hic_wire_pack_i16: per-slot widths proven for the
    plane's table, 637 / 597 bits per block) plus its rebased RLE tile
    records to gather_to, which unpacks them and runs the scan + emit of the whole
    image -- codec.jpeg_encode's single stream (codec.py:55-99,286-301) ends on
    gather_to (self.whole.sym_len / sym_val / dc / counts), with no host sync and
    no per-shard entropy pass.  See stream_item / pack / finish."""

    def __init__(self, H, W, rank=None, world=None, group=None, max_len=15, gather_to=None, fused=None,
                 gather_kind="blocks"):
        if gather_kind not in ("blocks", "stream"):
            raise ValueError("gather_kind must be 'blocks' or 'stream'")
        if gather_kind == "stream" and gather_to is None:
            raise ValueError("gather_kind 'stream' needs gather_to")
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        self.group = group
        self.H, self.W = H, W
        self.rows = plan(H, self.world)[self.rank]
        self.ranges = block_ranges(H, W, self.world)
        self.gather_to = gather_to
        self.gather_kind = gather_kind
        if fused is None:
            # one decision for every rank (the record layout of the whole stream
            # depends on it): fused only if every shard can run the fused kernel
            fused = all(pipeline.encoder_layout(H, W, rr)[0] for rr in plan(H, self.world))
        self.whole = None
        out = None
        if gather_to is not None and self.rank == gather_to:
            if gather_kind == "stream":
                # the whole image's entropy stage lives here: its buffers are the
                # landing zone, this rank's encoder writes its slice in place.  Its
                # RLE records follow the SHARDS' layout (wire_ranges sizes and packs
                # them with it): a whole image past 2 GiB of input cannot run the fused
                # kernel, its shards can, and their chroma records are half tiles
                self.whole = pipeline.Encoder(H, W, max_len=max_len,
                                              landing_rpt=pipeline.encoder_layout(H, W, self.rows, fused)[1])
                self.full_coef, self.full_dc = self.whole.coef, self.whole.dc
            else:
                self.full_coef, self.full_dc = {}, {}
                for k in CHANNELS:
                    n = self.ranges[k][-1][1]
                    self.full_coef[k] = device.empty((n, 64), torch.int16)
                    self.full_dc[k] = device.empty((n,), torch.int32)
            out = {}
            for k in CHANNELS:
                b0, b1 = self.ranges[k][self.rank]
                out[k] = (self.full_coef[k][b0:b1], self.full_dc[k][b0:b1])
        self.enc = pipeline.Encoder(H, W, max_len=max_len, rows=self.rows, out=out, fused=fused)
        self.span = self.enc.input_span()
        self.all_summ = device.zeros((self.world, 3, 4), torch.int64)
        self.stitch = device.zeros((3, 4), torch.int64)
        self.all_counts = device.zeros((self.world, 3), torch.int64)
        if gather_kind == "stream":
            self.records = records_aligned(self.ranges, self.enc.rpt)
            self.wranges = wire_ranges(self.ranges, self.enc.rpt, self.records)
            if self.rank == gather_to:
                self.wire_full = {k: device.empty((self.wranges[k][-1][1],), torch.uint8) for k in CHANNELS}
                self.wire_send = None
            else:
                self.wire_full = None
                self.wire_send = {k: device.empty((self.wranges[k][self.rank][1] - self.wranges[k][self.rank][0],),
                                                  torch.uint8) for k in CHANNELS}

    @property
    def wire_flag(self):
        """The out-of-width flag this rank's pack raised (the trailer of its segment;
        0 on the gathering rank, whose blocks never travel)."""
        if self.wire_send is None:
            return device.zeros((1,), torch.int32)
        return self.wire_send["lum"][-TRAILER_BYTES:].view(torch.int32)[:1] | \
            self.wire_send["cr"][-TRAILER_BYTES:].view(torch.int32)[:1] | \
            self.wire_send["cb"][-TRAILER_BYTES:].view(torch.int32)[:1]

    @property
    def wire_bytes(self):
        """Bytes of one image on the wire (every rank's segments, all channels)."""
        return sum(self.wranges[k][-1][1] for k in CHANNELS) if self.gather_kind == "stream" else None

    def pack(self, stream=None):
        """gather_kind "stream", a rank other than gather_to: this rank's blocks into
        the wire format and its tile records, rebased, behind them (on `stream`)."""
        wire_batch("hic_wire_pack_batch", self.pack_jobs(), stream)

    def pack_jobs(self):
        """hic_wire_job per channel of pack(): the blocks into the wire segment, the
        flag in its trailer (cleared by the pack), the records rebased behind the
        blocks.  The buffers are this encoder's for its lifetime: built once."""
        if getattr(self, "_pack_jobs", None) is None:
            self._pack_jobs = self._make_pack_jobs()
        return self._pack_jobs

    def _make_pack_jobs(self):
        lib = _lib.load()
        jobs = []
        for k in CHANNELS:
            b0, b1 = self.ranges[k][self.rank]
            n = b1 - b0
            w = self.wire_send[k]
            wb = lib.hic_wire_bytes(n, TABLE_OF[k])
            nrec = -(-n * self.enc.rpt[k] // 64) if self.records else 0
            jobs.append(_lib.WireJob(self.enc.coef[k].data_ptr(), w.data_ptr(), n, TABLE_OF[k],
                                     w.data_ptr() + w.numel() - TRAILER_BYTES,
                                     self.enc.ws[k].data_ptr() if nrec else None, nrec, b0 * 63,
                                     w.data_ptr() + wb if nrec else None, None))
        return jobs

    def stream_item(self):
        """(mine, full, ranges, dst) of this image's wire gather for
        gather_blocks_group / RcclGather.gather_group (byte tensors, byte ranges)."""
        if self.wire_send is not None:
            mine, full = {k: (self.wire_send[k],) for k in CHANNELS}, None
        else:  # gather_to: its own segment is never sent (the C-ABI sees it in place)
            mine = {k: (self.wire_full[k][slice(*self.wranges[k][self.rank])],) for k in CHANNELS}
            full = {k: (self.wire_full[k],) for k in CHANNELS}
        return mine, full, self.wranges, self.gather_to

    def finish(self, stream=None):
        """gather_to, after the wire gather: every other rank's blocks unpacked into
        the whole image, the tile records placed (or, when the shards do not start
        on record boundaries, recomputed by a tile pass), then the whole image's
        scan + emit (one stream, no stitch).  On `stream`."""
        s = device.stream_ptr(stream)
        whole = self.whole
        if whole.rpt != self.enc.rpt:
            raise RuntimeError("landing zone record layout %r != the shards' %r" % (whole.rpt, self.enc.rpt))
        if getattr(self, "_finish_jobs", None) is None:  # fixed buffers: built once
            self._finish_jobs = self._make_finish_jobs()
        jobs, flags = self._finish_jobs
        if jobs:
            _lib.call("hic_wire_unpack_batch", len(jobs), jobs, s)
        if not self.records:
            for k in CHANNELS:
                _lib.call("hic_rle_tile_records_i16", device.ptr(whole.coef[k]), whole.coef[k].shape[0],
                          whole.max_len, device.ptr(whole.ws[k]), s)
        whole.entropy(stream)
        # the senders' flags override the counts after the scan (HIC_COUNT_WIRE_OVERFLOW):
        # one launch on `stream`, no host sync
        if flags:
            _lib.call("hic_wire_flags_apply", len(flags), flags, s)

    def _make_finish_jobs(self):
        """finish()'s batches as ctypes arrays: every other rank's segments unpacked
        and every rank's records placed (hic_wire_unpack_batch: 3 launches for all
        channels and peers), and the senders' flags -> counts."""
        lib = _lib.load()
        whole = self.whole
        jobs, flags = [], []
        for c, k in enumerate(CHANNELS):
            rpt = self.enc.rpt[k]  # the layout wire_ranges sized the segments with
            for r in range(self.world):
                b0, b1 = self.ranges[k][r]
                n = b1 - b0
                nrec = -(-n * rpt // 64) if self.records else 0
                dst_rec = whole.ws[k].data_ptr() + (b0 * rpt // 64) * REC_BYTES
                if r == self.rank:
                    if nrec:
                        jobs.append(_lib.WireJob(None, None, 0, TABLE_OF[k], None, self.enc.ws[k].data_ptr(), nrec,
                                                 b0 * 63, dst_rec, None))
                    continue
                o0, o1 = self.wranges[k][r]
                seg = self.wire_full[k].data_ptr() + o0
                jobs.append(_lib.WireJob(whole.coef[k][b0:b1].data_ptr(), seg, n, TABLE_OF[k], None,
                                         seg + lib.hic_wire_bytes(n, TABLE_OF[k]) if nrec else None, nrec, 0,
                                         dst_rec if nrec else None, None))
                # the sender's out-of-width flag (its segment's trailer) -> this channel's count
                flags.append(_lib.WireJob(None, None, 0, TABLE_OF[k], self.wire_full[k].data_ptr() + o1 - TRAILER_BYTES,
                                          None, 0, 0, None, whole.counts.data_ptr() + 8 * c))
        if len(jobs) > 32 or len(flags) > 32:
            raise ValueError("world %d: more than 32 wire segments per image" % self.world)
        return ((_lib.WireJob * len(jobs))(*jobs) if jobs else None,
                (_lib.WireJob * len(flags))(*flags) if flags else None)

    @property
    def pixels(self):
        return self.enc.pixels

    def encode(self, rgb_rows, stream=None, dct_events=None):
        """rgb_rows: device uint8 tensor of image rows self.span (shard + halo).
        Everything, the collectives included, runs in order on `stream` (RCCL
        enqueues on torch's current stream, so it is made current here)."""
        if stream is not None:
            with torch.cuda.stream(stream):
                return self._encode(rgb_rows, stream, dct_events)
        return self._encode(rgb_rows, None, dct_events)

    def _encode(self, rgb_rows, stream, dct_events):
        enc = self.enc
        enc.transform(rgb_rows, stream, in_row0=self.span[0], dct_events=dct_events)
        summ = enc.shard_summaries(stream)
        # the exchange step: 96 bytes per rank over RCCL
        _all_gather(self.all_summ.view(self.world * 3, 4), summ, group=self.group)
        s = device.stream_ptr(stream)
        for c in range(3):
            _lib.call("hic_rle_stitch", ctypes.c_void_p(self.all_summ.data_ptr() + 8 * 4 * c), self.world, self.rank,
                      12, device.ptr(self.stitch[c]), s)
        enc.entropy(stream, stitch=self.stitch)
        _all_gather(self.all_counts.view(-1), enc.counts, group=self.group)

    def offsets(self):
        """(this rank's symbol offset per channel, global totals) -- host ints (syncs)."""
        c = self.all_counts.cpu().numpy()
        for r in range(self.world):
            for ci, k in enumerate(CHANNELS):
                pipeline.check_count(int(c[r, ci]), "%s (rank %d)" % (k, r))
        return c[:self.rank].sum(0), c.sum(0)

    def gather_coefficients(self, stream=None):
        """Reassemble the whole image's zig-zag coefficient blocks and DC
        differences on rank gather_to: one grouped batch of RCCL sends / receives on
        `stream`, sized by the shard plan (no host sync).  Returns
        {channel: (coef, dc)} whole-image device tensors on gather_to, None elsewhere."""
        if self.gather_to is None:
            raise ValueError("ShardEncoder(gather_to=...) was not set")
        if stream is not None:
            with torch.cuda.stream(stream):
                return self._gather_coefficients()
        return self._gather_coefficients()

    def _gather_coefficients(self):
        mine, full, ranges, dst = self.gather_item()
        gather_blocks(mine, full, ranges, self.rank, self.world, dst, self.group)
        return full

    def gather_item(self):
        """(mine, full, ranges, dst) of this encoder's gather, for gather_blocks_group."""
        if self.gather_to is None:
            raise ValueError("ShardEncoder(gather_to=...) was not set")
        full = {k: (self.full_coef[k], self.full_dc[k]) for k in CHANNELS} if self.rank == self.gather_to else None
        mine = {k: (self.enc.coef[k], self.enc.dc[k]) for k in CHANNELS}
        return mine, full, self.ranges, self.gather_to


def encode_group(encoders, rgb_rows_list, stream=None, dct_events=None):
    """The sharded encodes of several images (one ShardEncoder each, same plan)
    with their exchange steps batched: every image's transform and channel
    summaries, ONE all-gather of all the summaries (n x 96 bytes per rank), the
    stitch records and entropy coding of every image, ONE all-gather of all the
    symbol counts.  Two small collectives per group instead of two per image: at N
    GPUs each is a latency-bound RCCL all-gather, which would otherwise bound the
    per-image time.  Equal, image by image, to ShardEncoder.encode.  dct_events:
    None or one entry (None or device.KernelEvents) per image."""
    if stream is not None:
        with torch.cuda.stream(stream):
            return _encode_group(encoders, rgb_rows_list, stream, dct_events)
    return _encode_group(encoders, rgb_rows_list, None, dct_events)


def _encode_group(encoders, rgb_rows_list, stream, dct_events):
    e0 = encoders[0]
    n, world = len(encoders), e0.world
    # the group's shard transforms in one launch (pipeline.transform_batch)
    pipeline.transform_batch([se.enc for se in encoders], rgb_rows_list, stream,
                             in_row0s=[se.span[0] for se in encoders], dct_events=dct_events)
    if all(se.gather_kind == "stream" for se in encoders):
        return  # the entropy stage runs on the gathering rank (gather_streams_group)
    summs = []
    for se in encoders:
        summs.append(se.enc.shard_summaries(stream))
    allsumm = torch.empty((world, n, 3, 4), dtype=torch.int64, device=summs[0].device)
    _all_gather(allsumm.view(world * n * 3, 4), torch.stack(summs).view(n * 3, 4), group=e0.group)
    s = device.stream_ptr(stream)
    for i, se in enumerate(encoders):
        se.all_summ.copy_(allsumm[:, i])
        for c in range(3):
            _lib.call("hic_rle_stitch", ctypes.c_void_p(se.all_summ.data_ptr() + 8 * 4 * c), world, se.rank, 12,
                      device.ptr(se.stitch[c]), s)
        se.enc.entropy(stream, stitch=se.stitch)
    allcounts = torch.empty((world, n, 3), dtype=torch.int64, device=summs[0].device)
    _all_gather(allcounts.view(-1), torch.stack([se.enc.counts for se in encoders]).view(-1), group=e0.group)
    for i, se in enumerate(encoders):
        se.all_counts.copy_(allcounts[:, i])


def gather_coefficients_group(encoders, group=None):
    """The gathers of several ShardEncoders (one image each, typically with
    different gather_to ranks) in ONE grouped RCCL batch on the current stream
    (gather_blocks_group).  Returns each encoder's whole-image {channel: (coef, dc)}
    on its gather_to rank, None elsewhere."""
    items = [e.gather_item() for e in encoders]
    e0 = encoders[0]
    gather_blocks_group(items, e0.rank, e0.world, group if group is not None else e0.group)
    return [it[1] for it in items]


def gather_streams_group(encoders, group=None, rccl=None, stream=None):
    """gather_kind "stream": the wire gathers of several images (image j to rank j)
    in ONE grouped batch, then each receiving rank's unpack + scan + emit, all on
    `stream` (default: the current one) with no host sync.  rccl: a RcclGather to
    move the bytes through the C-ABI instead of torch.distributed.  Returns each
    encoder's whole-image pipeline.Encoder (its stream) on its gather_to rank, None
    elsewhere."""
    st = stream if stream is not None else torch.cuda.current_stream()
    with torch.cuda.stream(st):
        # every image this rank sends, all channels: one batch (the job array of a
        # group of encoders is built once: their buffers are fixed)
        cache = _pack_arrays.setdefault(encoders[0], {})
        key = tuple(id(e) for e in encoders)
        hit = cache.get(key)
        if hit is not None and all(r() is e for r, e in zip(hit[0], encoders)):
            arr = hit[1]
        else:  # (an id can come back on a new encoder: the weak references tell)
            jobs = [j for e in encoders if e.rank != e.gather_to for j in e.pack_jobs()]
            arr = [(_lib.WireJob * len(jobs[i:i + 32]))(*jobs[i:i + 32]) for i in range(0, len(jobs), 32)]
            hit = None
            cache[key] = ([weakref.ref(e) for e in encoders], arr)
        for a in arr:
            _lib.call("hic_wire_pack_batch", len(a), a, device.stream_ptr(st))
        e0 = encoders[0]
        grp = group if group is not None else e0.group
        if rccl is not None:
            rccl.gather_group([e.stream_item() for e in encoders], st)
        elif dist.get_backend(grp) != "gloo":
            # the group's P2P operations over fixed buffers: built once (their
            # Python construction, ~42 per 8-rank group, would otherwise bound the
            # per-group host time), posted as one batch each time
            per_group = cache[key][2] if len(cache[key]) > 2 else {}
            ops = per_group.get(id(grp)) if hit is not None else None
            if ops is None:
                ops = _p2p_ops([e.stream_item() for e in encoders], e0.rank, e0.world, grp)
                per_group[id(grp)] = ops
                cache[key] = (cache[key][0], arr, per_group)
            for req in dist.batch_isend_irecv(ops) if ops else ():
                req.wait()
        else:
            gather_blocks_group([e.stream_item() for e in encoders], e0.rank, e0.world, grp)
        for e in encoders:
            if e.rank == e.gather_to:
                e.finish(st)
    return [e.whole for e in encoders]


# gather_streams_group: first encoder -> {(encoder ids): (weak refs, the group's pack
# job arrays, {process group id: its P2P operations})}
_pack_arrays = weakref.WeakKeyDictionary()


def wire_batch(fn, jobs, stream=None):
    """One of the batched wire calls over a job list (32 jobs per call)."""
    s = device.stream_ptr(stream)
    for i in range(0, len(jobs), 32):
        part = jobs[i:i + 32]
        arr = (_lib.WireJob * len(part))(*part)
        _lib.call(fn, len(part), arr, s)


def gather_blocks(mine, full, ranges, rank, world, dst, group=None):
    """The grouped gather itself (device-agnostic, so the CPU gloo tests run this
    exact code): mine = {channel: (tensor, ...)} this rank's block slices; full =
    {channel: (tensor, ...)} the whole-image tensors on dst (None elsewhere), the
    same tuple layout, first dimension = blocks; ranges = block_ranges(...).  dst
    receives every other rank's slices in place with ONE batch_isend_irecv group
    (RCCL: sends / receives on the current stream, no host sync); dst's own slice
    is expected to be written in place already.  gloo with device tensors (the
    one-GPU rehearsal) stages through the host."""
    gather_blocks_group([(mine, full, ranges, dst)], rank, world, group)


def _p2p_ops(items, rank, world, group):
    """gather_blocks_group's P2P operations (device tensors, an RCCL group: received
    in place) as a reusable list."""
    ops = []
    for mine, full, ranges, dst in items:
        if rank == dst:
            for r in range(world):
                if r == dst:
                    continue
                for k in CHANNELS:
                    b0, b1 = ranges[k][r]
                    for t in full[k]:
                        ops.append(dist.P2POp(dist.irecv, _wire(t[b0:b1]), r, group=group))
        else:
            for k in CHANNELS:
                for t in mine[k]:
                    ops.append(dist.P2POp(dist.isend, _wire(t.contiguous()), dst, group=group))
    return ops


def gather_blocks_group(items, rank, world, group=None):
    """Several images' gathers in ONE batch_isend_irecv group: items = [(mine,
    full, ranges, dst)] as gather_blocks, each with its own destination.  With the
    destinations spread over the ranks (image j of a group of N lands on rank j)
    every rank both sends and receives, so all xGMI links carry data in both
    directions at once -- N gathers into one rank would queue on that rank's 7
    ingress links.  Every rank lists the items in the same order (a sender's and a
    receiver's operations pair up per peer in posting order)."""
    ops, landing = [], []
    gloo = dist.get_backend(group) == "gloo"
    for mine, full, ranges, dst in items:
        if rank == dst:
            for r in range(world):
                if r == dst:
                    continue
                for k in CHANNELS:
                    b0, b1 = ranges[k][r]
                    for t in full[k]:
                        t = _wire(t[b0:b1])
                        buf = torch.empty(t.shape, dtype=t.dtype) if (gloo and t.is_cuda) else t
                        ops.append(dist.P2POp(dist.irecv, buf, r, group=group))
                        landing.append((t, buf))
        else:
            for k in CHANNELS:
                for t in mine[k]:
                    t = _wire(t.contiguous())
                    ops.append(dist.P2POp(dist.isend, t.cpu() if (gloo and t.is_cuda) else t, dst, group=group))
    for req in dist.batch_isend_irecv(ops) if ops else ():
        req.wait()
    for t, buf in landing:
        if buf is not t:
            t.copy_(buf)


class RcclGather:
    """The gather through the C-ABI (hic_gather_*, include/hiccup_hip.h): an RCCL
    communicator of the process group's ranks, made by the library itself (rank
    0's id crosses over the process group), and gather_blocks_group's transfer as
    hic_gather_bytes calls inside ONE hic_gather_group_begin / _end.  The same
    exchange as gather_blocks_group for a caller that binds the C-ABI directly;
    the caller must have selected its GPU (torch.cuda.set_device)."""

    def __init__(self, group=None):
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        uid = ctypes.create_string_buffer(_lib.GATHER_ID_BYTES)
        if self.rank == 0:
            _lib.call("hic_gather_unique_id", uid)
        box = [uid.raw if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = ctypes.create_string_buffer(box[0], _lib.GATHER_ID_BYTES)
        self.comm = ctypes.c_void_p()
        _lib.call("hic_gather_comm_init", ctypes.byref(self.comm), uid, self.world, self.rank)

    def close(self):
        if self.comm:
            _lib.call("hic_gather_comm_destroy", self.comm)
            self.comm = ctypes.c_void_p()

    def gather_group(self, items, stream=None):
        """items = [(mine, full, ranges, dst)] as gather_blocks_group (every
        rank lists them in the same order); on the given (or current) stream."""
        s = device.stream_ptr(stream)
        I64 = ctypes.c_int64 * self.world
        # every item's layout checked before the RCCL group opens (a failure inside
        # it would leave the peers' halves of the group posted)
        for mine, full, ranges, dst in items:
            if not 0 <= dst < self.world:
                raise ValueError("gather root %d of world %d" % (dst, self.world))
            for k in CHANNELS:
                if len(ranges[k]) != self.world or any(b < a for a, b in ranges[k]):
                    raise ValueError("channel %s: bad receive layout %r" % (k, ranges[k]))
                if self.rank == dst and (full is None or len(full[k]) != len(mine[k])):
                    raise ValueError("channel %s: the root needs a receive buffer per sent tensor" % k)
        _lib.call("hic_gather_group_begin")
        try:
            for mine, full, ranges, dst in items:
                for k in CHANNELS:
                    for ti, t in enumerate(mine[k]):
                        row = t.stride(0) * t.element_size()  # bytes per block
                        t = _wire(t)
                        offs = I64(*[ranges[k][r][0] * row for r in range(self.world)])
                        nbytes = I64(*[(ranges[k][r][1] - ranges[k][r][0]) * row for r in range(self.world)])
                        if self.rank == dst:
                            f = full[k][ti]
                            _lib.call("hic_gather_bytes", self.comm, device.ptr(t), t.numel(), device.ptr(f), offs,
                                      nbytes, dst, s)
                        else:
                            _lib.call("hic_gather_bytes", self.comm, device.ptr(t), t.numel(), None, None, None,
                                      dst, s)
        finally:
            _lib.call("hic_gather_group_end")

    def gather_encoders(self, encoders, stream=None):
        """gather_coefficients_group through the C-ABI."""
        items = [e.gather_item() for e in encoders]
        self.gather_group(items, stream)
        return [it[1] for it in items]


def exchange_halo_rows(planes, rank, world, group=None):
    """pyrUp's halo for a row-sharded decode: every plane in `planes` is (buf, top,
    n_own) -- buf holds this rank's n_own rows at [top, top + n_own), with one halo row
    above (top = 1, rank > 0) and one below (row top + n_own, rank < world - 1).
    Each rank sends its first own row up and its last own row down and receives its
    halo rows, all in ONE batch_isend_irecv group (RCCL on the current stream; gloo
    with device tensors stages through the host)."""
    if world == 1:
        return
    ops, landing = [], []
    gloo = dist.get_backend(group) == "gloo"

    def send(t, peer):
        t = _wire(t.contiguous())
        ops.append(dist.P2POp(dist.isend, t.cpu() if (gloo and t.is_cuda) else t, peer, group=group))

    def recv(t, peer):
        t = _wire(t)
        buf = torch.empty(t.shape, dtype=t.dtype) if (gloo and t.is_cuda) else t
        ops.append(dist.P2POp(dist.irecv, buf, peer, group=group))
        landing.append((t, buf))

    for buf, top, n_own in planes:
        if rank > 0:
            send(buf[top], rank - 1)
            recv(buf[0], rank - 1)
        if rank < world - 1:
            send(buf[top + n_own - 1], rank + 1)
            recv(buf[top + n_own], rank + 1)
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    for t, buf in landing:
        if buf is not t:
            t.copy_(buf)


class ShardDecoder:
    """One rank's part of a tile-sharded decode (codec.jpeg_decode's RLE / DC /
    izigzag half + compression.jpeg_decompression, codec.py:397-425,
    compression.py:42-56) of an H x W image encoded by ShardEncoders of the same
    plan.  Each rank decodes its own slice of the channel streams (the stitch record
    of its encode says where the slice starts: carried zeros, previous DC), runs the
    inverse DCT on its block rows, exchanges one chroma row with each neighbour for
    pyrUp and converts its rows to RGB: image rows [2 c0, 2 c1) (= the shard's rows
    but for the last row of an odd-height image, as the whole-image decode)."""

    def __init__(self, H, W, rank=None, world=None, group=None):
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        self.group = group
        self.H, self.W = H, W
        self.rows = plan(H, self.world)[self.rank]
        r0, r1 = self.rows
        self.h, self.w = H // 2, W // 2
        self.c0, self.c1 = r0 // 2, min(self.h, r1 // 2)
        if self.c1 <= self.c0:
            raise ValueError("shard %r has no chroma rows" % (self.rows,))
        self.top = 1 if self.c0 > 0 else 0
        self.bot = 1 if self.c1 < self.h else 0
        nc = self.c1 - self.c0
        self.shapes = {"lum": (r1 - r0, W), "cr": (nc, self.w), "cb": (nc, self.w)}
        self.blocks, self.status = {}, device.zeros((3,), torch.int64)
        for k in CHANNELS:
            self.blocks[k] = device.empty((pipeline._nblk(*self.shapes[k]), 64), torch.int16)
        self.y = device.empty(self.shapes["lum"], torch.uint8)
        self.cbuf = {k: device.empty((self.top + nc + self.bot, self.w), torch.uint8) for k in ("cr", "cb")}
        self.rgb = device.empty((2 * nc, 2 * self.w, 3), torch.uint8)
        self._ws = {}

    @property
    def out_rows(self):
        """Image rows [a, b) of this rank's RGB output."""
        return 2 * self.c0, 2 * self.c1

    def decode(self, sym_len, sym_val, counts, dc, stitch, stream=None):
        """sym_len / sym_val / dc: {channel: device tensor} this rank's slices (as its
        ShardEncoder wrote them); counts: host ints per channel; stitch: (3, 4) int64
        device tensor, the encode's hic_rle_stitch records.  Runs on `stream` (made
        current for the halo exchange)."""
        if stream is not None:
            with torch.cuda.stream(stream):
                return self._decode(sym_len, sym_val, counts, dc, stitch, stream)
        return self._decode(sym_len, sym_val, counts, dc, stitch, None)

    def _decode(self, sym_len, sym_val, counts, dc, stitch, stream):
        self.planes(sym_len, sym_val, counts, dc, stitch, stream)
        self.halo()
        return self.colour(stream)

    def halo_views(self):
        """[(buf, top, n_own)] of the two chroma planes (exchange_halo_rows' layout)."""
        return [(self.cbuf[k], self.top, self.c1 - self.c0) for k in ("cr", "cb")]

    def halo(self):
        """The exchange step: one chroma row to / from each neighbour (current stream)."""
        exchange_halo_rows(self.halo_views(), self.rank, self.world, self.group)

    def planes(self, sym_len, sym_val, counts, dc, stitch, stream=None):
        """Stream slices -> blocks -> this rank's Y rows and chroma rows."""
        s = device.stream_ptr(stream)
        lib = _lib.load()
        nc = self.c1 - self.c0
        for i, k in enumerate(CHANNELS):
            h, w = self.shapes[k]
            n = self.blocks[k].shape[0]
            nsym = int(counts[i])
            pipeline.check_count(nsym, k)
            need = lib.hic_rld_workspace_bytes(nsym, n)
            if k not in self._ws or self._ws[k].numel() * 8 < need:
                self._ws[k] = device.workspace(need)
            _lib.call("hic_rle_decode_i16_shard", device.ptr(sym_len[k]), device.ptr(sym_val[k]), nsym,
                      device.ptr(dc[k]), n, device.ptr(stitch[i]), device.ptr(self.blocks[k]),
                      device.ptr(self.status[i:i + 1]), device.ptr(self._ws[k]), s)
            out = self.y if k == "lum" else self.cbuf[k][self.top:self.top + nc]
            _lib.call("hic_dequant_idct_u8", device.ptr(self.blocks[k]), _lib.LAYOUT_ZIGZAG_I16, h, w,
                      pipeline.TABLES[k], device.ptr(out), out.stride(0), s)

    def colour(self, stream=None):
        """pyrUp (with the halo rows) + YCrCb -> RGB of this rank's rows."""
        s = device.stream_ptr(stream)
        cr, cb = self.cbuf["cr"], self.cbuf["cb"]
        _lib.call("hic_ycrcb420_to_rgb_rows", device.ptr(self.y), self.y.stride(0), device.ptr(cr), device.ptr(cb),
                  self.c0 - self.top, cr.shape[0], self.h, self.w, self.c0, self.c1, device.ptr(self.rgb), s)
        return self.rgb

    def check_status(self):
        """Raise unless every channel's slice decoded to exactly its blocks (syncs)."""
        st = self.status.cpu().tolist()
        for i, k in enumerate(CHANNELS):
            want = self.blocks[k].shape[0] * 63
            if st[i] != want:
                raise ValueError("rank %d channel %s: stream slice covers %d AC positions, expected %d"
                                 % (self.rank, k, st[i], want))


def _wire(t):
    """The bytes of a contiguous tensor, as the uint8 view every point-to-point
    transfer moves: torch's NCCL (= RCCL) process group refuses int16 tensors
    ("data type is not supported for NCCL process group: Short"), and the
    coefficient blocks and symbol lengths are int16.  A receive into the view lands
    in the tensor itself."""
    if not t.is_contiguous():
        raise ValueError("point-to-point transfers need contiguous tensors")
    return t if t.dtype == torch.uint8 else t.view(torch.uint8)


def _send(t, dst, group):
    t = _wire(t)
    if t.is_cuda and dist.get_backend(group) == "gloo":
        t = t.cpu()
    dist.send(t, dst=dst, group=group)


def _recv(t, src, group):
    t = _wire(t)
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = torch.empty(t.shape, dtype=t.dtype)
        dist.recv(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.recv(t, src=src, group=group)


def gather_streams(se, dst=0):
    """Reassemble the global symbol / DC streams on rank `dst` (RCCL send/recv;
    tests and tools: the counts cross to the host first).  Returns {channel:
    (dc_diff, sym_len, sym_val)} host arrays on dst, None elsewhere."""
    se.offsets()  # raises on a failed rank
    counts = se.all_counts.cpu().numpy()
    nblk = torch.tensor([se.enc.dc[k].numel() for k in CHANNELS], dtype=torch.int64, device=se.all_counts.device)
    all_nblk = torch.zeros((se.world, 3), dtype=torch.int64, device=nblk.device)
    _all_gather(all_nblk.view(-1), nblk, group=se.group)
    all_nblk = all_nblk.cpu().numpy()
    out = {} if se.rank == dst else None
    for ci, k in enumerate(CHANNELS):
        enc = se.enc
        if se.rank == dst:
            tot_s, tot_b = int(counts[:, ci].sum()), int(all_nblk[:, ci].sum())
            L = torch.empty(tot_s, dtype=enc.sym_len[k].dtype, device=enc.sym_len[k].device)
            V = torch.empty(tot_s, dtype=enc.sym_val[k].dtype, device=enc.sym_val[k].device)
            D = torch.empty(tot_b, dtype=torch.int32, device=enc.dc[k].device)
            so, bo = 0, 0
            for r in range(se.world):
                n, nb = int(counts[r, ci]), int(all_nblk[r, ci])
                if r == dst:
                    L[so:so + n].copy_(enc.sym_len[k][:n])
                    V[so:so + n].copy_(enc.sym_val[k][:n])
                    D[bo:bo + nb].copy_(enc.dc[k])
                else:
                    for t in (L[so:so + n], V[so:so + n], D[bo:bo + nb]):
                        _recv(t, r, se.group)
                so += n
                bo += nb
            out[k] = (D.cpu().numpy(), L.cpu().numpy(), V.cpu().numpy())
        else:
            n = int(counts[se.rank, ci])
            for t in (enc.sym_len[k][:n], enc.sym_val[k][:n], enc.dc[k]):
                _send(t.contiguous(), dst, se.group)
    return out
