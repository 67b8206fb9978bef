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


class ShardEncoder:
    """One rank's part of a tile-sharded encode of an H x W RGB image.

    gather_to: the rank that reassembles the whole image's coefficient blocks and
    DC differences (gather_coefficients); None = no reassembly buffers."""

    def __init__(self, H, W, rank=None, world=None, group=None, max_len=15, gather_to=None):
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        self.group = group
        self.H, self.W = H, W
        self.rows = plan(H, self.world)[self.rank]
        self.ranges = block_ranges(H, W, self.world)
        self.gather_to = gather_to
        out = None
        if gather_to is not None and self.rank == gather_to:
            # whole-image buffers; this rank's encoder writes its slice in place
            self.full_coef, self.full_dc, out = {}, {}, {}
            for k in CHANNELS:
                n = self.ranges[k][-1][1]
                self.full_coef[k] = device.empty((n, 64), torch.int16)
                self.full_dc[k] = device.empty((n,), torch.int32)
                b0, b1 = self.ranges[k][self.rank]
                out[k] = (self.full_coef[k][b0:b1], self.full_dc[k][b0:b1])
        self.enc = pipeline.Encoder(H, W, max_len=max_len, rows=self.rows, out=out)
        self.span = self.enc.input_span()
        self.all_summ = device.zeros((self.world, 3, 4), torch.int64)
        self.stitch = device.zeros((3, 4), torch.int64)
        self.all_counts = device.zeros((self.world, 3), torch.int64)

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
        full = {k: (self.full_coef[k], self.full_dc[k]) for k in CHANNELS} if self.rank == self.gather_to else None
        mine = {k: (self.enc.coef[k], self.enc.dc[k]) for k in CHANNELS}
        gather_blocks(mine, full, self.ranges, self.rank, self.world, self.gather_to, self.group)
        return full


def gather_blocks(mine, full, ranges, rank, world, dst, group=None):
    """The grouped gather itself (device-agnostic, so the CPU gloo tests run this
    exact code): mine = {channel: (tensor, ...)} this rank's block slices; full =
    {channel: (tensor, ...)} the whole-image tensors on dst (None elsewhere), the
    same tuple layout, first dimension = blocks; ranges = block_ranges(...).  dst
    receives every other rank's slices in place with ONE batch_isend_irecv group
    (RCCL: sends / receives on the current stream, no host sync); dst's own slice
    is expected to be written in place already.  gloo with device tensors (the
    one-GPU rehearsal) stages through the host."""
    ops, landing = [], []
    gloo = dist.get_backend(group) == "gloo"
    if rank == dst:
        for r in range(world):
            if r == dst:
                continue
            for k in CHANNELS:
                b0, b1 = ranges[k][r]
                for t in full[k]:
                    t = t[b0:b1]
                    buf = torch.empty(t.shape, dtype=t.dtype) if (gloo and t.is_cuda) else t
                    ops.append(dist.P2POp(dist.irecv, buf, r, group=group))
                    landing.append((t, buf))
    else:
        for k in CHANNELS:
            for t in mine[k]:
                t = t.contiguous()
                ops.append(dist.P2POp(dist.isend, t.cpu() if (gloo and t.is_cuda) else t, dst, group=group))
    for req in dist.batch_isend_irecv(ops) if ops else ():
        req.wait()
    for t, buf in landing:
        if buf is not t:
            t.copy_(buf)


def _send(t, dst, group):
    if t.is_cuda and dist.get_backend(group) == "gloo":
        t = t.cpu()
    dist.send(t, dst=dst, group=group)


def _recv(t, src, group):
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
