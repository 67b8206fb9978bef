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
global offsets.  ``gather_streams`` optionally reassembles the coefficient stream
on one rank (point-to-point RCCL sends into offset slices).
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


class ShardEncoder:
    """One rank's part of a tile-sharded encode of an H x W RGB image."""

    def __init__(self, H, W, rank=None, world=None, group=None, max_len=15):
        self.rank = dist.get_rank(group) if rank is None else rank
        self.world = dist.get_world_size(group) if world is None else world
        self.group = group
        self.H, self.W = H, W
        self.rows = plan(H, self.world)[self.rank]
        self.enc = pipeline.Encoder(H, W, max_len=max_len, rows=self.rows)
        self.span = self.enc.input_span()
        self.all_summ = device.zeros((self.world, 3, 4), torch.int64)
        self.stitch = device.zeros((3, 4), torch.int64)
        self.all_counts = device.zeros((self.world, 3), torch.int64)

    @property
    def pixels(self):
        return self.enc.pixels

    def encode(self, rgb_rows, stream=None, dct_events=None):
        """rgb_rows: device uint8 tensor of image rows self.span (shard + halo)."""
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
        return c[:self.rank].sum(0), c.sum(0)


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
    """Reassemble the global symbol / DC streams on rank `dst` (RCCL send/recv).
    Returns {channel: (dc_diff, sym_len, sym_val)} host arrays on dst, None elsewhere."""
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
