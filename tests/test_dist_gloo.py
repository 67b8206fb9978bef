"""Multi-process (world_size 2 and 3, gloo on CPU) test of the tile-sharded
encode's exchange steps: each rank holds a block-row shard of the coefficient
streams, all-gathers its channel summaries with sharding.exchange, derives its
stitch record with sharding.stitch_host, run-length codes its slice, and rank 0
reassembles (a) the coefficient blocks + DC stream with sharding.gather_blocks --
the same grouped batch_isend_irecv code the RCCL path runs; (a') a group of
`world` images' gathers, image j to rank j, goes out as one batch
(sharding.gather_blocks_group, the bench's exchange); (a'') the stream gather:
blocks in the wire format (tests/wire_host.py) to the receiving rank, which
codes the whole stream -- and (b) the symbol
streams with point-to-point sends.  Both must equal the single-stream encode.
(c) Each rank then decodes its own slice (sharded decode: carried-zero skip, DC
chain from the stitch record, pyrUp halo rows from sharding.exchange_halo_rows)
and its RGB rows must equal the whole-image decode's.  (Per-shard compute here is the CPU oracle -- test
infrastructure; the GPU kernels for the same steps are covered by
tests/test_gpu_codec.py::test_shards_stitch_to_single_stream.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle.oracle as orc
from hiccup_amd import pipeline, sharding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _image(H, W, flat=None):
    rng = np.random.default_rng(42)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rgb[H // 3: H // 3 + 40] = 128  # zero runs crossing shard boundaries
    rgb[:, : W // 4] = 200
    if flat:  # a whole shard with no nonzero luma AC: the carried run chains through it
        rgb[flat[0]:flat[1]] = 128
    return rgb


def _zz_planes(rgb):
    y, cr, cb = orc.rgb_to_ycrcb(rgb)
    out = {}
    for k, p, t in (("lum", y, 0), ("cr", orc.pyr_down(cr), 1), ("cb", orc.pyr_down(cb), 1)):
        out[k] = orc.zigzag_blocks(orc.split_blocks(orc.dct_channel(p, t)).astype(np.int64))
    return out


def _summary(zz):
    ac = zz[:, 1:].reshape(-1)
    nz = np.flatnonzero(ac)
    return [len(ac) - 1 - (nz[-1] if len(nz) else -1), int(len(nz) > 0), int(zz[0, 0]), int(zz[-1, 0])]


def _rle_stitched(zz, st):
    carry, emit_eob, has_prev, prev_dc = (int(x) for x in st)
    dc = zz[:, 0].astype(np.int64)
    diff = orc.dpcm(dc)
    if has_prev:
        diff[0] = dc[0] - prev_dc
    ac = zz[:, 1:].reshape(-1)
    L, V = orc.rle_encode(np.concatenate([np.zeros(carry, np.int64), ac]), 15)
    if not emit_eob and (len(ac) == 0 or ac[-1] == 0):
        L, V = L[:-1], V[:-1]
    return diff, L, V


def _wire_ranges_host(ranges):
    """sharding.wire_ranges without records and without the library (CPU test)."""
    import wire_host
    out = {}
    for k in pipeline.CHANNELS:
        o, rr = 0, []
        for b0, b1 in ranges[k]:
            rr.append((o, o + wire_host.wire_bytes(b1 - b0, wire_host.TABLE_OF[k]) + sharding.TRAILER_BYTES))
            o = rr[-1][1]
        out[k] = rr
    return out


def _worker(rank, world, port, H, W, flat, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        zz = _zz_planes(_image(H, W, flat))
        r0, r1 = sharding.plan(H, world)[rank]
        ranges = sharding.block_ranges(H, W, world)
        mine = {}
        for k in pipeline.CHANNELS:
            nbx = -(-(W if k == "lum" else W // 2) // 8)
            if k == "lum":
                b0, b1 = (r0 // 8) * nbx, (-(-r1 // 8)) * nbx
            else:
                c1 = min(H // 2, r1 // 2)
                b0, b1 = (r0 // 16) * nbx, (-(-c1 // 8)) * nbx
            assert ranges[k][rank] == (b0, b1)
            mine[k] = zz[k][b0:b1]
        summ = torch.tensor([_summary(mine[k]) for k in pipeline.CHANNELS], dtype=torch.int64)
        allsum = sharding.exchange(summ, world).numpy()
        enc = {k: _rle_stitched(mine[k], sharding.stitch_host(allsum[:, c], rank))
               for c, k in enumerate(pipeline.CHANNELS)}
        # (a) the grouped coefficient / DC gather (sharding.gather_blocks)
        parts = {k: (torch.from_numpy(np.ascontiguousarray(mine[k], dtype=np.int16)),
                     torch.from_numpy(np.ascontiguousarray(enc[k][0], dtype=np.int32)))
                 for k in pipeline.CHANNELS}
        full = None
        if rank == 0:
            full = {k: (torch.full((len(zz[k]), 64), -7, dtype=torch.int16),
                        torch.full((len(zz[k]),), -7, dtype=torch.int32)) for k in pipeline.CHANNELS}
            for k in pipeline.CHANNELS:
                b0, b1 = ranges[k][0]
                full[k][0][b0:b1] = parts[k][0]
                full[k][1][b0:b1] = parts[k][1]
        sharding.gather_blocks(parts, full, ranges, rank, world, 0)
        if rank == 0:
            for k in pipeline.CHANNELS:
                results["blocks_" + k] = bool(
                    np.array_equal(full[k][0].numpy(), zz[k].astype(np.int16))
                    and np.array_equal(full[k][1].numpy(), orc.dpcm(zz[k][:, 0].astype(np.int64)).astype(np.int32)))
        # (a') one group of `world` images' gathers, image j to rank j
        # (sharding.gather_blocks_group, the bench's multi-GPU exchange)
        items = []
        for j in range(world):
            pj = {k: (parts[k][0] + j, parts[k][1] - j) for k in pipeline.CHANNELS}
            fj = None
            if rank == j:
                fj = {k: (torch.full((len(zz[k]), 64), -7, dtype=torch.int16),
                          torch.full((len(zz[k]),), -7, dtype=torch.int32)) for k in pipeline.CHANNELS}
                for k in pipeline.CHANNELS:
                    b0, b1 = ranges[k][rank]
                    fj[k][0][b0:b1] = pj[k][0]
                    fj[k][1][b0:b1] = pj[k][1]
            items.append((pj, fj, ranges, j))
        sharding.gather_blocks_group(items, rank, world)
        fj = items[rank][1]
        results["group_%d" % rank] = all(
            np.array_equal(fj[k][0].numpy(), zz[k].astype(np.int16) + rank)
            and np.array_equal(fj[k][1].numpy(), orc.dpcm(zz[k][:, 0].astype(np.int64)).astype(np.int32) - rank)
            for k in pipeline.CHANNELS)
        # (a'') the stream gather (gather_kind "stream", the bench's default): every
        # rank ships its blocks in the wire format (host restatement of
        # hic_wire_pack_i16) into the byte ranges of sharding.wire_ranges, image j to
        # rank j in one batch (sharding.gather_blocks_group, the code the GPU path
        # runs); the receiver unpacks, codes the WHOLE stream and must get the
        # single-stream encode
        import wire_host
        # W % 512 == 0: the fused kernel's record layout (chroma half tiles), every
        # shard on a record boundary, so the segments carry the shards' RLE tile
        # records rebased to whole-image positions behind their blocks (ShardEncoder
        # .pack / .finish); other widths: blocks only (the receiver's tile pass)
        rpt = pipeline.encoder_layout(H, W, (r0, r1))[1] if W % 512 == 0 else {k: 1 for k in pipeline.CHANNELS}
        records = sharding.records_aligned(ranges, rpt)
        assert records == (W % 512 == 0)
        wr = sharding.wire_ranges(ranges, rpt, records)  # hic_wire_bytes: host code, no GPU
        if not records:
            assert wr == _wire_ranges_host(ranges)

        def segment(k, blocks, b0):
            # blocks, [rebased records], trailer (the sender's out-of-width flag: 0)
            w = wire_host.pack(blocks, wire_host.TABLE_OF[k])
            seg = np.zeros(wr[k][rank][1] - wr[k][rank][0], np.uint8)
            seg[:len(w)] = w
            if records:
                per = 64 // rpt[k]
                rec = wire_host.rebase(wire_host.tile_records(blocks, per), b0 * 63)  # shard-local, then rebased
                seg[len(w):len(w) + rec.nbytes] = rec.reshape(-1).view(np.uint8)
            return seg

        items = []
        for j in range(world):
            mine_w = {k: (torch.from_numpy(segment(k, mine[k] + j if j else mine[k], ranges[k][rank][0]).copy()),)
                      for k in pipeline.CHANNELS}
            full_w = ({k: (torch.zeros(wr[k][-1][1], dtype=torch.uint8),) for k in pipeline.CHANNELS}
                      if rank == j else None)
            items.append((mine_w, full_w, wr, j))
        sharding.gather_blocks_group(items, rank, world)
        full_w = items[rank][1]
        ok = True
        for k in pipeline.CHANNELS:
            parts = []
            for r in range(world):
                b0, b1 = ranges[k][r]
                if r == rank:
                    parts.append(mine[k] + rank if rank else mine[k])
                else:
                    o0, o1 = wr[k][r]
                    parts.append(wire_host.unpack(full_w[k][0][o0:o1].numpy(), b1 - b0,
                                                  wire_host.TABLE_OF[k]).astype(np.int64))
            whole = np.concatenate(parts)
            want = zz[k] + rank if rank else zz[k]
            ok &= np.array_equal(whole, want)
            # every sender's trailer flag arrived clear
            ok &= all(int(full_w[k][0][wr[k][r][1] - sharding.TRAILER_BYTES:].view(torch.int32)[0]) == 0
                      for r in range(world) if r != rank)
            if records:
                # the placed records (ShardEncoder.finish: record b0 * rpt / 64 of the
                # whole image's workspace) == the whole image's own tile records
                per = 64 // rpt[k]
                recs = np.zeros((-(-len(want) // per), 3), np.int64)
                for r in range(world):
                    b0, b1 = ranges[k][r]
                    nrec = -(-(b1 - b0) * rpt[k] // 64)
                    if r == rank:
                        got = wire_host.rebase(wire_host.tile_records(parts[r], per), b0 * 63)
                    else:
                        o0, _ = wr[k][r]
                        wb = wire_host.wire_bytes(b1 - b0, wire_host.TABLE_OF[k])
                        got = full_w[k][0][o0 + wb:o0 + wb + nrec * 24].numpy().view(np.int64).reshape(nrec, 3)
                    recs[b0 * rpt[k] // 64:b0 * rpt[k] // 64 + nrec] = got
                ok &= np.array_equal(recs, wire_host.tile_records(want, per))
            L, V = orc.rle_encode(whole[:, 1:].reshape(-1), 15)
            eL, eV = orc.rle_encode(want[:, 1:].reshape(-1), 15)
            ok &= np.array_equal(L, eL) and np.array_equal(V, eV)
            ok &= np.array_equal(orc.dpcm(whole[:, 0]), orc.dpcm(want[:, 0]))
        results["stream_%d" % rank] = bool(ok)
        # (c) the sharded decode: this rank's stream slice -> blocks (carried zeros
        # skipped, DC chain from the previous shard), inverse DCT of its block rows,
        # pyrUp halo rows from the neighbours (sharding.exchange_halo_rows, the code
        # the RCCL path runs), colour of its rows == the whole-image decode's rows
        h, w = H // 2, W // 2
        c0, c1 = r0 // 2, min(h, r1 // 2)
        top, bot = int(c0 > 0), int(c1 < h)
        planes = {}
        for c, k in enumerate(pipeline.CHANNELS):
            st = sharding.stitch_host(allsum[:, c], rank)
            diff, L, V = enc[k]
            n = len(mine[k])
            ac = orc.rle_decode_shard(L, V, int(st[0]), n * 63).reshape(n, 63)
            dcs = np.cumsum(diff) + (int(st[3]) if st[2] else 0)
            blocks = orc.izigzag_blocks(np.concatenate([dcs[:, None], ac], axis=1))
            shape = (r1 - r0, W) if k == "lum" else (c1 - c0, w)
            planes[k] = orc.inv_dct_channel(orc.merge_blocks(blocks, shape), 0 if k == "lum" else 1)
        bufs = {}
        for k in ("cr", "cb"):
            b = torch.zeros((top + c1 - c0 + bot, w), dtype=torch.uint8)
            b[top:top + c1 - c0] = torch.from_numpy(planes[k])
            bufs[k] = b
        sharding.exchange_halo_rows([(bufs[k], top, c1 - c0) for k in ("cr", "cb")], rank, world)
        hl = bufs["cr"].shape[0]
        yl = np.zeros((2 * hl, 2 * w), np.uint8)
        yl[2 * top:2 * top + 2 * (c1 - c0)] = planes["lum"][:2 * (c1 - c0), :2 * w]
        rgb_l = orc.ycrcb_to_rgb(yl, orc.pyr_up(bufs["cr"].numpy()), orc.pyr_up(bufs["cb"].numpy()))
        mine_rgb = rgb_l[2 * top:2 * (top + c1 - c0)]
        y_w, cr_w, cb_w = (orc.inv_dct_channel(orc.merge_blocks(orc.izigzag_blocks(zz[k]), sh), t) for k, sh, t in
                           (("lum", (H, W), 0), ("cr", (h, w), 1), ("cb", (h, w), 1)))
        whole = orc.ycrcb_to_rgb(y_w[:2 * h, :2 * w], orc.pyr_up(cr_w), orc.pyr_up(cb_w))
        results["decode_%d" % rank] = bool(np.array_equal(mine_rgb, whole[2 * c0:2 * c1]))
        # reassemble on rank 0: sizes first, then point-to-point payloads
        sizes = torch.tensor([[len(enc[k][0]), len(enc[k][1])] for k in pipeline.CHANNELS], dtype=torch.int64)
        all_sizes = sharding.exchange(sizes, world).numpy()
        if rank == 0:
            got = {}
            for c, k in enumerate(pipeline.CHANNELS):
                parts = [enc[k]]
                for r in range(1, world):
                    nb, ns = all_sizes[r, c]
                    bufs = [torch.empty(nb, dtype=torch.int64), torch.empty(ns, dtype=torch.int64),
                            torch.empty(ns, dtype=torch.int64)]
                    for b in bufs:
                        dist.recv(b, src=r)
                    parts.append(tuple(b.numpy() for b in bufs))
                got[k] = tuple(np.concatenate([p[j] for p in parts]) for j in range(3))
            for k in pipeline.CHANNELS:
                diff = orc.dpcm(zz[k][:, 0].astype(np.int64))
                L, V = orc.rle_encode(zz[k][:, 1:].reshape(-1), 15)
                ok = (np.array_equal(got[k][0], diff) and np.array_equal(got[k][1], L)
                      and np.array_equal(got[k][2], V))
                results[k] = bool(ok)
        else:
            for k in pipeline.CHANNELS:
                for a in enc[k]:
                    dist.send(torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)), dst=0)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W,flat", [(2, 96, 80, None), (3, 130, 72, None), (4, 160, 48, None),
                                            (3, 144, 64, (48, 96)), (2, 64, 512, None),
                                            # the 8K plan's geometry: 270 unit rows over 8 ranks (34 / 33 each),
                                            # W % 512 == 0 (records rebased and gathered with the blocks)
                                            (8, 4320, 512, None)])
def test_sharded_exchange_gloo(world, H, W, flat):
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), H, W, flat, results), nprocs=world, join=True)
    exp = {k: True for k in pipeline.CHANNELS}
    exp.update({"blocks_" + k: True for k in pipeline.CHANNELS})
    exp.update({"decode_%d" % r: True for r in range(world)})
    exp.update({"group_%d" % r: True for r in range(world)})
    exp.update({"stream_%d" % r: True for r in range(world)})
    assert dict(results) == exp


def _link_worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    try:
        results[rank] = bench.measure_link(rank, world, nbytes=1 << 20, reps=2, device="cpu")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_measure_link_ring_gloo(world):
    """bench.measure_link (the N > 1 line's in-run link rate): a ring in which every
    rank takes part in each P2P batch, so it completes at any world size (gloo on
    CPU here; RCCL on the node) and every rank reports the same slowest-rank rate."""
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_link_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    got = dict(results)
    assert sorted(got) == list(range(world))
    assert len(set(got.values())) == 1 and list(got.values())[0] >= 0  # (GB/s to 0.1: gloo may round to 0)
