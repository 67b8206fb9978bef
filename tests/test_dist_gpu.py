"""Multi-process rehearsal of the tile-sharded encode on ONE GPU: world_size 2 and
3, every rank on cuda:0, gloo for the exchange (RCCL needs a GPU per rank; the
driver runs the real 8-GPU RCCL bench).  Each rank runs the HIP kernels on its
row shard (ShardEncoder: colour with halo, fused DCT + RLE tile records,
summaries, all-gather, device stitch, scan + emit), rank 0 reassembles the
streams with gather_streams, and the result must equal the single-GPU encode of
the whole image bit for bit.  Each rank then decodes its own slice
(ShardDecoder, halo rows over the process group) and its RGB rows must equal the
single-GPU decode's.  Finally `world` images are encoded and gathered as the
bench's strong mode does it (image j to rank j, one grouped batch), and each
rank's received image must equal its single-GPU encode: the int16 block gather
(gather_kind "blocks") and the stream gather (gather_kind "stream": wire-format
blocks + rebased tile records, the whole stream coded on the receiving rank)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _image(H, W, flat_rows=None):
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rgb[H // 3: H // 3 + 48] = 128   # all-zero AC runs across a shard boundary
    rgb[:, : W // 5] = 40            # a flat band: long carried runs
    if flat_rows:                    # a whole shard without any nonzero AC: the
        rgb[flat_rows[0]:flat_rows[1]] = 128  # carried run chains through it
    return rgb


def _rank(rank, world, port, H, W, flat_rows, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hiccup_amd import device, pipeline, sharding
    torch.cuda.set_device(0)
    rgb = _image(H, W, flat_rows)
    se = sharding.ShardEncoder(H, W, rank=rank, world=world, gather_to=0)
    a, b = se.span
    # a non-current stream: the collectives must follow it
    s = torch.cuda.Stream()
    se.encode(device.to_device(rgb[a:b]), stream=s)
    blocks = se.gather_coefficients(stream=s)
    # the sharded decode of this rank's slice (halo rows exchanged with the neighbours)
    sd = sharding.ShardDecoder(H, W, rank=rank, world=world)
    torch.cuda.synchronize()
    mine = sd.decode(se.enc.sym_len, se.enc.sym_val, se.enc.counts.cpu().tolist(), se.enc.dc, se.stitch, stream=s)
    torch.cuda.synchronize()
    sd.check_status()
    whole = pipeline.Encoder(H, W)
    whole.encode(device.to_device(rgb))
    whole.compact()  # a slot-layout encoder: the contiguous stream the plain decode reads
    wd = pipeline.Decoder(H, W)
    exp = device.to_host(wd.decode(whole.sym_len, whole.sym_val, whole.counts.cpu().tolist(), whole.dc))
    r0, r1 = sd.out_rows
    dec_ok = np.array_equal(device.to_host(mine), exp[r0:r1])
    oks = [None] * world
    dist.all_gather_object(oks, bool(dec_ok))
    got = sharding.gather_streams(se)
    if rank == 0:
        ref = whole.result()
        ok = True
        for k in pipeline.CHANNELS:
            D, L, V = got[k]
            ok &= np.array_equal(D, ref[k][1]) and np.array_equal(L, ref[k][2]) and np.array_equal(V, ref[k][3])
            # the grouped gather's whole-image blocks / DC stream
            ok &= np.array_equal(blocks[k][0].cpu().numpy(), ref[k][0])
            ok &= np.array_equal(blocks[k][1].cpu().numpy(), ref[k][1])
        offs, tot = se.offsets()
        ok &= [int(x) for x in tot] == [len(ref[k][2]) for k in pipeline.CHANNELS]
        ok &= all(oks)
        with open(out_path, "w") as f:
            f.write("ok" if ok else "mismatch")
    # the bench's grouped exchange: `world` different images, image j gathered to
    # rank j, all in one batch (sharding.gather_coefficients_group) on a process
    # group of its own; each rank checks the image it received
    xgroup = dist.new_group(list(range(world)))
    imgs = [np.roll(rgb, 8 * j, axis=1) for j in range(world)]
    ses = [sharding.ShardEncoder(H, W, rank=rank, world=world, gather_to=j) for j in range(world)]
    # the group's exchange steps batched: one summary and one count all-gather
    sharding.encode_group(ses, [device.to_device(img[a:b]) for img in imgs], stream=s)
    with torch.cuda.stream(s):
        fulls = sharding.gather_coefficients_group(ses, group=xgroup)
    torch.cuda.synchronize()
    refs = []
    for img in imgs:
        w_enc = pipeline.Encoder(H, W)
        w_enc.encode(device.to_device(img))
        refs.append(w_enc.result())
    ref = refs[rank]
    gok = all(np.array_equal(fulls[rank][k][0].cpu().numpy(), ref[k][0]) and
              np.array_equal(fulls[rank][k][1].cpu().numpy(), ref[k][1]) for k in pipeline.CHANNELS)
    gok &= all(fulls[j] is None for j in range(world) if j != rank)
    # every image's symbol stream (stitched per image inside the batched group)
    for j in range(world):
        got_j = sharding.gather_streams(ses[j])
        if rank == 0:
            gok &= all(np.array_equal(got_j[k][0], refs[j][k][1]) and np.array_equal(got_j[k][1], refs[j][k][2])
                       and np.array_equal(got_j[k][2], refs[j][k][3]) for k in pipeline.CHANNELS)
    # the stream gather (the bench's default): ranks only transform, ship wire-format
    # blocks + rebased tile records; the receiving rank codes the whole stream
    sss = [sharding.ShardEncoder(H, W, rank=rank, world=world, gather_to=j, gather_kind="stream")
           for j in range(world)]
    sharding.encode_group(sss, [device.to_device(img[a:b]) for img in imgs], stream=s)
    wholes = sharding.gather_streams_group(sss, group=xgroup, stream=s)
    torch.cuda.synchronize()
    got_w = wholes[rank].result()
    gok &= all(np.array_equal(got_w[k][i], ref[k][i]) for k in pipeline.CHANNELS for i in range(4))
    gok &= all(wholes[j] is None for j in range(world) if j != rank)
    gok &= all(int(e.wire_flag.item()) == 0 for e in sss)
    gok &= sss[rank].records == sharding.records_aligned(sss[rank].ranges, sss[rank].enc.rpt)
    # a coefficient outside its wire width on a sender (forced here): the flag rides
    # in the segment's trailer and the receiver marks that channel's stream invalid
    sss2 = [sharding.ShardEncoder(H, W, rank=rank, world=world, gather_to=j, gather_kind="stream")
            for j in range(world)]
    sharding.encode_group(sss2, [device.to_device(img[a:b]) for img in imgs], stream=s)
    torch.cuda.synchronize()
    for j in range(world):
        if j != rank:
            sss2[j].enc.coef["lum"][0, 5] = 32000  # > any luminance slot width
    wholes2 = sharding.gather_streams_group(sss2, group=xgroup, stream=s)
    torch.cuda.synchronize()
    c2 = wholes2[rank].counts.cpu().tolist()
    gok &= c2[0] == pipeline.COUNT_WIRE_OVERFLOW and c2[1] >= 0 and c2[2] >= 0
    gok &= all(int(sss2[j].wire_flag.item()) == 1 for j in range(world) if j != rank)
    goks = [None] * world
    dist.all_gather_object(goks, bool(gok))
    if rank == 0 and not all(goks):
        with open(out_path, "w") as f:
            f.write("grouped gather mismatch %s" % goks)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W,flat", [(2, 256, 384, None), (3, 4320 // 4, 7680 // 2, None),
                                            (3, 384, 256, (120, 264)), (2, 256, 1024, None),
                                            (3, 4320 // 4, 7680, None)])
def test_sharded_encode_multiprocess(world, H, W, flat):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "result")
        mp.spawn(_rank, args=(world, _free_port(), H, W, flat, out), nprocs=world, join=True)
        assert open(out).read() == "ok"


def _rccl_rank(rank, port, H, W, out_path):
    """RCCL itself on the one-GPU box: a world-size-1 nccl process group (RCCL refuses
    two ranks on one device) through the sharded encode's collectives (the summary
    and count all-gathers of encode_group, ShardEncoder.offsets) and the grouped
    P2P batch of the gather, here as sends / receives to self (through the byte
    views sharding._wire gives every transfer: the NCCL process group refuses int16)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from hiccup_amd import device, pipeline, sharding
    assert dist.get_backend() == "nccl"
    rgb = _image(H, W)
    xgroup = dist.new_group([0])
    se = sharding.ShardEncoder(H, W, rank=0, world=1, gather_to=0)
    s = torch.cuda.Stream()
    sharding.encode_group([se], [device.to_device(rgb)], stream=s)
    with torch.cuda.stream(s):
        fulls = sharding.gather_coefficients_group([se], group=xgroup)
        # the gather's P2P batch shape (P2POp pairs in one batch_isend_irecv group on
        # the current stream), rank to itself: every channel's blocks and DC stream
        copies, ops = [], []
        for k in pipeline.CHANNELS:
            for t in fulls[0][k]:
                dst = torch.empty_like(t)
                ops += [dist.P2POp(dist.isend, sharding._wire(t.contiguous()), 0, group=xgroup),
                        dist.P2POp(dist.irecv, sharding._wire(dst), 0, group=xgroup)]
                copies.append((t, dst))
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    torch.cuda.synchronize()
    whole = pipeline.Encoder(H, W)
    whole.encode(device.to_device(rgb))
    ref = whole.result()
    ok = all(np.array_equal(fulls[0][k][0].cpu().numpy(), ref[k][0]) and
             np.array_equal(fulls[0][k][1].cpu().numpy(), ref[k][1]) for k in pipeline.CHANNELS)
    ok &= all(torch.equal(a, b) for a, b in copies)
    got = sharding.gather_streams(se)
    ok &= all(np.array_equal(got[k][0], ref[k][1]) and np.array_equal(got[k][1], ref[k][2]) and
              np.array_equal(got[k][2], ref[k][3]) for k in pipeline.CHANNELS)
    offs, tot = se.offsets()
    ok &= [int(x) for x in tot] == [len(ref[k][2]) for k in pipeline.CHANNELS]
    # the same gather through the C-ABI (hic_gather_*: the library's own RCCL
    # communicator), into fresh whole-image buffers, and a root slice that is not in
    # place (hic_gather_bytes copies it)
    import ctypes
    from hiccup_amd import _lib
    g = sharding.RcclGather(group=xgroup)
    w, r = ctypes.c_int(), ctypes.c_int()
    _lib.call("hic_gather_comm_info", g.comm, ctypes.byref(w), ctypes.byref(r))
    ok &= (w.value, r.value) == (1, 0)
    se2 = sharding.ShardEncoder(H, W, rank=0, world=1, gather_to=0)
    se2.encode(device.to_device(rgb))
    full2 = g.gather_encoders([se2])[0]
    src = torch.arange(1000, dtype=torch.int16, device="cuda")
    dst = torch.zeros(1300, dtype=torch.int16, device="cuda")
    I64 = ctypes.c_int64 * 1
    _lib.call("hic_gather_bytes", g.comm, device.ptr(src), 2000, device.ptr(dst), I64(600), I64(2000), 0,
              device.stream_ptr())
    torch.cuda.synchronize()
    ok &= all(np.array_equal(full2[k][0].cpu().numpy(), ref[k][0]) and np.array_equal(full2[k][1].cpu().numpy(),
                                                                                        ref[k][1])
              for k in pipeline.CHANNELS)
    ok &= torch.equal(dst[300:1300], src) and int(dst[:300].abs().sum()) == 0
    try:  # argument errors come back as HIC_ERR_ARG
        _lib.call("hic_gather_bytes", g.comm, device.ptr(src), 2000, device.ptr(dst), I64(0), I64(10), 0, None)
        ok = False
    except ValueError:
        pass
    # the stream gather through the C-ABI transport (world 1: the whole image is
    # this rank's own shard; its records are rebased, the whole stream coded here)
    ss = sharding.ShardEncoder(H, W, rank=0, world=1, gather_to=0, gather_kind="stream")
    sharding.encode_group([ss], [device.to_device(rgb)], stream=s)
    whole_s = sharding.gather_streams_group([ss], group=xgroup, rccl=g, stream=s)[0]
    torch.cuda.synchronize()
    got_s = whole_s.result()
    ok &= all(np.array_equal(got_s[k][i], ref[k][i]) for k in pipeline.CHANNELS for i in range(4))
    g.close()
    with open(out_path, "w") as f:
        f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


def test_rccl_world1_exchange():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "result")
        mp.spawn(_rccl_rank, args=(_free_port(), 256, 1024, out), nprocs=1, join=True)
        assert open(out).read() == "ok"
