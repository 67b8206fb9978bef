"""GPU parity: RLE / DPCM / zig-zag kernels, jpeg_encode / jpeg_decode, the
device pipeline and the shard stitching, against the reference's golden outputs
(tests/golden/) and the C oracle at full size."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import oracle.oracle as orc  # noqa: E402
import oracle.oracle_c as orcc  # noqa: E402
from hiccup_amd import (_lib, codec, compression, device, hicimage, model, pipeline, settings,  # noqa: E402
                        sharding, transform)


def _names(d, prefix):
    return sorted(k[len(prefix):] for k in d if k.startswith(prefix))


@pytest.fixture(autouse=True)
def _block_size():
    settings.DEBUG = False
    yield
    settings.JPEG_BLOCK_SIZE = 8


def test_run_length_golden(golden_rle):
    g = golden_rle
    for name in _names(g, "in_"):
        arr, ml = g["in_" + name], int(g["ml_" + name])
        rl = codec.run_length_coding(arr, max_len=(ml if ml else None))
        assert [r.length for r in rl] == g["len_" + name].tolist(), name
        assert [r.value for r in rl] == g["val_" + name].tolist(), name
        dec = codec.decode_run_length(rl, len(arr))
        assert dec == g["dec_" + name].tolist(), name


def test_codectest_cases():
    # codectest.py:20-67,125-191
    rl = codec.run_length_coding(transform.zigzag(np.array([[1, 2], [3, 4]]))[1:])
    assert rl == [codec.RunLength(3, 0), codec.RunLength(2, 0), codec.RunLength(4, 0)]
    assert [s.length for s in codec.run_length_coding(np.array([0] * 17 + [1]), max_len=0xF)] == [14, 2]
    assert codec.run_length_coding(np.array([0, 0, 5]))[-1].is_trailing is False
    assert codec.run_length_coding(np.array([0, 0, 5, 0, 0]))[-1].is_trailing is True
    rle = [codec.RunLength(value=0, length=14), codec.RunLength(value=31, length=0)]
    assert codec.run_length_coding(codec.decode_run_length(rle, 15), max_len=0xF) == rle
    arr = [int(x) for x in np.random.default_rng(3).integers(-5, 5, 10000)]
    assert codec.decode_run_length(codec.run_length_coding(np.array(arr)), 10000) == arr
    with pytest.raises(ZeroDivisionError):
        codec.run_length_coding([1, 0, 2], max_len=0)
    with pytest.raises(TypeError):
        codec.decode_run_length([], 5)


def _decode_i16(L, V, dc, nblk, generic):
    with _lib.knobs(rld_generic=1 if generic else 0):
        return _decode_i16_call(L, V, dc, nblk)


def _decode_i16_call(L, V, dc, nblk):
    lib = _lib.load()
    Ld, Vd, dcd = (device.to_device(np.ascontiguousarray(a)) for a in (L.astype(np.uint8), V.astype(np.int16),
                                                                        dc.astype(np.int32)))
    blocks = torch.full((nblk, 64), -7, dtype=torch.int16, device="cuda")  # poison: every slot must be written
    status = device.zeros((1,), torch.int64)
    ws = device.workspace(lib.hic_rld_workspace_bytes(len(L), nblk))
    _lib.call("hic_rle_decode_i16", device.ptr(Ld), device.ptr(Vd), len(L), device.ptr(dcd), nblk, 64,
              device.ptr(blocks), device.ptr(status), device.ptr(ws), device.stream_ptr())
    return device.to_host(blocks), int(status.cpu()[0])


@pytest.mark.parametrize("kind", ["dense", "sparse", "zero", "last_only", "first_only", "striped", "no_eob",
                                  "dense_long"])
def test_rle_decode_blocks_hot_path(kind, monkeypatch):
    """hic_rle_decode_i16's block-assembling path (LDS windows over 4096-symbol
    tiles, edge blocks shared between tiles, EOB tail fill) against the oracle's
    streams (codec.py:55-113) and against the generic scatter path.  dense_long:
    37.8M symbols, 9.2k symbol tiles, past one 8192-tile chunk of the tile-offset
    scan, so the multi-workgroup scan runs."""
    rng = np.random.default_rng(len(kind))
    nblk = 600_000 if kind == "dense_long" else 5000
    zz = np.zeros((nblk, 64), np.int32)
    if kind in ("dense", "dense_long"):
        zz[:] = rng.integers(-40, 41, (nblk, 64))
    elif kind == "sparse":  # runs far longer than a window, crossing tiles
        m = rng.random((nblk, 64)) < 0.004
        zz[m] = rng.integers(1, 9, m.sum())
    elif kind == "last_only":
        zz[-1, 63] = 5
    elif kind == "first_only":
        zz[0, 1] = -3
    elif kind == "striped":  # dense bands between empty stretches
        band = (np.arange(nblk) // 300) % 2 == 0
        zz[band] = rng.integers(-3, 4, (band.sum(), 64))
    elif kind == "no_eob":
        zz[:] = rng.integers(-5, 6, (nblk, 64))
    zz[:, 0] = rng.integers(-900, 900, nblk)
    ac = zz[:, 1:].reshape(-1)
    L, V = orcc.rle_encode(ac, 15)
    if kind == "no_eob":  # a truncated stream: the remaining positions decode as zeros, status < n_ac
        L, V = L[:-1000], V[:-1000]
    dc = orcc.dpcm(zz[:, 0].copy())
    got, st = _decode_i16(L, V, dc, nblk, False)
    ref, rst = _decode_i16(L, V, dc, nblk, True)
    np.testing.assert_array_equal(got, ref)
    assert st == rst
    if kind != "no_eob":
        np.testing.assert_array_equal(got.astype(np.int32), zz)
        assert st == nblk * 63


def test_rle_long_carried_runs():
    """A nonzero after thousands of all-zero blocks: the cooperative filler path."""
    n = 63 * 5000
    arr = np.zeros(n, np.int64)
    arr[[3, 40000, n - 70000, n - 2]] = [5, -7, 9, 1]
    rl = codec.run_length_coding(arr)
    L, V = orc.rle_encode(arr, 15)
    assert [r.length for r in rl] == L.tolist() and [r.value for r in rl] == V.tolist()
    rl1 = codec.run_length_coding(arr, max_len=1)
    L1, V1 = orc.rle_encode(arr, 1)
    assert [r.length for r in rl1] == L1.tolist() and [r.value for r in rl1] == V1.tolist()


@pytest.mark.parametrize("max_len", [15, 4, 1])
def test_rle_encode_i16_hot_path(max_len):
    """hic_rle_encode_i16 on int16 zig-zag blocks of 64 (the wave-tile hot path):
    dense tiles, sparse tiles, all-zero stretches and a dense tile after a long
    carried run (the unstaged path with wave-cooperative fillers)."""
    rng = np.random.default_rng(max_len)
    nblk = 64 * 40 + 17
    blocks = rng.integers(-40, 41, (nblk, 64)).astype(np.int16)
    blocks[64:200] *= (rng.random((136, 64)) < 0.05)            # sparse
    blocks[300:700, 1:] = 0                                      # long zero stretch (AC only)
    blocks[900:1000] = 0
    blocks[1000:1064] = rng.integers(1, 9, (64, 64))             # dense tile after 100 zero blocks
    blocks[2000:2100, 5:] = 0
    nb = blocks.shape[0]
    ws = device.workspace(_lib.load().hic_rle_workspace_bytes(nb, 64))
    d_blocks = device.to_device(blocks)
    cap = nb * 63 + 1
    L = device.empty((cap,), torch.uint8)
    V = device.empty((cap,), torch.int16)
    dc = device.empty((nb,), torch.int32)
    cnt = device.zeros((1,), torch.int64)
    import ctypes
    _lib.call("hic_rle_encode_i16", device.ptr(d_blocks), nb, 64, max_len, ctypes.c_void_p(0), device.ptr(dc),
              device.ptr(L), device.ptr(V), cap, device.ptr(cnt), device.ptr(ws), device.stream_ptr())
    n = int(device.to_host(cnt)[0])
    eL, eV = orc.rle_encode(blocks[:, 1:].reshape(-1).astype(np.int64), max_len)
    np.testing.assert_array_equal(device.to_host(L)[:n].astype(np.int64), eL)
    np.testing.assert_array_equal(device.to_host(V)[:n].astype(np.int64), eV)
    np.testing.assert_array_equal(device.to_host(dc), orc.dpcm(blocks[:, 0].astype(np.int64)))


def test_jpeg_encode_golden(golden_codec):
    g = golden_codec
    for name in _names(g, "bs_"):
        settings.JPEG_BLOCK_SIZE = int(g["bs_" + name])
        ci = model.CompressedImage(*(g["in_%s_%s" % (ch, name)] for ch in ("lum", "cr", "cb")))
        hic = codec.jpeg_encode(ci)
        p = hic.payloads
        assert len(p) == 20 and hic.hic_type == model.Compression.JPEG
        for k, ch in enumerate(("lum", "cr", "cb")):
            for j, kind in enumerate(("dch", "avh", "alh")):
                table = p[3 * j + k].payloads
                assert [t.numbers[0] for t in table] == g["%sv_%s_%s" % (kind, ch, name)].tolist(), (name, kind)
                assert [t.numbers[1] for t in table] == g["%sc_%s_%s" % (kind, ch, name)].tolist(), (name, kind)
            for j, kind in enumerate(("dcb", "avb", "alb")):
                assert p[9 + 3 * j + k].payload == str(g["%s_%s_%s" % (kind, ch, name)]), (name, kind)
        assert p[18].numbers == tuple(g["shape0_" + name]) and p[19].numbers == tuple(g["shape1_" + name])
        # codectest.py:69-80: first DC table entry of the lum channel
        if name == "t_encode":
            assert p[0].payloads[0].numbers == (1, "1")
        # bytes round trip of the container (hicimagetest.py)
        back = hicimage.HicImage.from_bytes(hic.byte_stream())
        assert all(a == b for a, b in zip(hic.payloads, back.payloads))
        if int(g["decfail_" + name]):
            with pytest.raises(AssertionError):
                codec.jpeg_decode(hic)
        else:
            dec = codec.jpeg_decode(hic)
            for ch in ("lum", "cr", "cb"):
                np.testing.assert_array_equal(dec.as_dict[ch], g["dec_%s_%s" % (ch, name)])
            assert dec == ci


def test_encode_channel_lenna(golden_lenna):
    g = golden_lenna
    for ch in ("cr", "cb"):
        dc, L, V = codec.encode_channel(g["q_" + ch])
        np.testing.assert_array_equal(dc, g["dc_" + ch])
        np.testing.assert_array_equal(L, g["acl_" + ch])
        np.testing.assert_array_equal(V, g["acv_" + ch])
    dc, L, V = codec.encode_channel(g["q_y"][:256])
    np.testing.assert_array_equal(L, g["acl_y256"])
    np.testing.assert_array_equal(V, g["acv_y256"])


COLOUR_SHAPES = ((64, 64), (37, 50), (130, 258), (2, 2), (3, 7), (1080, 1920), (4, 4), (5, 4), (9, 8), (2, 8),
                 (33, 252), (35, 500), (71, 996), (64, 7680))


@pytest.mark.parametrize("variant", [{}, {"color_seg": 16}, {"color_tiled": 1}])
def test_colour_kernels_vs_restatement(variant):
    with _lib.knobs(**variant):
        _colour_kernels_vs_restatement()


def _colour_kernels_vs_restatement():
    rng = np.random.default_rng(8)
    for H, W in COLOUR_SHAPES:
        rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        y, cr, cb = compression.ycrcb420_device(device.to_device(rgb))
        ry, rcr, rcb = orcc.rgb_to_ycrcb(rgb)
        np.testing.assert_array_equal(device.to_host(y), ry, err_msg=str((H, W)))
        np.testing.assert_array_equal(device.to_host(cr), orcc.pyr_down(rcr), err_msg=str((H, W)))
        np.testing.assert_array_equal(device.to_host(cb), orcc.pyr_down(rcb), err_msg=str((H, W)))
        if H >= 2 and W >= 2:
            np.testing.assert_array_equal(transform.down_sample(ry), orcc.pyr_down(ry))
        np.testing.assert_array_equal(transform.up_sample(rcr), orcc.pyr_up(rcr))
    # transformtest.py:122-146
    np.testing.assert_array_equal(transform.up_sample(np.full((2, 2), 2, np.uint8)), np.full((4, 4), 2, np.uint8))
    np.testing.assert_array_equal(transform.down_sample(np.full((4, 4), 2, np.uint8)), np.full((2, 2), 2, np.uint8))


@pytest.mark.parametrize("variant", [{}, {"color_tiled": 1}])
def test_decode_colour_vs_restatement(variant):
    """hic_ycrcb420_to_rgb (pyrUp of both chroma planes, crop of Y, YCrCb -> RGB:
    compression.py:51-56, transform.py:151-158,269-277) against the restatement,
    every shape of COLOUR_SHAPES plus a wide multi-strip plane."""
    with _lib.knobs(**variant):
        _decode_colour_vs_restatement()


def _decode_colour_vs_restatement():
    rng = np.random.default_rng(9)
    for H, W in COLOUR_SHAPES + ((34, 16384 + 6),):
        h, w = H // 2, W // 2
        if h == 0 or w == 0:
            continue
        y = rng.integers(0, 256, (H, W), dtype=np.uint8)
        cr = rng.integers(0, 256, (h, w), dtype=np.uint8)
        cb = rng.integers(0, 256, (h, w), dtype=np.uint8)
        yd, crd, cbd = (device.to_device(a) for a in (y, cr, cb))
        out = device.empty((2 * h, 2 * w, 3), torch.uint8)
        _lib.call("hic_ycrcb420_to_rgb", device.ptr(yd), yd.stride(0), device.ptr(crd), device.ptr(cbd), h, w,
                  device.ptr(out), device.stream_ptr())
        exp = orcc.ycrcb_to_rgb(y[:2 * h, :2 * w], orcc.pyr_up(cr), orcc.pyr_up(cb))
        np.testing.assert_array_equal(device.to_host(out), exp, err_msg=str((H, W)))


def test_jpeg_compression_roundtrip(golden_lenna):
    g = golden_lenna
    ci = compression.jpeg_compression(g["rgb"])
    np.testing.assert_array_equal(ci.luminance_component, g["q_y"])
    np.testing.assert_array_equal(ci.red_chrominance_component, g["q_cr"])
    np.testing.assert_array_equal(ci.blue_chrominance_component, g["q_cb"])
    rgb = compression.jpeg_decompression(ci)
    up = lambda p: orcc.pyr_up(p)  # noqa: E731
    exp = orcc.ycrcb_to_rgb(g["rec_y"], up(g["rec_cr"]), up(g["rec_cb"]))
    np.testing.assert_array_equal(rgb, exp)
    err = np.abs(rgb.astype(np.int32) - g["rgb"].astype(np.int32)).mean()
    assert err < 6.0


def _oracle_encode(rgb):
    y, cr, cb = orcc.rgb_to_ycrcb(rgb)
    planes = {"lum": (y, 0), "cr": (orcc.pyr_down(cr), 1), "cb": (orcc.pyr_down(cb), 1)}
    out = {}
    for k, (p, t) in planes.items():
        q = orcc.dct_channel(p, t, threads=16)
        zz = orcc.zigzag_blocks(q, 8)
        L, V = orcc.rle_encode(zz[:, 1:].reshape(-1), 15)
        out[k] = (zz, orcc.dpcm(zz[:, 0].copy()), L, V)
    return out


@pytest.mark.parametrize("H,W", [(64, 96), (4320, 7680), (250, 330), (512, 768), (512, 1024), (272, 1536),
                                 (2160, 3840), (1088, 1920), (32, 16)])
def test_pipeline_encoder(H, W):
    """The device encoder vs the C oracle, on its default path (fused when W % 512
    == 0 and H % 16 == 0, else the two-kernel chain) and, for any W, H multiples of
    16, on the fused kernel (W % 512 != 0: a ragged last strip)."""
    rng = np.random.default_rng(H)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    if H in (250, 272):
        rgb[:, :100] = 128  # flat region: all-zero AC blocks, long runs
    if H == 512:  # few grey levels: exact quantiser ties on the fast DCT path
        rgb = (rng.integers(0, 4, (H, W, 1)) * 85).astype(np.uint8).repeat(3, 2)
    enc = pipeline.Encoder(H, W)
    assert enc.fused == (W % 16 == 0 and H % 16 == 0)
    assert enc.seg == (enc.fused and W % 512 != 0)
    exp = _oracle_encode(rgb)
    # the fused kernel with a tile pass for a ragged last strip (an encoder with a tile
    # index) and the two-kernel chain beside the default
    variants = [enc]
    if enc.seg:
        variants += [pipeline.Encoder(H, W, fused=True, index=True), pipeline.Encoder(H, W, fused=False)]
    for e in variants:
        e.encode(device.to_device(rgb))
        got_e = e.result()
        for k in pipeline.CHANNELS:
            zz, dc, L, V = got_e[k]
            ezz, edc, eL, eV = exp[k]
            np.testing.assert_array_equal(zz.astype(np.int32), ezz, err_msg=(k, e.fused))
            np.testing.assert_array_equal(dc, edc, err_msg=(k, e.fused))
            np.testing.assert_array_equal(L.astype(np.int32), eL, err_msg=(k, e.fused))
            np.testing.assert_array_equal(V.astype(np.int32), eV, err_msg=(k, e.fused))
    got = enc.result()
    # decode back through the device chain: equals the oracle's inverse
    dec = pipeline.Decoder(H, W)
    dev = {k: (device.to_device(got[k][2]), device.to_device(got[k][3]), device.to_device(got[k][1]))
           for k in pipeline.CHANNELS}
    counts = [len(got[k][2]) for k in pipeline.CHANNELS]
    rgb2 = device.to_host(dec.decode({k: v[0] for k, v in dev.items()}, {k: v[1] for k, v in dev.items()}, counts,
                                     {k: v[2] for k, v in dev.items()}))
    assert np.all(dec.status.cpu().numpy() == [len(got[k][0]) * 63 for k in pipeline.CHANNELS])
    rec = {}
    for k, (p, t) in {"lum": (H, 0), "cr": (0, 1), "cb": (0, 1)}.items():
        zz = exp[k][0]
        h, w = (H, W) if k == "lum" else (H // 2, W // 2)
        raster = orc.merge_blocks(zz[:, np.argsort(orc.ZZ8)].reshape(-1, 8, 8), (h, w))
        rec[k] = orcc.inv_dct_channel(raster, t)
    h, w = H // 2, W // 2
    exp_rgb = orcc.ycrcb_to_rgb(rec["lum"][:2 * h, :2 * w], orcc.pyr_up(rec["cr"]), orcc.pyr_up(rec["cb"]))
    np.testing.assert_array_equal(rgb2, exp_rgb)


_IDX_SHAPES = [(64, 96), (512, 1024), (272, 1536), (1088, 1920), (4320, 7680), (16, 16), (250, 330), (37, 53),
               (24, 40), (40, 24), (8, 8), (16, 512), (48, 1536)]


# slots False only where the default is the slot layout (elsewhere it is the same case)
@pytest.mark.parametrize("kind", ["random", "levels", "blocks", "flat"])
@pytest.mark.parametrize("H,W,slots", [(h, w, None) for h, w in _IDX_SHAPES] +
                         [(h, w, False) for h, w in _IDX_SHAPES if pipeline.slots_eligible(h, w)])
def test_indexed_decode(H, W, kind, slots):
    """Encoder(index=True) + Decoder.decode(index=...): one wave per 64-block
    tile from the encoder-side index, counts read on the device -- the blocks and
    RGB equal the plain decode's, the status equals nblk * 63, on fused (half-tile
    chroma records) and two-kernel-chain encoders, with empty tiles and long
    carried runs (flat).  slots None: the default, which for W % 512 == 0 is the
    slot layout (the decoders read the slots through the close's record index);
    False: the coefficient chain's tile index.  (24, 40) / (40, 24): chroma planes of
    half blocks beside whole luma blocks; (8, 8): one block."""
    if kind == "blocks" and (H % 8 or W % 8):
        pytest.skip("the blocks image needs whole 8x8 blocks")
    rgb = _structured_rgb(kind, H, W, H * 7 + W)
    enc = pipeline.Encoder(H, W, index=True, slots=slots)
    assert enc.slots == (slots is None and pipeline.slots_eligible(H, W))
    enc.encode(device.to_device(rgb))
    enc.materialize()  # slot layout: the contiguous stream and the blocks, for the plain decode
    counts = enc.counts.cpu().tolist()
    # the index the emit wrote (hic_rle_job16.d_index) == hic_rle_tile_index_i16's
    for k in pipeline.CHANNELS:
        if enc.slots:
            break
        ix = torch.full_like(enc.index[k], -5)
        _lib.call("hic_rle_tile_index_i16", device.ptr(enc.coef[k]), enc.coef[k].shape[0], enc.rpt[k],
                  device.ptr(enc.ws[k]), device.ptr(ix), device.stream_ptr())
        assert torch.equal(ix, enc.index[k]), k
    d1, d2, d3 = pipeline.Decoder(H, W), pipeline.Decoder(H, W), pipeline.Decoder(H, W)
    r1 = d1.decode(enc.sym_len, enc.sym_val, counts, enc.dc)
    r2 = d2.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index, keep_blocks=True)
    torch.cuda.synchronize()
    for k in pipeline.CHANNELS:
        assert torch.equal(d2.blocks[k], enc.coef[k]), k
        assert torch.equal(d1.blocks[k], d2.blocks[k]), k
    want = [enc.coef[k].shape[0] * 63 for k in pipeline.CHANNELS]
    assert d2.status.cpu().tolist() == want
    assert torch.equal(r1, r2)
    # the fused decode + IDCT (no blocks in HBM): the same planes and RGB
    r3 = d3.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index, planes=True)
    torch.cuda.synchronize()
    for k in pipeline.CHANNELS:
        assert torch.equal(d3.pix[k], d1.pix[k]), k
    assert d3.status.cpu().tolist() == want
    assert torch.equal(r1, r3)
    # whole blocks: the luminance decode goes straight to RGB (hic_rle_decode_idct_rgb_indexed,
    # no Y plane); ragged planes keep the planes path.  Same chroma planes, same RGB.
    d4 = pipeline.Decoder(H, W)
    d4.pix["lum"].fill_(0)
    r4 = d4.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index)
    torch.cuda.synchronize()
    for k in ("cr", "cb"):
        assert torch.equal(d4.pix[k], d1.pix[k]), k
    assert d4.status.cpu().tolist() == want
    assert torch.equal(r1, r4)
    assert bool(d4.pix["lum"].any()) == (H % 8 != 0 or W % 8 != 0)  # which path ran
    # Cr and Cb in one launch (the default) or one launch each: the same
    d5 = pipeline.Decoder(H, W, chroma_pair=False)
    assert torch.equal(d5.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index), r1)
    for k in ("cr", "cb"):
        assert torch.equal(d5.pix[k], d4.pix[k]), k


@pytest.mark.parametrize("mode", ["rgb", "planes", "blocks"])
@pytest.mark.parametrize("W", [192, 512])
def test_indexed_decode_failed_count(mode, W):
    """A failed encode's symbol count (< 1) decodes nothing of that channel and
    reports status -1 (include/hiccup_hip.h, hic_rle_decode_i16_indexed) on every
    indexed form -- the fused RGB kernel, the per-plane decode-IDCT, the block
    decode -- while the other channels decode as usual (W 512: the slot layout's
    decoders)."""
    H = 128
    enc = pipeline.Encoder(H, W, index=True)
    assert enc.slots == (W == 512)
    enc.encode(device.to_device(_structured_rgb("random", H, W, 11)))
    good = pipeline.Decoder(H, W)
    r_good = good.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index).clone()
    for ch in range(3):
        counts = enc.counts.clone()
        counts[ch] = 0
        dec = pipeline.Decoder(H, W)
        dec.decode(enc.sym_len, enc.sym_val, counts, enc.dc, index=enc.index,
                   planes=(mode == "planes"), keep_blocks=(mode == "blocks"))
        st = dec.status.cpu().tolist()
        want = [enc.coef[k].shape[0] * 63 for k in pipeline.CHANNELS]
        want[ch] = -1
        assert st == want, (ch, st)
        with pytest.raises(ValueError):
            dec.check_status()
    good.check_status()
    assert r_good.any()


def _structured_rgb(kind, H, W, seed):
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    if kind == "levels":  # 4 grey levels: exact ties at DC / (4,4) / the (2,2) class
        return (rng.integers(0, 4, (H, W, 1)) * 85).astype(np.uint8).repeat(3, 2)
    if kind == "colour_levels":  # 2 levels per channel independently
        return (rng.integers(0, 2, (H, W, 3)) * 255).astype(np.uint8)
    if kind == "blocks":  # constant 8x8 blocks and symmetric 2x2 patterns
        b = rng.integers(0, 256, (H // 8, W // 8, 3), dtype=np.uint8)
        img = b.repeat(8, 0).repeat(8, 1)
        img[::2, ::2] = 255 - img[::2, ::2]
        return img
    if kind == "flat":  # all-zero AC runs spanning whole strips and unit rows
        img = np.full((H, W, 3), 128, np.uint8)
        img[H // 2:H // 2 + 3, W // 3] = 7
        return img
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["random", "levels", "colour_levels", "blocks", "flat"])
@pytest.mark.parametrize("H,W", [(16, 512), (144, 2048), (1088, 1536)])
def test_fused_encoder_matches_two_kernel_chain(kind, H, W):
    """hic_encode420_u8 (colour + pyrDown + DCT + tile records in one kernel, exact
    tie fallbacks in place) == the two-kernel chain (hic_rgb_to_ycrcb420 +
    hic_dct_quant_rle_u8_batch), symbols and DC streams included (the fused chroma
    records are 32-block half tiles)."""
    rgb = _structured_rgb(kind, H, W, H + W)
    x = device.to_device(rgb)
    exp = pipeline.Encoder(H, W, fused=False)
    exp.encode(x)
    b = exp.result()
    # the fused kernel writing coefficients + records, and (W % 512 == 0) the slot layout
    encs = [pipeline.Encoder(H, W, fused=True, slots=False)]
    if pipeline.slots_eligible(H, W):
        encs.append(pipeline.Encoder(H, W, fused=True))
        assert encs[-1].slots
    for got in encs:
        got.encode(x)
        a = got.result()
        for k in pipeline.CHANNELS:
            for j, what in enumerate(("coef", "dc", "sym_len", "sym_val")):
                np.testing.assert_array_equal(a[k][j], b[k][j], err_msg="%s %s slots %s" % (k, what, got.slots))
    # the shard summaries read the half-tile records (a whole ragged image keeps one
    # record per strip segment instead: no shard summaries)
    got = encs[0]
    if not got.seg:
        np.testing.assert_array_equal(got.shard_summaries().cpu().numpy(), exp.shard_summaries().cpu().numpy())


@pytest.mark.parametrize("kind", ["random", "levels", "blocks", "flat"])
@pytest.mark.parametrize("H,W", [(2160, 3840), (1088, 1920), (32, 528), (48, 16), (16, 1040), (2048, 16),
                                 (1024, 48)])
def test_fused_encoder_ragged_matches_chain(kind, H, W):
    """Widths that are not a multiple of 512: the fused kernel's last strip is
    ragged (lanes past W store nothing, the right-border pixel goes to the strip's
    last lane); the whole image's encoder writes one RLE record per strip segment
    (hic_encode420_seg_u8) and the scan / emit walk row segments -- symbols and DC
    equal the two-kernel chain's; with a tile index the records come from a tile
    pass after the launch (hic_encode420_u8), equal too.  2048x16 and 1024x48 are
    the narrow, tall shapes whose segment records outnumber their 64-block tiles
    (ADVICE r4)."""
    test_fused_encoder_matches_two_kernel_chain(kind, H, W)
    rgb = _structured_rgb(kind, H, W, H + W)
    x = device.to_device(rgb)
    got, exp = pipeline.Encoder(H, W, fused=True, index=True), pipeline.Encoder(H, W, fused=False)
    assert not got.seg
    got.encode(x)
    exp.encode(x)
    a, b = got.result(), exp.result()
    for k in pipeline.CHANNELS:
        for j, what in enumerate(("coef", "dc", "sym_len", "sym_val")):
            np.testing.assert_array_equal(a[k][j], b[k][j], err_msg="%s %s" % (k, what))


@pytest.mark.parametrize("order", [0, 2, 4, 6])
@pytest.mark.parametrize("kind", ["random", "levels", "flat"])
@pytest.mark.parametrize("H,W", [(16, 512), (48, 1024), (80, 2048), (272, 1536), (144, 1040), (2160, 3840)])
def test_fused_encoder_unit_order(kind, H, W, order):
    """knob encode_order (0: a workgroup = 4 strips side by side; + 2: workgroups
    remapped XCD-major; + 4: odd unit rows run their colour rows bottom-up; ragged
    last strips included) == the two-kernel chain."""
    with _lib.knobs(encode_order=order):
        test_fused_encoder_matches_two_kernel_chain(kind, H, W)


@pytest.mark.parametrize("H,W", [(2048, 16), (1024, 48), (4096, 32)])
def test_seg_workspace_canary_and_refusal(H, W):
    """the row-segment records of a narrow, tall image need more
    workspace than its 64-block tiles.  Every workspace is followed by a canary that
    must survive the fused encode and the scan / emit (nothing is written past the
    size hic_rle_rows_workspace_bytes gives), and a workspace one record short is
    refused by both the fused kernel's launcher and the rows batch (HIC_ERR_ARG,
    nothing launched)."""
    lib = _lib.load()
    rgb = device.to_device(np.random.default_rng(W).integers(0, 256, (H, W, 3), dtype=np.uint8))
    enc = pipeline.Encoder(H, W)
    assert enc.seg
    canary = 0x5A5A5A5A5A5A5A5A
    for k in pipeline.CHANNELS:
        n = enc.ws[k].numel()
        buf = device.zeros((n + 64,), torch.int64)
        buf[n:] = canary
        enc.ws[k] = buf
    enc.encode(rgb)
    ref = pipeline.Encoder(H, W, fused=False)
    ref.encode(rgb)
    a, b = enc.result(), ref.result()
    for k in pipeline.CHANNELS:
        n = enc.ws[k].numel() - 64
        assert (enc.ws[k][n:] == canary).all().item(), k
        for j in range(4):
            np.testing.assert_array_equal(a[k][j], b[k][j], err_msg=k)
    # one record (3 words) short: refused
    r0 = enc.ws_bytes["lum"]
    enc.ws_bytes["lum"] = r0 - 24
    with pytest.raises(ValueError, match="workspace"):
        enc.transform(rgb)
    with pytest.raises(ValueError, match="workspace"):
        enc.entropy()
    enc.ws_bytes["lum"] = r0
    tiles = lib.hic_rle_workspace_bytes(enc.coef["lum"].shape[0], 64)
    assert tiles < r0  # the tile-sized workspace the advisor found too small


@pytest.mark.timeout(900)
def test_16k_roundtrip_vs_oracle():
    """BASELINE configs[4] on one GPU: a 16384 x 16384 random RGB image (the
    config's seed) through the device encoder and decoder.  The encoder's
    coefficients, DC differences and both symbol arrays equal the CPU restatement's
    (the C oracle's colour, DCT, zig-zag, DPCM and RLE of the whole image; round 4,
    before only properties of the stream were checked at this size), the stream's
    properties hold (counts, DC integration, EOB), and the reconstruction is
    bit-exact against the restatement of the reference's chain (cvtColor ->
    pyrDown -> dct_channel -> inv_dct_channel -> pyrUp -> cvtColor,
    compression.py:16-56); PSNR vs the input is the same number."""
    H = W = 16384
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    enc = pipeline.Encoder(H, W, index=True)
    enc.encode(device.to_device(rgb))
    got = enc.result()
    exp = _oracle_encode(rgb)
    for k in pipeline.CHANNELS:
        for j, what in enumerate(("coef", "dc", "sym_len", "sym_val")):
            np.testing.assert_array_equal(np.asarray(got[k][j]).astype(np.int32), exp[k][j], err_msg=(k, what))
    del got, exp
    counts = enc.counts.cpu().tolist()
    nblk = {k: enc.coef[k].shape[0] for k in pipeline.CHANNELS}
    for k, c in zip(pipeline.CHANNELS, counts):
        assert 0 < c <= nblk[k] * 63 + 1, k
    dec = pipeline.Decoder(H, W)
    rec_dev = dec.decode(enc.sym_len, enc.sym_val, counts, enc.dc)
    # every AC position of every block was reconstructed from the stream
    assert dec.status.cpu().tolist() == [nblk[k] * 63 for k in pipeline.CHANNELS]
    # the decoder's blocks are the encoder's coefficients (RLE / DPCM inverse)
    for k in pipeline.CHANNELS:
        assert torch.equal(dec.blocks[k], enc.coef[k]), k
    rec = device.to_host(rec_dev)
    # the indexed decode (encoder-side tile index, device counts): the same
    dec2 = pipeline.Decoder(H, W)
    rec2 = dec2.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index, keep_blocks=True)
    assert dec2.status.cpu().tolist() == [nblk[k] * 63 for k in pipeline.CHANNELS]
    for k in pipeline.CHANNELS:
        assert torch.equal(dec2.blocks[k], enc.coef[k]), k
    assert torch.equal(rec2, rec_dev)
    rec3 = dec2.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index)  # fused decode + IDCT
    assert dec2.status.cpu().tolist() == [nblk[k] * 63 for k in pipeline.CHANNELS]
    assert torch.equal(rec3, rec_dev)
    del dec2, rec2, rec3
    del enc, dec, rec_dev
    torch.cuda.empty_cache()
    y, cr, cb = orcc.rgb_to_ycrcb(rgb)
    ry = orcc.inv_dct_channel(orcc.dct_channel(y, 0, threads=16), 0)
    rc = [orcc.pyr_up(orcc.inv_dct_channel(orcc.dct_channel(orcc.pyr_down(c), 1, threads=16), 1)) for c in (cr, cb)]
    exp = orcc.ycrcb_to_rgb(ry, rc[0], rc[1])
    np.testing.assert_array_equal(rec, exp)
    mse = np.mean((rec.astype(np.float64) - rgb) ** 2)
    assert 10 * np.log10(255.0 ** 2 / mse) > 10.0


@pytest.mark.parametrize("H,W,world,flat", [(4320, 7680, 8, None), (250, 330, 3, None), (96, 64, 2, None),
                                            (144, 96, 3, (48, 96)), (2160, 3840, 3, None)])
def test_shards_stitch_to_single_stream(H, W, world, flat):
    """Row shards (with pyrDown halos) + the stitch record reproduce the
    single-GPU stream exactly, and each shard's decode of its own slice
    (ShardDecoder: carried zeros skipped, DC chain from the stitch record, pyrUp
    halo rows from the neighbours) reproduces its rows of the single-GPU decode
    (the multi-GPU path, simulated on one device; flat = a shard with no nonzero
    luma AC, so a carried run chains through it)."""
    rng = np.random.default_rng(W)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rgb[H // 3: H // 3 + 40] = 128  # zero runs that cross shard boundaries
    if flat:
        rgb[flat[0]:flat[1]] = 128
    whole = pipeline.Encoder(H, W)
    whole.encode(device.to_device(rgb))
    ref = whole.result()
    encs = []
    for rows in sharding.plan(H, world):
        e = pipeline.Encoder(H, W, rows=rows)
        a, b = e.input_span()
        e.transform(device.to_device(rgb[a:b]))
        encs.append(e)
    summ = np.stack([e.shard_summaries().cpu().numpy() for e in encs])  # (world, 3, 4)
    allsum = device.to_device(summ)
    stitches = []
    for r, e in enumerate(encs):
        st = device.zeros((3, 4), torch.int64)
        for c in range(3):
            import ctypes
            _lib.call("hic_rle_stitch", ctypes.c_void_p(allsum.data_ptr() + 32 * c), world, r, 12,
                      device.ptr(st[c]), device.stream_ptr())
            np.testing.assert_array_equal(st[c].cpu().numpy(), sharding.stitch_host(summ[:, c], r))
        e.entropy(stitch=st)
        stitches.append(st)
    parts = [e.result() for e in encs]
    for k in pipeline.CHANNELS:
        zz = np.concatenate([p[k][0] for p in parts])
        np.testing.assert_array_equal(zz, ref[k][0], err_msg=k)
        for j in (1, 2, 3):
            np.testing.assert_array_equal(np.concatenate([p[k][j] for p in parts]), ref[k][j], err_msg=(k, j))
    # sharded decode: every shard decodes its own slice; the halo rows are copied
    # between the shards' buffers here (exchange_halo_rows does it over RCCL)
    whole_dec = pipeline.Decoder(H, W)
    exp = device.to_host(whole_dec.decode(whole.sym_len, whole.sym_val, whole.counts.cpu().tolist(), whole.dc))
    decs = [sharding.ShardDecoder(H, W, rank=r, world=world) for r in range(world)]
    for d, e, st in zip(decs, encs, stitches):
        d.planes(e.sym_len, e.sym_val, e.counts.cpu().tolist(), e.dc, st)
    for r, d in enumerate(decs):
        for (buf, top, n), k in zip(d.halo_views(), ("cr", "cb")):
            if r > 0:
                pb, pt, pn = decs[r - 1].halo_views()[0 if k == "cr" else 1]
                buf[0].copy_(pb[pt + pn - 1])
            if r < world - 1:
                nb, nt, _ = decs[r + 1].halo_views()[0 if k == "cr" else 1]
                buf[top + n].copy_(nb[nt])
    for r, d in enumerate(decs):
        got = device.to_host(d.colour())
        d.check_status()
        a, b = d.out_rows
        np.testing.assert_array_equal(got, exp[a:b], err_msg="rank %d" % r)


@pytest.mark.timeout(600)
def test_shards_stitch_16k():
    """BASELINE configs[4]'s size (16384 x 16384) over 8 shards: sharded encode
    == the whole stream, every shard's decode == its rows of the whole decode."""
    test_shards_stitch_to_single_stream(16384, 16384, 8, None)


@pytest.mark.parametrize("H,W", [(1088, 1920), (1088, 2048)])
def test_two_stream_overlap_matches_single_stream(H, W):
    """bench.py's default: consecutive images alternate over two HIP streams with 4
    rotating encoders.  Every encoder's output after the overlapped run equals a
    one-stream encode of the same image (no buffer shared across streams; W 2048:
    the slot layout)."""
    rng = np.random.default_rng(11)
    imgs = [device.to_device(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)) for _ in range(3)]
    encs = [pipeline.Encoder(H, W) for _ in range(4)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    last = {}
    for i in range(12):
        with torch.cuda.stream(streams[i % 2]):
            encs[i % 4].encode(imgs[i % 3])
        last[i % 4] = i % 3
    torch.cuda.synchronize()
    ref = {}
    for j in range(3):
        e = pipeline.Encoder(H, W)
        e.encode(imgs[j])
        ref[j] = e.result()
    for n, e in enumerate(encs):
        got, exp = e.result(), ref[last[n]]
        for k in pipeline.CHANNELS:
            for a, b in zip(got[k], exp[k]):
                np.testing.assert_array_equal(a, b, err_msg="%d %s" % (n, k))


@pytest.mark.parametrize("dtype,kind", [(np.uint8, "lengths"), (np.int16, "values"), (np.int32, "dc"),
                                        (np.int16, "single"), (np.int32, "skewed"), (np.uint8, "tail")])
def test_huffman_device_vs_host(dtype, kind):
    """GPU histogram (first-appearance order) + GPU bit packing == the host tree
    builder and string encoder (huffman.py, pinned against the reference's golden
    tables and bit strings in test_cpu_host / test_jpeg_encode_golden)."""
    from hiccup_amd import huffman
    rng = np.random.default_rng(hash(kind) % 1000)
    n = 300_001
    if kind == "lengths":
        keys = rng.integers(0, 15, n)
    elif kind == "values":
        keys = np.round(rng.laplace(0, 40, n)).clip(-3277, 3277)
    elif kind == "dc":
        keys = rng.integers(-4096, 4097, n)
    elif kind == "single":
        keys = np.full(n, -7)
    elif kind == "skewed":  # deep trees: long codes
        keys = (rng.geometric(0.5, n) - 1) * 3 - 40
    else:  # a few rare keys at the end of the stream
        keys = np.concatenate([rng.integers(0, 3, n - 5), [200, 201, 250, 255, 0]])
    keys = keys.astype(dtype)
    ds = huffman.DeviceStream(device.to_device(keys))
    uniq, counts = huffman.first_appearance_counts(keys)
    assert ds.keys_in_order == uniq
    host = huffman.HuffmanTree.construct_from_counts(uniq, counts)
    assert ds.tree.encode_table() == host.encode_table()
    packed, nbits = ds.packed()
    bits = host.encode_keys(keys)
    assert nbits == len(bits)
    got = hicimage.BitStringP.from_packed(packed, nbits)
    assert got.payload == bits
    assert got.byte_stream == hicimage.BitStringP(bits).byte_stream


@pytest.mark.parametrize("kind", ["lengths", "values", "dc", "single", "skewed", "tail", "equal8"])
def test_huffman_decode_device(kind):
    """hic_huffman_decode (speculative subsequences + resynchronisation + the
    serial chain) == the reference's bit walk (decode_data), on trees rebuilt from
    the tables as jpeg_decode builds them: short codes, codes past the 12-bit
    lookup (skewed), a one-symbol table, and equal 3-bit codes that never
    resynchronise on 1024-bit subsequences (equal8: the chain path)."""
    from hiccup_amd import huffman
    rng = np.random.default_rng(len(kind))
    n = 200_003
    if kind == "lengths":
        keys = rng.integers(0, 15, n)
    elif kind == "values":
        keys = np.round(rng.laplace(0, 40, n)).clip(-3277, 3277)
    elif kind == "dc":
        keys = rng.integers(-4096, 4097, n)
    elif kind == "single":
        keys = np.full(n, -7)
    elif kind == "skewed":
        keys = (rng.geometric(0.35, n) - 1) * 3 - 40
    elif kind == "equal8":
        keys = rng.integers(0, 8, n)
    else:
        keys = np.concatenate([rng.integers(0, 3, n - 5), [200, 201, 250, 255, 0]])
    keys = keys.astype(np.int32)
    ds = huffman.DeviceStream(device.to_device(keys))
    packed, nbits = ds.packed()
    codes = ds.tree.codes()
    if kind == "skewed":
        assert max(len(c) for c in codes.values()) > 12
    if kind == "equal8":
        assert set(len(c) for c in codes.values()) == {3}
    dec = huffman.HuffmanTree.construct_from_coding(ds.tree.encode_table())
    assert dec.decode_packed(packed, nbits) == keys.tolist()
    # trailing bits that finish no code are dropped (the reference's reduce)
    ends = np.cumsum([len(codes[int(k)]) for k in keys])
    for cut in (1, 2, 5):
        m = int(np.searchsorted(ends, nbits - cut, side="right"))
        assert dec.decode_packed(packed, nbits - cut) == keys[:m].tolist()


def test_huffman_decode_device_edges():
    """Empty and one-bit streams, a table whose unused codes decode to None, a
    one-leaf encoding tree's missing '0' child (AttributeError, as the reference's
    walk raises), and a stream too short for one subsequence."""
    from hiccup_amd import huffman
    t = huffman.HuffmanTree.construct_from_coding([(5, "1")])  # "0" decodes to None
    for bits in ["", "1", "0", "10", "0110", "1" * 3000 + "0" * 77]:
        bsp = hicimage.BitStringP(bits)
        assert t.decode_packed(*bsp.packed_bits()) == t.decode_data(bits), bits
    single = huffman.HuffmanTree.construct_from_data([3, 3, 3])
    assert single.decode_packed(*hicimage.BitStringP("111").packed_bits()) == [3, 3, 3]
    with pytest.raises(AttributeError):
        single.decode_packed(*hicimage.BitStringP("1" * 5000 + "0" + "1" * 5000).packed_bits())
    tree = huffman.HuffmanTree.construct_from_data([1, 2, 2, 3, 3, 3, 4, 4, 4, 4])
    for bits in ["001", "0010001", "01" * 700 + "0"]:
        assert tree.decode_packed(*hicimage.BitStringP(bits).packed_bits()) == tree.decode_data(bits)


@pytest.mark.parametrize("N", [2, 3, 8])
def test_transform_batch_equals_shard_launches(N):
    """pipeline.transform_batch (hic_encode420_batch_u8: a multi-GPU group's row
    shards, one per image, in one launch) writes the same coefficients and RLE tile
    records as one hic_encode420_u8 launch per shard; its timing events all span the
    launch; a group it cannot batch (W % 512 != 0) runs shard by shard."""
    H, W = 1088, 1024
    imgs = [device.to_device(np.random.default_rng(N + i).integers(0, 256, (H, W, 3), dtype=np.uint8))
            for i in range(N)]
    rows = sharding.plan(H, N)
    # shard j of image j (a group: image j's shard for this rank is its j-th)
    def make():
        return [pipeline.Encoder(H, W, rows=rows[j]) for j in range(N)]
    one, bat = make(), make()
    spans = [e.input_span() for e in one]
    ins = [imgs[j][spans[j][0]:spans[j][1]] for j in range(N)]
    assert all(e.batchable() for e in one)
    for e, x, sp in zip(one, ins, spans):
        e.transform(x, in_row0=sp[0])
    evs = [device.KernelEvents() if j % 2 == 0 else None for j in range(N)]
    pipeline.transform_batch(bat, ins, in_row0s=[sp[0] for sp in spans], dct_events=evs)
    torch.cuda.synchronize()
    for a, b in zip(one, bat):
        for k in pipeline.CHANNELS:
            assert torch.equal(a.coef[k], b.coef[k]), k
            assert torch.equal(a.ws[k], b.ws[k]), k
    assert all(ev.elapsed_ms() > 0 for ev in evs if ev is not None)
    # W % 512 != 0: not batchable, one launch per shard, same result
    W2 = 768
    img2 = device.to_device(np.random.default_rng(7).integers(0, 256, (H, W2, 3), dtype=np.uint8))
    e1 = [pipeline.Encoder(H, W2, rows=rows[j]) for j in range(N)]
    e2 = [pipeline.Encoder(H, W2, rows=rows[j]) for j in range(N)]
    assert not any(e.batchable() for e in e1)
    sp2 = [e.input_span() for e in e1]
    for e, sp in zip(e1, sp2):
        e.transform(img2[sp[0]:sp[1]], in_row0=sp[0])
    pipeline.transform_batch(e2, [img2[sp[0]:sp[1]] for sp in sp2], in_row0s=[sp[0] for sp in sp2])
    for a, b in zip(e1, e2):
        for k in pipeline.CHANNELS:
            assert torch.equal(a.coef[k], b.coef[k]), k


@pytest.mark.parametrize("kind", ["random", "wide", "ragged"])
def test_jpeg_encode_int16_path_equals_int32(kind, monkeypatch):
    """jpeg_encode's 8x8 fast path (int16 zig-zag blocks + the 16-bit RLE) writes the
    same container as the int32 path (forced by reporting every plane wide), and a
    plane holding a coefficient outside int16 falls back to the int32 path by
    itself (the fast path's blocks of it are not exact)."""
    rng = np.random.default_rng({"random": 1, "wide": 2, "ragged": 3}[kind])
    H, W = (123, 205) if kind == "ragged" else (256, 384)
    planes = [rng.integers(-300, 301, (H, W)).astype(np.int32),
              rng.integers(-60, 61, ((H + 1) // 2, (W + 1) // 2)).astype(np.int32),
              rng.integers(-60, 61, ((H + 1) // 2, (W + 1) // 2)).astype(np.int32)]
    planes[0][::8, ::8] = rng.integers(-2000, 2001, planes[0][::8, ::8].shape)  # DC-like values
    if kind == "wide":
        planes[1][5, 9] = 40000
        planes[0][17, 3] = -33000
    ci = model.CompressedImage(*planes)
    settings.JPEG_BLOCK_SIZE = 8
    fast = codec.jpeg_encode(ci).byte_stream()
    real = codec.encode_channel_device8

    def forced_wide(*a, **k):
        dc, L, V, cnt, wide = real(*a, **k)
        return dc, L, V, cnt, torch.ones_like(wide)

    monkeypatch.setattr(codec, "encode_channel_device8", forced_wide)
    assert codec.jpeg_encode(ci).byte_stream() == fast
    monkeypatch.undo()
    if kind != "ragged":  # (partial blocks: the reference's decode asserts, codec.py:418)
        back = codec.jpeg_decode(hicimage.HicImage.from_bytes(fast))
        for a, b in zip(planes, back.as_dict.values()):
            np.testing.assert_array_equal(a, np.asarray(b))


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.int32])
def test_key_range_all_widths(dtype):
    """hic_key_range (the histograms' bin range) == numpy min / max for every key
    width, at lengths around the vectorised int32 form's 4-key loads and at an
    address that is not 16-byte aligned (the one-key form)."""
    from hiccup_amd import huffman
    rng = np.random.default_rng(5)
    info = np.iinfo(dtype)
    for n in (1, 3, 4, 5, 1023, 4096 + 3, 1_000_001):
        keys = rng.integers(max(info.min, -40000), min(info.max, 40000) + 1, n).astype(dtype)
        d = device.to_device(keys)
        assert huffman.device_key_range(d, n) == (int(keys.min()), int(keys.max())), (n, dtype)
        if n > 2:
            assert huffman.device_key_range(d[1:], n - 1) == (int(keys[1:].min()), int(keys[1:].max()))


def test_huffman_decode_batch_streams():
    """codec.jpeg_decode's batched decode (hic_huffman_decode_batch through
    codec._huffman_streams_device) == one decode_data walk per stream: native flat
    trees and node-object trees side by side, a table with a None leaf, an empty
    stream, a one-leaf tree; a missing child in one stream raises AttributeError
    only after every earlier stream decoded, and the first failure in payload order
    wins over a later one."""
    from hiccup_amd import codec, huffman
    rng = np.random.default_rng(11)
    payloads, trees, want = [], [], []
    for kind in ("values", "lengths", "none_leaf", "empty", "single", "skewed"):
        if kind == "none_leaf":
            t = huffman.HuffmanTree.construct_from_coding([(5, "1"), (6, "01")])  # "00" decodes to None
            bits = "1011" * 300 + "1"
            payloads.append(hicimage.BitStringP(bits))
            trees.append(t)
            want.append(t.decode_data(bits))
            continue
        keys = {"values": np.round(rng.laplace(0, 40, 50_001)), "lengths": rng.integers(0, 15, 70_000),
                "empty": np.array([4, 4, 9]), "single": np.full(33, 7),
                "skewed": (rng.geometric(0.35, 30_000) - 1) * 3 - 40}[kind].astype(np.int64)
        table = huffman.CodeBook(*huffman.first_appearance_counts(keys)).encode_table()
        codes = dict(table)
        bits = "" if kind == "empty" else "".join(codes[int(k)] for k in keys)
        t = huffman.FlatCodes.from_table(table) or huffman.HuffmanTree.construct_from_coding(table)
        payloads.append(hicimage.BitStringP(bits))
        trees.append(t)
        want.append([] if kind == "empty" else keys.tolist())
    assert isinstance(trees[0], huffman.FlatCodes) and isinstance(trees[4], huffman.HuffmanTree)
    got = codec._huffman_streams_device(payloads, trees)
    for (d, n), w in zip(got, want):
        assert n == len(w) and d[:n].cpu().tolist() == [x for x in w], n
    # a one-leaf encoding tree walks into its missing '0' child
    bad = huffman.HuffmanTree.construct_from_data([3, 3, 3])
    bad_bits = hicimage.BitStringP("1" * 5000 + "0" + "1" * 50)
    with pytest.raises(AttributeError):
        codec._huffman_streams_device(payloads[:2] + [bad_bits] + payloads[2:], trees[:2] + [bad] + trees[2:])
    # first failure in payload order: an out-of-int32 leaf value (ValueError) before the walk error
    big = huffman.HuffmanTree.construct_from_coding([(2 ** 40, "1"), (1, "0")])
    with pytest.raises(ValueError):
        codec._huffman_streams_device([hicimage.BitStringP("10"), bad_bits], [big, bad])


def test_huffman_decode_device_full_size():
    """An 8K-sized AC value stream (22 M symbols, Laplace keys): GPU pack then GPU
    decode returns the keys (compared on the device)."""
    from hiccup_amd import huffman
    rng = np.random.default_rng(8)
    n = 22_000_000
    keys = device.to_device(np.round(rng.laplace(0, 6, n)).clip(-2047, 2047).astype(np.int32))
    ds = huffman.DeviceStream(keys)
    packed, nbits = ds.packed()
    dec = huffman.HuffmanTree.construct_from_coding(ds.tree.encode_table())
    buf = np.zeros(-(-nbits // 32) * 4, np.uint8)
    buf[:packed.size] = packed
    out, cnt, ints = dec.decode_device(device.to_device(buf), nbits)
    assert ints and cnt == n
    assert torch.equal(out[:n], keys)


@pytest.mark.parametrize("nkeys", [8, 5, 16])
def test_huffman_decode_device_equal_length_codes(nkeys):
    """a near-uniform table gives every key the same code length L
    (3 bits for 8 keys, 4 for 16); with 1024-bit subsequences and L not dividing
    1024 the speculative starts never resynchronise and the decode fell to the serial
    one-thread chain.  Subsequences are now a multiple of L bits: 30 M coded bits
    decode to the keys, and in well under a second (5 keys: unequal lengths, the
    usual resynchronisation)."""
    import time
    from hiccup_amd import huffman
    rng = np.random.default_rng(nkeys)
    n = 10_000_000
    keys = device.to_device(rng.integers(0, nkeys, n).astype(np.int32))
    ds = huffman.DeviceStream(keys)
    packed, nbits = ds.packed()
    dec = huffman.HuffmanTree.construct_from_coding(ds.tree.encode_table())
    if nkeys in (8, 16):
        assert dec.min_code_length() == {8: 3, 16: 4}[nkeys]
    buf = np.zeros(-(-nbits // 32) * 4, np.uint8)
    buf[:packed.size] = packed
    bits = device.to_device(buf)
    dec.decode_device(bits, nbits)  # warm-up (LUT build, workspace)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, cnt, ints = dec.decode_device(bits, nbits)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert ints and cnt == n
    assert torch.equal(out[:n], keys)
    assert dt < 0.5, "%.3f s for %d bits" % (dt, nbits)


def test_wire_batches():
    """hic_wire_pack_batch / _unpack_batch (a multi-GPU group's segments in 3
    launches) == one hic_wire_pack_i16 / _unpack_i16 + hic_rle_records_rebase per
    segment, over mixed tables and sizes, a records-only job and a segment with a
    value outside its width (its flag alone raised); hic_wire_flags_apply turns a
    raised flag into HIC_COUNT_WIRE_OVERFLOW and leaves the other counts."""
    import wire_host
    rng = np.random.default_rng(3)
    spec = [(0, 1), (1, 65), (0, 777), (1, 64), (0, 4100), (1, 3)]
    jobs, want, outs, flags, backs = [], [], [], [], []
    for i, (table, nblk) in enumerate(spec):
        blocks = wire_host.random_blocks(rng, nblk, table)
        if i == 2:
            blocks[nblk // 3, 5] = 1 << (wire_host.WIDTHS[table][5] - 1)  # one past its width
        b = device.to_device(blocks)
        nb = _lib.load().hic_wire_bytes(nblk, table)
        nrec = -(-nblk // 64)
        rec = device.to_device(rng.integers(-1, 10 ** 6, (nrec, 3)).astype(np.int64))
        wire = device.empty((nb + 24 * nrec,), torch.uint8)
        flag = device.full((1,), 7, torch.int32) if hasattr(device, "full") else torch.full((1,), 7, dtype=torch.int32,
                                                                                          device="cuda")
        jobs.append(_lib.WireJob(b.data_ptr(), wire.data_ptr(), nblk, table, flag.data_ptr(), rec.data_ptr(), nrec,
                                 1000 * i, wire.data_ptr() + nb, None))
        want.append((blocks, table, rec, nb, nrec, 1000 * i))
        outs.append((b, wire, rec))
        flags.append(flag)
    # a records-only job
    rec_only = device.to_device(rng.integers(-1, 10 ** 6, (10, 3)).astype(np.int64))
    rec_dst = device.empty((10, 3), torch.int64)
    jobs.append(_lib.WireJob(None, None, 0, 0, None, rec_only.data_ptr(), 10, 5, rec_dst.data_ptr(), None))
    sharding.wire_batch("hic_wire_pack_batch", jobs)
    torch.cuda.synchronize()
    def rebased(r, shift):
        r = r.copy()
        r[:, :2] = np.where(r[:, :2] >= 0, r[:, :2] + shift, r[:, :2])
        return r
    for i, ((blocks, table, rec, nb, nrec, shift), (_, wire, _), flag) in enumerate(zip(want, outs, flags)):
        w = device.to_host(wire)
        if i != 2:  # (the host restatement refuses the out-of-width value)
            np.testing.assert_array_equal(w[:nb], wire_host.pack(blocks, table), err_msg=str(i))
        np.testing.assert_array_equal(w[nb:].view(np.int64).reshape(nrec, 3), rebased(device.to_host(rec), shift))
        assert int(flag.item()) == (1 if i == 2 else 0), i
    np.testing.assert_array_equal(device.to_host(rec_dst), rebased(device.to_host(rec_only), 5))
    # unpack: the segments back into blocks, their records rebased again
    ujobs, backs = [], []
    for (blocks, table, rec, nb, nrec, shift), (_, wire, _) in zip(want, outs):
        back = device.empty((blocks.shape[0], 64), torch.int16)
        rdst = device.empty((nrec, 3), torch.int64)
        ujobs.append(_lib.WireJob(back.data_ptr(), wire.data_ptr(), blocks.shape[0], table, None,
                                  wire.data_ptr() + nb, nrec, 1, rdst.data_ptr(), None))
        backs.append((back, rdst))
    sharding.wire_batch("hic_wire_unpack_batch", ujobs)
    for i, ((blocks, table, rec, nb, nrec, shift), (back, rdst)) in enumerate(zip(want, backs)):
        if i != 2:
            np.testing.assert_array_equal(device.to_host(back), blocks, err_msg=str(i))
        np.testing.assert_array_equal(device.to_host(rdst), rebased(rebased(device.to_host(rec), shift), 1))
    counts = torch.tensor([11, 22, 33], dtype=torch.int64, device="cuda")
    fj = [_lib.WireJob(None, None, 0, 0, flags[i].data_ptr(), None, 0, 0, None, counts.data_ptr() + 8 * c)
          for c, i in ((0, 0), (1, 2), (2, 1))]
    sharding.wire_batch("hic_wire_flags_apply", fj)
    assert counts.cpu().tolist() == [11, pipeline.COUNT_WIRE_OVERFLOW, 33]


@pytest.mark.parametrize("table", [0, 1])
@pytest.mark.parametrize("nblk", [1, 63, 64, 65, 777, 129600])
def test_wire_pack_unpack(nblk, table):
    """The gather's wire format: hic_wire_pack_i16 == the host restatement
    (tests/wire_host.py, which the CPU gloo test of the stream gather uses) for
    every slot anywhere in its proven width, unpack inverts it, a value one past a
    slot's width raises the flag, and hic_rle_records_rebase shifts record
    positions (-1 kept).  A real 8K encode's blocks pack losslessly too."""
    import wire_host
    rng = np.random.default_rng(nblk + table)
    blocks = wire_host.random_blocks(rng, nblk, table)
    lib = _lib.load()
    nb = lib.hic_wire_bytes(nblk, table)
    assert nb == wire_host.wire_bytes(nblk, table)
    b = device.to_device(blocks)
    wire = device.empty((nb,), torch.uint8)
    flag = device.zeros((1,), torch.int32)
    _lib.call("hic_wire_pack_i16", device.ptr(b), nblk, table, device.ptr(wire), device.ptr(flag),
              device.stream_ptr())
    got = device.to_host(wire)
    np.testing.assert_array_equal(got, wire_host.pack(blocks, table))
    assert int(flag.item()) == 0
    back = device.empty((nblk, 64), torch.int16)
    _lib.call("hic_wire_unpack_i16", device.ptr(wire), nblk, table, device.ptr(back), device.stream_ptr())
    np.testing.assert_array_equal(device.to_host(back), blocks)
    bad = blocks.copy()
    j = int(rng.integers(0, 64))
    bad[nblk // 2, j] = 1 << (wire_host.WIDTHS[table][j] - 1)
    _lib.call("hic_wire_pack_i16", device.ptr(device.to_device(bad)), nblk, table, device.ptr(wire),
              device.ptr(flag), device.stream_ptr())
    assert int(flag.item()) == 1
    rec = rng.integers(-1, 10 ** 6, (nblk, 3)).astype(np.int64)
    out = device.empty((nblk, 3), torch.int64)
    _lib.call("hic_rle_records_rebase", device.ptr(device.to_device(rec)), nblk, 1234567, device.ptr(out),
              device.stream_ptr())
    exp = rec.copy()
    exp[:, :2] = np.where(rec[:, :2] >= 0, rec[:, :2] + 1234567, rec[:, :2])
    np.testing.assert_array_equal(device.to_host(out), exp)
    if nblk == 129600:  # the extreme-value images of the structured kinds, through a real encode
        for kind in ("random", "colour_levels", "blocks"):
            enc = pipeline.Encoder(4320 // 4, 7680 // 2)
            enc.encode(device.to_device(_structured_rgb(kind, 4320 // 4, 7680 // 2, 3)))
            k = "lum" if table == 0 else "cr"
            coef = enc.coef[k]
            w2 = device.empty((lib.hic_wire_bytes(coef.shape[0], table),), torch.uint8)
            flag.zero_()
            _lib.call("hic_wire_pack_i16", device.ptr(coef), coef.shape[0], table, device.ptr(w2),
                      device.ptr(flag), device.stream_ptr())
            back2 = device.empty(tuple(coef.shape), torch.int16)
            _lib.call("hic_wire_unpack_i16", device.ptr(w2), coef.shape[0], table, device.ptr(back2),
                      device.stream_ptr())
            assert int(flag.item()) == 0 and torch.equal(back2, coef), kind


def test_huffman_device_streams_batch_equals_single():
    """huffman.DeviceStreams (the batched form codec.jpeg_encode and
    Encoder.hic_image use) == one DeviceStream per stream: trees and packed bits,
    over streams of mixed key widths, lengths and alphabets."""
    from hiccup_amd import huffman
    rng = np.random.default_rng(11)
    raw = [rng.integers(0, 15, 70_001).astype(np.uint8), np.round(rng.laplace(0, 30, 123_457)).astype(np.int16),
           rng.integers(-2000, 2001, 9_999).astype(np.int32), np.full(17, 5, np.int16),
           ((rng.geometric(0.4, 50_000) - 1) * 2).astype(np.int32), rng.integers(0, 2, 3).astype(np.uint8)]
    devs = [device.to_device(k) for k in raw]
    # a stream given as a prefix of a longer buffer (the symbol buffers' form)
    devs.append(device.to_device(np.concatenate([raw[1], raw[1][:100]])))
    lens = [k.size for k in raw] + [raw[1].size]
    ds = huffman.DeviceStreams(list(zip(devs, lens)))
    packs = ds.packed()
    for i, (d, n) in enumerate(zip(devs, lens)):
        one = huffman.DeviceStream(d, n)
        assert ds.trees[i].encode_table() == one.tree.encode_table(), i
        p1, b1 = one.packed()
        assert packs[i][1] == b1 and np.array_equal(packs[i][0], p1), i


def test_encoder_hic_image_equals_jpeg_encode():
    """pipeline.Encoder.hic_image (GPU streams + GPU Huffman) == codec.jpeg_encode of
    the same quantized planes (the reference's encode path on its own output)."""
    H, W = 272, 1024
    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rgb[:, :300] = 90
    enc = pipeline.Encoder(H, W)
    enc.encode(device.to_device(rgb))
    hic = enc.hic_image()
    res = enc.result()
    planes = {}
    for k, (h, w) in enc.shapes.items():
        zz = res[k][0].astype(np.int32)
        planes[k] = orc.merge_blocks(zz[:, np.argsort(orc.ZZ8)].reshape(-1, 8, 8), (h, w))
    ref = codec.jpeg_encode(model.CompressedImage(planes["lum"], planes["cr"], planes["cb"]))
    assert len(hic.payloads) == len(ref.payloads) == 20
    for i, (a, b) in enumerate(zip(hic.payloads, ref.payloads)):
        assert a == b, i
    assert hic.byte_stream() == ref.byte_stream()


def test_encoder_hic_image_on_side_stream():
    """The whole encode + hic_image on a non-current stream: the histograms, key
    ranges, code tables and packed bits are read after that stream's kernels, and
    the temporaries live on it.  A large image gives the reads a chance
    to overtake an unsynchronised stream.  == the same on the current stream."""
    H, W = 2160, 3840
    rng = np.random.default_rng(31)
    rgb = device.to_device(rng.integers(0, 256, (H, W, 3), dtype=np.uint8))
    ref_enc = pipeline.Encoder(H, W)
    ref_enc.encode(rgb)
    ref = ref_enc.hic_image()
    side = torch.cuda.Stream()
    enc = pipeline.Encoder(H, W)
    torch.cuda.synchronize()  # the encoder's zero-filled workspaces were written on the current stream
    enc.encode(rgb, stream=side)
    got = enc.hic_image(stream=side)
    assert got.byte_stream() == ref.byte_stream()
