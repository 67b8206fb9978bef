"""GPU parity: forward / inverse 8x8 DCT kernels vs the reference's outputs.

Small cases are compared with the golden fixtures the reference itself produced
(tests/golden/make_golden.py); full 4K / 8K planes are compared bit-exactly with
the C oracle (oracle/hiccup_oracle.c, pinned against the same fixtures).
"""
import zlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import oracle.oracle as orc  # noqa: E402
import oracle.oracle_c as orcc  # noqa: E402
from hiccup_amd import _lib, device, model, quantization, transform  # noqa: E402

QT = {0: model.QTables.JPEG_LUMINANCE, 1: model.QTables.JPEG_CHROMINANCE}


def _names(d, prefix):
    return sorted(k[len(prefix):] for k in d if k.startswith(prefix))


def test_dct_channel_golden(golden_transform):
    g = golden_transform
    for name in _names(g, "in_"):
        tab = int(g["tab_" + name])
        q = transform.dct_channel(g["in_" + name], QT[tab])
        assert q.dtype == np.int32
        np.testing.assert_array_equal(q, g["q_" + name], err_msg=name)


def test_inv_dct_channel_golden(golden_transform):
    g = golden_transform
    for name in _names(g, "in_"):
        tab = int(g["tab_" + name])
        rec = transform.inv_dct_channel(g["q_" + name], QT[tab])
        assert rec.dtype == np.uint8
        np.testing.assert_array_equal(rec, g["rec_" + name], err_msg=name)
    for name in _names(g, "icin_"):
        tab = int(g["ictab_" + name])
        np.testing.assert_array_equal(transform.inv_dct_channel(g["icin_" + name], QT[tab]),
                                      g["icout_" + name], err_msg=name)


def test_inv_dct_float_planes(golden_transform):
    """jpeg_decode hands float64 (integer-valued) planes to inv_dct_channel."""
    g = golden_transform
    q = g["q_r256_lum"].astype(np.float64)
    np.testing.assert_array_equal(transform.inv_dct_channel(q, QT[0]), g["rec_r256_lum"])


def test_dct2_idct2_bits(golden_transform):
    g = golden_transform
    out = transform.dct2(g["dct2_in"])
    assert np.array_equal(out.view(np.int64), g["dct2_out"].view(np.int64))
    back = transform.idct2(g["dct2_out"])
    assert np.array_equal(back.view(np.int64), g["idct2_out"].view(np.int64))


def test_quantize_helpers(golden_transform):
    # quantizationtest.py:12-25
    mat = np.ones((8, 8))
    mat[0, 0] = 16
    q = quantization.jpeg_quantize(mat, model.QTables.JPEG_LUMINANCE)
    assert q[0][0] == 1 and np.sum(q) == 1
    g = golden_transform
    b = g["dct2_out"]
    for tab in (0, 1):
        exp = np.round(b / orc.TABLES[tab]).astype(np.int32)
        np.testing.assert_array_equal(quantization.jpeg_quantize(b, QT[tab]), exp)
        np.testing.assert_array_equal(quantization.invert_jpeg_quantize(exp, QT[tab]), exp * orc.TABLES[tab])


def test_constant_images():
    # transformtest.py:148-161
    assert np.sum(transform.dct_channel(np.full((120, 80), 128, np.uint8), model.QTables.JPEG_CHROMINANCE)) == 0
    assert np.abs(np.sum(transform.dct_channel(np.ones((120, 80), np.uint8), model.QTables.JPEG_LUMINANCE))) > 0
    assert np.sum(transform.dct_channel(np.zeros((120, 80), np.uint8), model.QTables.JPEG_LUMINANCE)) < 1e-10


@pytest.mark.parametrize("layout", [_lib.LAYOUT_RASTER_I32, _lib.LAYOUT_RASTER_I16, _lib.LAYOUT_ZIGZAG_I16])
@pytest.mark.parametrize("shape", [(64, 64), (37, 53), (8, 200), (130, 7)])
def test_layouts_roundtrip(layout, shape):
    rng = np.random.default_rng(sum(shape) + layout)
    plane = rng.integers(0, 256, shape, dtype=np.uint8)
    for tab in (0, 1):
        exp = orcc.dct_channel(plane, tab)
        coef = transform.dct_channel_device(device.to_device(plane), tab, layout)
        got = device.to_host(coef)
        if layout == _lib.LAYOUT_ZIGZAG_I16:
            np.testing.assert_array_equal(got.astype(np.int32), orcc.zigzag_blocks(exp, 8))
        else:
            np.testing.assert_array_equal(got.astype(np.int32), exp)
        rec = transform.inv_dct_channel_device(coef, shape[0], shape[1], tab, layout)
        np.testing.assert_array_equal(device.to_host(rec), orcc.inv_dct_channel(exp, tab))


@pytest.mark.parametrize("path", [-1, _lib.DCT_PATH_EXACT])
@pytest.mark.parametrize("H,W", [(4096, 4096), (4320, 7680)])
def test_full_size_bit_exact(H, W, path):
    """BASELINE configs 2/3 plane sizes, bit-exact against the C oracle (multi-threaded),
    on the default forward path (float64 AAN) and the exact pocketfft replica."""
    with _lib.knobs(dct_path=path):
        _full_size_bit_exact(H, W)


def _full_size_bit_exact(H, W):
    rng = np.random.default_rng(2)
    plane = rng.integers(0, 256, (H, W), dtype=np.uint8)
    exp = orcc.dct_channel(plane, 0, threads=16)
    coef = transform.dct_channel_device(device.to_device(plane), 0, _lib.LAYOUT_ZIGZAG_I16)
    zz = device.to_host(coef)
    raster = orc.merge_blocks(zz[:, np.argsort(orc.ZZ8)].reshape(-1, 8, 8), (H, W))
    np.testing.assert_array_equal(raster.astype(np.int32), exp)
    # inverse: a size-independent property -- dequant+IDCT of the GPU coefficients
    rec = device.to_host(transform.inv_dct_channel_device(coef, H, W, 0, _lib.LAYOUT_ZIGZAG_I16))
    np.testing.assert_array_equal(rec[:1024], orcc.inv_dct_channel(exp[:1024], 0))
    # reconstruction quality is what a JPEG-style lum table gives on noise
    assert np.mean(np.abs(rec.astype(np.int32) - plane.astype(np.int32))) < 40


def test_tie_blocks_many():
    """Exact .5 quotients at DC / (4,4) on 100k random blocks (25% / ~3% of blocks)."""
    rng = np.random.default_rng(11)
    plane = rng.integers(0, 256, (8 * 250, 8 * 400), dtype=np.uint8)
    for tab in (0, 1):
        np.testing.assert_array_equal(transform.dct_channel(plane, QT[tab]), orcc.dct_channel(plane, tab, threads=8))


@pytest.mark.parametrize("path", [_lib.DCT_PATH_F64, _lib.DCT_PATH_EXACT])
@pytest.mark.parametrize("kind", ["levels4", "nearflat", "stripes", "checker", "blur"])
def test_fast_path_structured_ties(kind, path):
    with _lib.knobs(dct_path=path):
        _structured_ties(kind)


def _structured_plane(kind, H, W):
    rng = np.random.default_rng(zlib.crc32(kind.encode()))
    if kind == "random":
        return rng.integers(0, 256, (H, W), dtype=np.uint8)
    if kind == "levels4":
        return (rng.integers(0, 4, (H, W)) * 85).astype(np.uint8)
    if kind == "nearflat":
        return (128 + rng.integers(-4, 5, (H, W))).astype(np.uint8)
    if kind == "stripes":
        plane = np.where((np.arange(W) // rng.integers(1, 4)) % 2 == 0, 255, 0).astype(np.uint8)[None].repeat(H, 0)
        plane[rng.random((H, W)) < 0.01] = 128
        return plane
    if kind == "checker":
        plane = (((np.arange(H)[:, None] + np.arange(W)[None]) % 2) * 255).astype(np.uint8)
        plane ^= rng.integers(0, 2, (H, W), dtype=np.uint8)
        return plane
    # else ("blur"): chroma-like: pyrDown of noise, many coefficients near +-1/2
    return orcc.pyr_down(rng.integers(0, 256, (2 * H, 2 * W), dtype=np.uint8))


def _structured_ties(kind):
    """Planes that drive the AAN fast paths into their tie handling: 4-level and
    near-flat pixels give exact (2,2)-class and (4,4) ties and the rare whole-set
    redo; stripes / checkerboards give large saturated coefficients.  Every
    layout and both tables, fused RLE-tile variant included, vs the C oracle."""
    H, W = 8 * 160, 8 * 320
    plane = _structured_plane(kind, H, W)
    d = device.to_device(plane)
    for tab in (0, 1):
        exp = orcc.dct_channel(plane, tab, threads=8)
        for layout in (_lib.LAYOUT_RASTER_I32, _lib.LAYOUT_RASTER_I16, _lib.LAYOUT_ZIGZAG_I16):
            got = device.to_host(transform.dct_channel_device(d, tab, layout))
            if layout == _lib.LAYOUT_ZIGZAG_I16:
                got = orc.merge_blocks(got[:, np.argsort(orc.ZZ8)].reshape(-1, 8, 8), (H, W))
            np.testing.assert_array_equal(got.astype(np.int32), exp, err_msg=(kind, tab, layout))
        # the fused variant (DCT + RLE tile records) writes the same coefficients
        nblk = (H // 8) * (W // 8)
        out = device.empty((nblk, 64), torch.int16)
        ws = device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64))
        _lib.call("hic_dct_quant_rle_u8", device.ptr(d), H, W, W, tab, 15, device.ptr(out), device.ptr(ws),
                  device.stream_ptr(), None, None)
        got = orc.merge_blocks(device.to_host(out)[:, np.argsort(orc.ZZ8)].reshape(-1, 8, 8), (H, W))
        np.testing.assert_array_equal(got.astype(np.int32), exp, err_msg=(kind, tab, "fused"))


def test_bad_args():
    with pytest.raises(ValueError):
        transform.dct_channel(np.zeros((8, 8), np.uint8), model.QTables.JPEG_LUMINANCE, block_size=4)
    with pytest.raises(ValueError):
        transform.dct_channel(np.zeros((8, 8, 3), np.uint8), model.QTables.JPEG_LUMINANCE)
    dev = device.to_device(np.zeros((8, 8), np.uint8))
    out = device.empty((8, 8), torch.int32)
    with pytest.raises(ValueError):
        _lib.call("hic_dct_quant_u8", device.ptr(dev), 8, 8, 8, 7, 0, device.ptr(out), device.stream_ptr())
    with pytest.raises(ValueError):
        _lib.call("hic_dct_quant_u8", device.ptr(dev), 8, 8, 8, 0, 9, device.ptr(out), device.stream_ptr())


@pytest.mark.parametrize("path", [_lib.DCT_PATH_F64, _lib.DCT_PATH_EXACT])
@pytest.mark.parametrize("kind", ["random", "levels4", "nearflat", "blur", "checker"])
@pytest.mark.parametrize("H,W", [(8, 16), (8 * 61, 16 * 7), (8 * 33, 8 * 130), (8 * 160, 8 * 320)])
def test_plane_dct_rle_records(kind, path, H, W):
    """The plane DCT's fused RLE tile records (k_dct_planes, partial
    last sets included) drive the channel RLE: symbols and DC
    differences of hic_dct_quant_rle_u8 + hic_rle_encode_i16_tiles_batch equal the
    C oracle's run_length_coding / differential_coding (codec.py:47-99)."""
    plane = _structured_plane(kind, H, W)
    d = device.to_device(plane)
    nblk = (H // 8) * (W // 8)
    lib = _lib.load()
    for tab in (0, 1):
        exp = orcc.zigzag_blocks(orcc.dct_channel(plane, tab), 8)
        eL, eV = orcc.rle_encode(exp[:, 1:].reshape(-1), 15)
        out = device.empty((nblk, 64), torch.int16)
        ws = device.workspace(lib.hic_rle_workspace_bytes(nblk, 64))
        with _lib.knobs(dct_path=path):
            _lib.call("hic_dct_quant_rle_u8", device.ptr(d), H, W, W, tab, 15, device.ptr(out), device.ptr(ws),
                      device.stream_ptr(), None, None)
        cap = nblk * 63 + 1
        L, V = device.empty((cap,), torch.uint8), device.empty((cap,), torch.int16)
        dc, cnt = device.empty((nblk,), torch.int32), device.zeros((1,), torch.int64)
        job = (_lib.RleJob16 * 1)()
        job[0] = _lib.RleJob16(out.data_ptr(), nblk, None, dc.data_ptr(), L.data_ptr(), V.data_ptr(), cap,
                               cnt.data_ptr(), ws.data_ptr(), 1)
        _lib.call("hic_rle_encode_i16_tiles_batch", 1, job, 15, device.stream_ptr())
        np.testing.assert_array_equal(device.to_host(out).astype(np.int32), exp, err_msg=(kind, tab))
        c = int(cnt.cpu().item())
        assert c == len(eL), (kind, tab, c, len(eL))
        np.testing.assert_array_equal(device.to_host(L[:c]).astype(np.int32), eL, err_msg=(kind, tab))
        np.testing.assert_array_equal(device.to_host(V[:c]).astype(np.int32), eV, err_msg=(kind, tab))
        np.testing.assert_array_equal(device.to_host(dc), orcc.dpcm(exp[:, 0].copy()), err_msg=(kind, tab))


@pytest.mark.parametrize("path", [_lib.DCT_PATH_F64, _lib.DCT_PATH_EXACT])
@pytest.mark.parametrize("waves_per_cu", [-1, 1])
@pytest.mark.parametrize("kind", ["random", "levels4"])
def test_plane_batch_three_planes(kind, waves_per_cu, path):
    """hic_dct_quant_rle_u8_batch over BASELINE configs[2]'s three planes (8K Y +
    two 4K chroma) in one launch: with few persistent waves each wave walks sets of
    different planes and tables, and (float64 path) keeps several flagged sets for
    its pass after the loop.  Coefficients,
    DC differences and symbols vs the C oracle."""
    _plane_batch([(4320, 7680, 0), (2160, 3840, 1), (2160, 3840, 1)], kind, waves_per_cu, path)


@pytest.mark.parametrize("table", [0, 1])
@pytest.mark.parametrize("kind", ["random", "levels4"])
def test_plane_batch_one_table_records(kind, table):
    """A batch whose planes share one table runs the kernel compiled for that table
    (literal quantiser constants), RLE tile records included: coefficients, DC
    differences and symbols vs the C oracle."""
    _plane_batch([(8 * 45, 8 * 96, table), (8 * 30 + 8, 8 * 64 + 24, table), (8 * 52, 8 * 70, table)], kind, -1, -1)


@pytest.mark.parametrize("kind", ["random", "nearflat"])
def test_plane_batch_sixteen_planes(kind):
    """The batched launch at its maximum: 16 planes of mixed tables and sizes (incl.
    a partial last set) in ONE launch of the default kernel, as the back-to-back
    measurement runs it."""
    shapes = [(8 * 40 + 8 * (i % 3), 8 * 64 + 24 * i, i % 2) for i in range(16)]
    _plane_batch(shapes, kind, -1, -1)


@pytest.mark.parametrize("path", [_lib.DCT_PATH_F64, _lib.DCT_PATH_EXACT])
@pytest.mark.parametrize("waves_per_cu", [-1, 1])
@pytest.mark.parametrize("kind", ["random", "levels4", "nearflat", "blur"])
def test_plane_batch_records_free(kind, waves_per_cu, path):
    """The records-free batched pass (no RLE workspaces: north_star's DCT + quantize
    + zig-zag, what the back-to-back measurement runs): 8K Y + two 4K chroma planes,
    then 16 small planes of mixed tables whose block rows hold < 32, 32..63 and >= 64
    blocks with partial last sets; with one persistent wave per CU each wave walks
    many sets of different planes and keeps its tie sets for after the loop."""
    shapes = [(4320, 7680, 0), (2160, 3840, 1), (2160, 3840, 1)]
    small = [(8 * (5 + 3 * i), 8 * (7 + 9 * i), i % 2) for i in range(16)]
    # one table for every plane: the launch takes the kernel compiled for that table
    luma = [(8 * (40 + i), 8 * (64 + 5 * i), 0) for i in range(4)]
    chroma = [(8 * (33 + 2 * i), 8 * (70 + 3 * i), 1) for i in range(3)]
    # every plane's rows hold whole 64-block sets
    aligned = [(4320, 7680, 0), (4320, 7680, 0), (8 * 21, 1536, 1)] + \
        [(8 * (3 + i), 1024, i % 2) for i in range(5)]
    for sh in (shapes, small, luma, chroma, aligned):
        planes, outs, jobs = [], [], (_lib.DctPlaneJob * len(sh))()
        for i, (h, w, t) in enumerate(sh):
            p = _structured_plane(kind, h, w)
            planes.append((p, device.to_device(p)))
            outs.append(device.empty(((h // 8) * (w // 8), 64), torch.int16))
            jobs[i] = _lib.DctPlaneJob(planes[i][1].data_ptr(), h, w, w, t, outs[i].data_ptr(), None)
        with _lib.knobs(dct_waves_per_cu=waves_per_cu, dct_path=path):
            _lib.call("hic_dct_quant_rle_u8_batch", len(sh), jobs, 15, device.stream_ptr(), None, None)
        for i, (h, w, t) in enumerate(sh):
            exp = orcc.zigzag_blocks(orcc.dct_channel(planes[i][0], t, threads=16), 8)
            np.testing.assert_array_equal(device.to_host(outs[i]).astype(np.int32), exp, err_msg=(kind, i, h, w))


def _plane_batch(shapes, kind, waves_per_cu, path):
    lib = _lib.load()
    planes, outs, wss = [], [], []
    n = len(shapes)
    jobs = (_lib.DctPlaneJob * n)()
    for i, (h, w, t) in enumerate(shapes):
        p = _structured_plane(kind, h, w) if i == 0 else np.ascontiguousarray(_structured_plane(kind, h, w)[::-1])
        nblk = (h // 8) * (w // 8)
        planes.append((p, device.to_device(p)))
        outs.append(device.empty((nblk, 64), torch.int16))
        wss.append(device.workspace(lib.hic_rle_workspace_bytes(nblk, 64)))
        jobs[i] = _lib.DctPlaneJob(planes[i][1].data_ptr(), h, w, w, t, outs[i].data_ptr(), wss[i].data_ptr())
    with _lib.knobs(dct_waves_per_cu=waves_per_cu, dct_path=path):
        _lib.call("hic_dct_quant_rle_u8_batch", n, jobs, 15, device.stream_ptr(), None, None)
    for i, (h, w, t) in enumerate(shapes):
        nblk = (h // 8) * (w // 8)
        exp = orcc.zigzag_blocks(orcc.dct_channel(planes[i][0], t, threads=16), 8)
        np.testing.assert_array_equal(device.to_host(outs[i]).astype(np.int32), exp, err_msg=(kind, i))
        cap = nblk * 63 + 1
        L, V = device.empty((cap,), torch.uint8), device.empty((cap,), torch.int16)
        dc, cnt = device.empty((nblk,), torch.int32), device.zeros((1,), torch.int64)
        job = (_lib.RleJob16 * 1)()
        job[0] = _lib.RleJob16(outs[i].data_ptr(), nblk, None, dc.data_ptr(), L.data_ptr(), V.data_ptr(), cap,
                               cnt.data_ptr(), wss[i].data_ptr(), 1)
        _lib.call("hic_rle_encode_i16_tiles_batch", 1, job, 15, device.stream_ptr())
        eL, eV = orcc.rle_encode(exp[:, 1:].reshape(-1), 15)
        c = int(cnt.cpu().item())
        assert c == len(eL), (kind, i, c, len(eL))
        np.testing.assert_array_equal(device.to_host(L[:c]).astype(np.int32), eL, err_msg=(kind, i))
        np.testing.assert_array_equal(device.to_host(V[:c]).astype(np.int32), eV, err_msg=(kind, i))
        np.testing.assert_array_equal(device.to_host(dc), orcc.dpcm(exp[:, 0].copy()), err_msg=(kind, i))


def test_measurement_probes():
    """bench.py's in-run floors: hic_probe_copy copies; hic_probe_plane writes each 8x8
    block's 64 pixel bytes then the same rows with their halves swapped (128 B per
    block, block order) -- it moves the plane pass's bytes, including a partial set."""
    lib_src = np.random.default_rng(5).integers(0, 256, 1 << 16, dtype=np.uint8)
    a, b = device.to_device(lib_src), device.empty((1 << 16,), torch.uint8)
    _lib.call("hic_probe_copy", device.ptr(a), device.ptr(b), 1 << 16, 0, device.stream_ptr(), None, None)
    np.testing.assert_array_equal(device.to_host(b), lib_src)
    H, W = 8 * 9, 8 * 15  # 135 blocks: two full sets and a partial one
    plane = np.random.default_rng(6).integers(0, 256, (H, W), dtype=np.uint8)
    out = device.empty((135, 64), torch.int16)
    _lib.call("hic_probe_plane", device.ptr(device.to_device(plane)), H, W, device.ptr(out), 0, device.stream_ptr(),
              None, None)
    got = device.to_host(out).view(np.uint8).reshape(135, 128)
    blocks = plane.reshape(9, 8, 15, 8).swapaxes(1, 2).reshape(135, 8, 8)
    np.testing.assert_array_equal(got[:, :64], blocks.reshape(135, 64))
    swapped = blocks.reshape(135, 8, 2, 4)[:, :, ::-1, :].reshape(135, 64)
    np.testing.assert_array_equal(got[:, 64:], swapped)
    with pytest.raises(ValueError):
        _lib.call("hic_probe_copy", device.ptr(a), device.ptr(b), 17, 0, device.stream_ptr(), None, None)
    # hic_probe_encode420 (the fused encoder's byte pattern): every unit writes all
    # its coefficient slots and its three records (record word 2 = the pass: 0 / 1
    # for the unit's two Y block rows, 2 for its chroma), in every unit order
    H, W = 80, 1024
    rgb = device.to_device(np.random.default_rng(7).integers(0, 256, (H, W, 3), dtype=np.uint8))
    for order in (0, 6):
        co = [device.zeros(((H // 8) * (W // 8), 64), torch.int16)] + \
             [device.zeros(((H // 16) * (W // 16), 64), torch.int16) for _ in range(2)]
        for t in co:
            t.fill_(0x5A5A)
        ry = device.zeros(((H // 8) * (W // 512) * 3,), torch.int64)
        rc = device.zeros(((H // 16) * (W // 512) * 3,), torch.int64)
        ry.fill_(-7)
        rc.fill_(-7)
        with _lib.knobs(encode_order=order):
            _lib.call("hic_probe_encode420", device.ptr(rgb), H, W, *[device.ptr(t) for t in co], device.ptr(ry),
                      device.ptr(rc), device.stream_ptr(), None, None)
        for t in co:
            assert int((device.to_host(t) == 0x5A5A).sum()) < 16, order  # (a folded word may equal it by chance)
        np.testing.assert_array_equal(device.to_host(ry).reshape(-1, 3)[:, 2],
                                      np.repeat(np.arange(H // 8) % 2, W // 512), err_msg=str(order))
        assert (device.to_host(rc).reshape(-1, 3)[:, 2] == 2).all(), order
    with pytest.raises(ValueError):
        _lib.call("hic_probe_encode420", device.ptr(rgb), H, 1000, *[device.ptr(t) for t in co], device.ptr(ry),
                  device.ptr(rc), device.stream_ptr(), None, None)


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.int32, np.float32, np.float64, np.bool_])
def test_pinned_host_copies(dtype):
    """device.to_device / to_host above the pinned-staging threshold (4 MiB) return
    new arrays equal to the input for every dtype the API moves, in both directions,
    back to back (the staging buffer is reused and grown), and to_host_f64 /
    to_device_i32 keep the host checks' results and errors."""
    rng = np.random.default_rng(11)
    for shape in [(1500, 1000, 3), (2049, 1031)]:
        a = (rng.integers(0, 2, shape) if dtype == np.bool_ else rng.integers(-100, 100, shape)).astype(dtype)
        t = device.to_device(a)
        assert t.shape == a.shape and t.is_cuda
        b = device.to_host(t)
        assert b.dtype == a.dtype and b.shape == a.shape
        np.testing.assert_array_equal(b, a)
        t.add_(1) if dtype != np.bool_ else t.logical_not_()
        np.testing.assert_array_equal(b, a)  # a copy, not a view of the staging buffer
    p = rng.integers(-5000, 5000, (2048, 1024)).astype(np.int32)
    f = device.to_host_f64(device.to_device(p))
    assert f.dtype == np.float64
    np.testing.assert_array_equal(f, p)
    g = device.to_device_i32(p.astype(np.float64), "bad", "range")
    assert g.dtype == torch.int32
    np.testing.assert_array_equal(device.to_host(g), p)
    q = p.astype(np.float64)
    q[7, 9] = 0.5
    with pytest.raises(ValueError, match="bad"):
        device.to_device_i32(q, "bad", "range")
    q[7, 9] = 2.0 ** 31
    with pytest.raises(ValueError, match="range"):
        device.to_device_i32(q, "bad", "range")
    q[7, 9] = np.nan
    with pytest.raises(ValueError, match="bad"):
        device.to_device_i32(q, "bad", "range")


@pytest.mark.parametrize("dtype", [np.uint8, np.int32, np.float64, np.bool_])
def test_pinned_host_copies_chunked(dtype, monkeypatch):
    """Copies larger than a staging buffer go in _CHUNK pieces through the two pinned
    buffers, each chunk's host copy beside the next chunk's DMA (the chunk lowered to
    4 MiB + 8 here so that a ~13 MB copy takes four, the last one short)."""
    monkeypatch.setattr(device, "_CHUNK", (4 << 20) + 8)
    monkeypatch.setattr(device, "_staging", [None, None])
    rng = np.random.default_rng(12)
    a = (rng.integers(0, 2, (1601, 2051)) if dtype == np.bool_ else rng.integers(-100, 100, (1601, 2051))).astype(dtype)
    if a.nbytes < 3 * device._CHUNK:
        a = np.concatenate([a] * (1 + 3 * device._CHUNK // a.nbytes))
    t = device.to_device(a)
    np.testing.assert_array_equal(device.to_host(t), a)
    assert all(b is None or b.numel() <= device._CHUNK for b in device._staging)
    if dtype == np.int32:
        np.testing.assert_array_equal(device.to_host_f64(t), a.astype(np.float64))
