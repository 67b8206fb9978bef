"""The slot-layout encode (round 6, hiccup_amd/csrc/slots.h): the fused kernel
writes every RLE record's symbols and DC differences itself, one scan launch
closes the carried runs.  Its stream -- materialized contiguously -- and the
zig-zag blocks decoded from it equal the coefficient chain's (the fused kernel's
coefficients + scan + emit, itself pinned to the C oracle and the reference's
fixtures in test_gpu_codec.py), bit for bit, on images that stress each part of
the emission: dense random blocks, exact-tie levels, long zero runs inside blocks
(fillers in the slot), runs carried over many records (fillers before a slot),
an all-zero image (the stream is one EOB), and luminance blocks whose zig-zag
slot 3 needs 13 bits (the kernel's direct-store path).  Reference:
codec.run_length_coding / differential_coding (codec.py:47-99,286-301)."""
import numpy as np
import pytest
import torch

from hiccup_amd import device, pipeline

pytestmark = pytest.mark.gpu


def _img(kind, H, W, seed):
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    if kind == "levels":  # 4 grey levels: exact quantiser ties
        return (rng.integers(0, 4, (H, W, 1)) * 85).astype(np.uint8).repeat(3, 2)
    if kind == "colour_levels":
        return (rng.integers(0, 2, (H, W, 3)) * 255).astype(np.uint8)
    if kind == "smooth":  # natural-image-like: few nonzero AC, long runs inside blocks
        y, x = np.mgrid[0:H, 0:W]
        base = 128 + 60 * np.sin(x / 37.0) * np.cos(y / 23.0) + rng.normal(0, 3, (H, W))
        return np.clip(np.stack([base, base * 0.9 + 10, 255 - base], -1), 0, 255).astype(np.uint8)
    if kind == "sparse":  # flat but for scattered pixels: zero runs carried across many records
        img = np.full((H, W, 3), 128, np.uint8)
        n = max(1, H * W // 20000)
        img[rng.integers(0, H, n), rng.integers(0, W, n)] = rng.integers(0, 256, (n, 3), dtype=np.uint8)
        return img
    if kind == "zero":  # every AC coefficient zero: the stream is the single EOB
        return np.full((H, W, 3), 128, np.uint8)
    if kind == "wide":  # grey rows [255 255 0 0 0 0 255 255]: raster (0, 2) = zig-zag slot 3 ~ +-2130
        row = np.array([255, 255, 0, 0, 0, 0, 255, 255], np.uint8)
        img = np.tile(row, W // 8)[None, :].repeat(H, 0)
        img = np.where(rng.integers(0, 2, (H // 8, W // 8)).repeat(8, 0).repeat(8, 1) == 1, img, 255 - img)
        img[: H // 2, : W // 2] = rng.integers(0, 256, (H // 2, W // 2))  # beside ordinary blocks
        return img[..., None].repeat(3, 2).astype(np.uint8)
    raise ValueError(kind)


KINDS = ["random", "levels", "colour_levels", "smooth", "sparse", "zero", "wide"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("H,W", [(16, 512), (48, 1024), (272, 1536), (1088, 2048)])
def test_slots_equal_coefficient_chain(kind, H, W):
    """Slot layout == the coefficient chain: counts, contiguous symbols, DC
    differences and the blocks decoded from the slots; the decoders reading the
    slots (RGB, planes, blocks) == the chain's indexed decoders."""
    rgb = device.to_device(_img(kind, H, W, H + W))
    got = pipeline.Encoder(H, W, index=True)
    exp = pipeline.Encoder(H, W, index=True, slots=False)
    assert got.slots and not exp.slots
    got.encode(rgb)
    exp.encode(rgb)
    a, b = got.result(), exp.result()
    assert got.counts.cpu().tolist() == exp.counts.cpu().tolist()
    for k in pipeline.CHANNELS:
        for j, what in enumerate(("coef", "dc", "sym_len", "sym_val")):
            np.testing.assert_array_equal(a[k][j], b[k][j], err_msg="%s %s" % (k, what))
    if kind == "zero":
        for k in pipeline.CHANNELS:
            assert a[k][2].tolist() == [0] and a[k][3].tolist() == [0], k
    if kind == "wide":  # the direct-store path was taken: slot 3 outside 12 bits
        assert np.abs(a["lum"][0][:, 3].astype(np.int32)).max() > 2047
    want = [got.coef[k].shape[0] * 63 for k in pipeline.CHANNELS]
    for planes, keep in ((False, False), (True, False), (False, True)):
        d1, d2 = pipeline.Decoder(H, W), pipeline.Decoder(H, W)
        r1 = d1.decode(got.sym_len, got.sym_val, got.counts, got.dc, index=got.index, planes=planes, keep_blocks=keep)
        r2 = d2.decode(exp.sym_len, exp.sym_val, exp.counts, exp.dc, index=exp.index, planes=planes, keep_blocks=keep)
        torch.cuda.synchronize()
        assert torch.equal(r1, r2), (planes, keep)
        assert d1.status.cpu().tolist() == want
        for k in ("cr", "cb"):
            assert torch.equal(d1.pix[k], d2.pix[k]), (k, planes, keep)
        if keep:
            for k in pipeline.CHANNELS:
                assert torch.equal(d1.blocks[k], exp.coef[k]), k
    d3 = pipeline.Decoder(H, W, chroma_pair=False)
    assert torch.equal(d3.decode(got.sym_len, got.sym_val, got.counts, got.dc, index=got.index), r2)


def test_slots_hic_image_and_repeat():
    """Encoding a second image into the same slot-layout encoder (the records,
    index and DC patch are rewritten, not accumulated) and hic_image from the
    slots == a fresh coefficient-chain encoder's."""
    H, W = 272, 1024
    enc = pipeline.Encoder(H, W)
    assert enc.slots
    for seed, kind in ((1, "random"), (2, "sparse"), (3, "smooth")):
        x = device.to_device(_img(kind, H, W, seed))
        enc.encode(x)
        ref = pipeline.Encoder(H, W, slots=False)
        ref.encode(x)
        assert enc.hic_image().byte_stream() == ref.hic_image().byte_stream(), kind
        a, b = enc.result(), ref.result()
        for k in pipeline.CHANNELS:
            for j in range(4):
                np.testing.assert_array_equal(a[k][j], b[k][j], err_msg=(kind, k, j))


def test_slots_refused_shapes():
    """slots=True on a shape the slot layout cannot take raises; the default falls
    back to the coefficient chain there."""
    for H, W, kw in ((16, 768, {}), (24, 512, {}), (16, 512, {"max_len": 14}), (64, 1024, {"rows": (0, 32)})):
        with pytest.raises(ValueError):
            pipeline.Encoder(H, W, slots=True, **kw)
        assert not pipeline.Encoder(H, W, **kw).slots
