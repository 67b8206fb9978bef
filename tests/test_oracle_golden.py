"""Pin the CPU oracles (numpy + C) against the reference's own outputs.

The fixtures under tests/golden/ were produced by tests/golden/make_golden.py,
which runs the reference (hiccup @ /root/reference) itself.  Every check here
is bit-exact (integer / byte / float64 bit patterns).
"""
import numpy as np
import pytest

import oracle.oracle as orc
import oracle.oracle_c as orcc


def _names(d, prefix):
    return sorted(k[len(prefix):] for k in d if k.startswith(prefix))


def test_tables(golden_tables):
    np.testing.assert_array_equal(golden_tables["lum_table"], orc.LUM_TABLE)
    np.testing.assert_array_equal(golden_tables["chr_table"], orc.CHR_TABLE)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8])
def test_zigzag_indices(golden_tables, n):
    np.testing.assert_array_equal(golden_tables["zz%d" % n], orc.zigzag_indices(n))
    np.testing.assert_array_equal(golden_tables["zz%d" % n], orcc.zigzag_indices(n))


def test_zigzag_nonsquare(golden_tables):
    np.testing.assert_array_equal(golden_tables["zz3x5"], orc.zigzag_indices(3, 5))
    np.testing.assert_array_equal(golden_tables["zz3x5"], orcc.zigzag_indices(3, 5))


def test_zigzag_reference_example():
    # transformtest.py:96-105
    m = np.array([[1, 2, 3], [4, 5, 6], [7, 8, 9]])
    assert m.reshape(-1)[orc.zigzag_indices(3)].tolist() == [1, 4, 2, 3, 5, 7, 8, 6, 9]


def test_dct2_idct2_bits(golden_transform):
    g = golden_transform
    a = orc.dct2(g["dct2_in"].astype(np.float64))
    assert np.array_equal(a.view(np.int64), g["dct2_out"].view(np.int64))
    b = orc.idct2(g["dct2_out"])
    assert np.array_equal(b.view(np.int64), g["idct2_out"].view(np.int64))
    for i in range(8):
        assert np.array_equal(orcc.dct2(g["dct2_in"][i]).view(np.int64), g["dct2_out"][i].view(np.int64))
        assert np.array_equal(orcc.idct2(g["dct2_out"][i]).view(np.int64), g["idct2_out"][i].view(np.int64))


def test_dct_channel_cases(golden_transform):
    g = golden_transform
    names = _names(g, "in_")
    assert len(names) >= 15
    for name in names:
        plane, tab = g["in_" + name], int(g["tab_" + name])
        q = orc.dct_channel(plane, tab)
        np.testing.assert_array_equal(q, g["q_" + name], err_msg=name)
        np.testing.assert_array_equal(orcc.dct_channel(plane, tab), g["q_" + name], err_msg=name)
        np.testing.assert_array_equal(orcc.dct_channel(plane, tab, threads=3), g["q_" + name], err_msg=name)


def test_inv_dct_channel_cases(golden_transform):
    g = golden_transform
    for name in _names(g, "in_"):
        tab = int(g["tab_" + name])
        np.testing.assert_array_equal(orc.inv_dct_channel(g["q_" + name], tab), g["rec_" + name], err_msg=name)
        np.testing.assert_array_equal(orcc.inv_dct_channel(g["q_" + name], tab), g["rec_" + name], err_msg=name)
    for name in _names(g, "icin_"):
        tab = int(g["ictab_" + name])
        np.testing.assert_array_equal(orc.inv_dct_channel(g["icin_" + name], tab), g["icout_" + name])
        np.testing.assert_array_equal(orcc.inv_dct_channel(g["icin_" + name], tab), g["icout_" + name])


def test_tie_planes_really_tie(golden_transform):
    """The tie fixtures exercise exact .5 quotients at (0,0) and (4,4)."""
    plane = g = golden_transform["in_ties_lum"].astype(np.int64) - 128
    blocks = orc.split_blocks(plane)
    s = np.array([1, -1, -1, 1, 1, -1, -1, 1])
    b44 = 2 * np.einsum("bmn,m,n->b", blocks, s, s)
    assert np.sum(b44 % 68 == 34) >= 200
    assert np.sum(blocks.sum((1, 2)) % 4 == 2) >= 50
    del g


def test_rle_cases(golden_rle):
    g = golden_rle
    names = _names(g, "in_")
    for name in names:
        arr, ml = g["in_" + name], int(g["ml_" + name])
        L, V = orc.rle_encode(arr, ml)
        np.testing.assert_array_equal(L, g["len_" + name], err_msg=name)
        np.testing.assert_array_equal(V, g["val_" + name], err_msg=name)
        L2, V2 = orcc.rle_encode(arr, ml)
        np.testing.assert_array_equal(L2, g["len_" + name], err_msg=name)
        np.testing.assert_array_equal(V2, g["val_" + name], err_msg=name)
        dec = orc.rle_decode(g["len_" + name], g["val_" + name], len(arr))
        np.testing.assert_array_equal(dec, g["dec_" + name], err_msg=name)
        dec2 = orcc.rle_decode(g["len_" + name], g["val_" + name], len(arr))
        np.testing.assert_array_equal(dec2, g["dec_" + name], err_msg=name)
    np.testing.assert_array_equal(orc.rle_decode([14, 0], [0, 31], 15), g["dec_accidental"])


def test_codec_front_half(golden_codec):
    g = golden_codec
    for name in _names(g, "bs_"):
        bs = int(g["bs_" + name])
        for ch in ("lum", "cr", "cb"):
            plane = g["in_%s_%s" % (ch, name)]
            blocks = orc.split_blocks(plane, bs)
            zz = orc.zigzag_blocks(blocks)
            np.testing.assert_array_equal(orc.dpcm(zz[:, 0]), g["dc_%s_%s" % (ch, name)])
            L, V = orc.rle_encode(zz[:, 1:].reshape(-1), 15)
            np.testing.assert_array_equal(L, g["acl_%s_%s" % (ch, name)])
            np.testing.assert_array_equal(V, g["acv_%s_%s" % (ch, name)])
            if bs == 8:
                dc, L2, V2 = orcc.encode_plane(plane)
                np.testing.assert_array_equal(dc, g["dc_%s_%s" % (ch, name)])
                np.testing.assert_array_equal(L2, g["acl_%s_%s" % (ch, name)])
                np.testing.assert_array_equal(V2, g["acv_%s_%s" % (ch, name)])


def test_lenna(golden_lenna):
    g = golden_lenna
    for ch, tab in (("y", 0), ("cr", 1), ("cb", 1)):
        q = orcc.dct_channel(g[ch], tab)
        np.testing.assert_array_equal(q, g["q_" + ch])
        np.testing.assert_array_equal(orcc.inv_dct_channel(q, tab), g["rec_" + ch])
        dc, L, V = orcc.encode_plane(q)
        np.testing.assert_array_equal(dc, g["dc_" + ch])
        if ch != "y":
            np.testing.assert_array_equal(L, g["acl_" + ch])
            np.testing.assert_array_equal(V, g["acv_" + ch])
    dc, L, V = orcc.encode_plane(g["q_y"][:256])
    np.testing.assert_array_equal(L, g["acl_y256"])
    np.testing.assert_array_equal(V, g["acv_y256"])


def test_opencv_restatements_agree():
    """numpy and C restatements of the (unpinned) OpenCV kernels agree, and the
    reference's own pins hold (transformtest.py:122-146: constant 2 survives)."""
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (37, 50, 3), dtype=np.uint8)
    for a, b in zip(orc.rgb_to_ycrcb(rgb), orcc.rgb_to_ycrcb(rgb)):
        np.testing.assert_array_equal(a, b)
    y, cr, cb = orc.rgb_to_ycrcb(rgb)
    np.testing.assert_array_equal(orc.ycrcb_to_rgb(y, cr, cb), orcc.ycrcb_to_rgb(y, cr, cb))
    for shape in ((37, 50), (16, 16), (5, 3), (1, 7)):
        p = rng.integers(0, 256, shape, dtype=np.uint8)
        if shape[0] >= 2 and shape[1] >= 2:
            np.testing.assert_array_equal(orc.pyr_down(p), orcc.pyr_down(p))
        np.testing.assert_array_equal(orc.pyr_up(p), orcc.pyr_up(p))
    two = np.full((4, 4), 2, np.uint8)
    np.testing.assert_array_equal(orc.pyr_down(two), np.full((2, 2), 2, np.uint8))
    np.testing.assert_array_equal(orc.pyr_up(two[:2, :2]), np.full((4, 4), 2, np.uint8))
