"""CPU tests: the C-ABI library and its declarations, and the host-side parts of
the package (Huffman back end, container, helpers) against the reference's
golden payloads.  No GPU, no kernel calls."""
import ctypes
import os
import re

import numpy as np
import pytest

from hiccup_amd import _lib, hicimage, huffman, iohelper, sharding, transform, utils

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "hiccup_hip.h")


def _declared():
    txt = open(HEADER).read()
    return dict((m.group(2), m.group(3)) for m in
                re.finditer(r"^(int|size_t)\s+(hic_\w+)\(([^;]*?)\);", txt, re.M | re.S))


def test_header_and_library_symbols():
    decl = _declared()
    assert len(decl) >= 25
    lib = ctypes.CDLL(_lib.LIB_PATH)  # loads without a GPU
    for name in decl:
        assert hasattr(lib, name), name


def test_ctypes_signatures_match_header():
    decl = _declared()
    assert set(decl) == set(_lib.SIGNATURES)
    for name, args in decl.items():
        nargs = 0 if args.strip() == "void" else len([a for a in args.split(",") if a.strip()])
        assert nargs == len(_lib.SIGNATURES[name][1]), name
    assert _lib.load().hic_abi_version() == 4
    # argument kinds: every pointer parameter is bound as a pointer, every scalar
    # with the header's width and signedness
    kinds = {"int64_t": ctypes.c_int64, "int": ctypes.c_int, "int32_t": ctypes.c_int32, "size_t": ctypes.c_size_t,
             "uint32_t": ctypes.c_uint32, "float": ctypes.c_float}
    for name, args in decl.items():
        if args.strip() == "void":
            continue
        for i, (a, t) in enumerate(zip(args.split(","), _lib.SIGNATURES[name][1])):
            a = " ".join(a.split())
            if "*" in a:
                assert t in (ctypes.c_void_p, ctypes.c_char_p) or hasattr(t, "_type_") and t._type_ == "P" \
                    or issubclass(t, ctypes._Pointer) or t.__name__.startswith("LP_") or \
                    t.__name__.endswith("_Array"), (name, i, a, t)
            else:
                base = a.rsplit(" ", 1)[0].replace("const ", "")
                assert base in kinds, (name, i, a)
                assert ctypes.sizeof(t) == ctypes.sizeof(kinds[base]) and t not in (ctypes.c_void_p,), (name, i, a, t)


def test_last_error_roundtrip():
    lib = _lib.load()
    rc = lib.hic_dct_quant_u8(None, 8, 8, 8, 0, 0, None, None)
    assert rc == _lib.HIC_ERR_ARG
    assert "null pointer" in _lib.last_error()
    with pytest.raises(ValueError):
        _lib.check(rc, "x")


def test_ctypes_structs_match_header(tmp_path):
    """The job structs' ctypes mirrors (_lib.RleJob16, _lib.DctPlaneJob) have the
    header's size and field offsets, as gcc lays them out."""
    import subprocess
    structs = {"hic_rle_job16": _lib.RleJob16, "hic_dct_plane_job": _lib.DctPlaneJob, "hic_slot_job": _lib.SlotJob,
               "hic_huffman_decode_job": _lib.HuffDecodeJob, "hic_encode420_job": _lib.Encode420Job,
               "hic_wire_job": _lib.WireJob}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hiccup_hip.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append('  printf("%s size %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('  printf("%s %s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                         text=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got["%s size" % cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got["%s %s" % (cname, f)]) == getattr(py, f).offset, (cname, f)


def test_round6_batch_entry_points_refuse_bad_jobs():
    """The round-6 batch entry points check every job before any device call:
    refused here without a GPU (HIC_ERR_ARG, nothing launched)."""
    lib = _lib.load()
    p = 1 << 20  # never dereferenced (16-byte aligned)
    # shard transforms: job count, a shape that is not 16-row aligned, a null buffer
    job = _lib.Encode420Job(p, 0, 64, 64, 1024, 0, 64, p, p, p, p, p, p)
    assert lib.hic_encode420_batch_u8(0, (_lib.Encode420Job * 1)(job), 15, None, None, None) == _lib.HIC_ERR_ARG
    assert lib.hic_encode420_batch_u8(9, (_lib.Encode420Job * 9)(*[job] * 9), 15, None, None, None) == _lib.HIC_ERR_ARG
    bad = _lib.Encode420Job(p, 0, 64, 64, 1024, 0, 24, p, p, p, p, p, p)
    assert lib.hic_encode420_batch_u8(2, (_lib.Encode420Job * 2)(job, bad), 15, None, None, None) == _lib.HIC_ERR_ARG
    ragged = _lib.Encode420Job(p, 0, 64, 64, 768, 0, 64, p, p, p, p, p, p)  # records need a tile pass
    assert lib.hic_encode420_batch_u8(1, (_lib.Encode420Job * 1)(ragged), 15, None, None, None) == _lib.HIC_ERR_ARG
    assert "512" in _lib.last_error()
    # wire batches: a bad table, a null wire buffer, records without a destination, too many jobs
    w = _lib.WireJob(p, p, 64, 0, p, None, 0, 0, None, None)
    for badw in (_lib.WireJob(p, p, 64, 2, p, None, 0, 0, None, None), _lib.WireJob(p, None, 64, 0, p, None, 0, 0, None, None),
                 _lib.WireJob(p, p, 64, 0, p, p, 1, 0, None, None)):
        assert lib.hic_wire_pack_batch(2, (_lib.WireJob * 2)(w, badw), None) == _lib.HIC_ERR_ARG
        assert lib.hic_wire_unpack_batch(2, (_lib.WireJob * 2)(w, badw), None) == _lib.HIC_ERR_ARG
    assert lib.hic_wire_pack_batch(33, (_lib.WireJob * 33)(*[w] * 33), None) == _lib.HIC_ERR_ARG
    assert lib.hic_wire_pack_batch(1, (_lib.WireJob * 1)(_lib.WireJob(p, p, 64, 0, None, None, 0, 0, None, None)),
                                   None) == _lib.HIC_ERR_ARG  # a pack needs its flag
    # Huffman decode batch: a job whose tree is not a tree
    child = np.array([1, -2, -3, -4], np.int32)  # node 1 exists, node 0's '1' child -> 1, node 1 children leaves
    bad_child = np.array([0, -2], np.int32)       # the root as its own child
    ok_job = _lib.HuffDecodeJob(p, 64, child.ctypes.data, 2, None, 3, p, 64, p, 0, 0)
    bad_job = _lib.HuffDecodeJob(p, 64, bad_child.ctypes.data, 1, None, 1, p, 64, p, 0, 0)
    assert lib.hic_huffman_decode_batch(2, (_lib.HuffDecodeJob * 2)(ok_job, bad_job), None) == _lib.HIC_ERR_ARG
    assert "tree edge" in _lib.last_error()
    assert lib.hic_zigzag8_blocks_i16(None, 8, 8, p, p, None) == _lib.HIC_ERR_ARG


def test_decode_rgb_indexed_arguments():
    """hic_rle_decode_idct_rgb_indexed refuses what its kernel cannot take before
    any device call: null pointers, planes that are not whole 8x8 blocks, a short or
    unaligned RGB pitch, unaligned chroma planes."""
    lib = _lib.load()
    p16 = ctypes.c_void_p(1 << 20)  # never dereferenced
    args = lambda H, W, cr=p16, stride=None: (p16, p16, p16, p16, p16, H, W, cr, p16, p16,
                                              3 * W if stride is None else stride, p16, None)
    assert lib.hic_rle_decode_idct_rgb_indexed(None, *args(64, 64)[1:]) == _lib.HIC_ERR_ARG
    assert "null pointer" in _lib.last_error()
    for H, W in ((60, 64), (64, 62), (0, 64)):
        assert lib.hic_rle_decode_idct_rgb_indexed(*args(H, W)) == _lib.HIC_ERR_ARG, (H, W)
    assert lib.hic_rle_decode_idct_rgb_indexed(*args(64, 64, stride=3 * 64 - 8)) == _lib.HIC_ERR_ARG
    assert lib.hic_rle_decode_idct_rgb_indexed(*args(64, 64, stride=3 * 64 + 4)) == _lib.HIC_ERR_ARG
    assert lib.hic_rle_decode_idct_rgb_indexed(*args(64, 64, cr=ctypes.c_void_p((1 << 20) + 2))) == _lib.HIC_ERR_ARG
    assert "aligned" in _lib.last_error()


def test_decode_pair_indexed_arguments():
    """hic_rle_decode_idct_u8_indexed_pair checks both planes' pointers before any
    device call."""
    lib = _lib.load()
    p16 = ctypes.c_void_p(1 << 20)  # never dereferenced
    two = lambda a=p16, b=p16: (ctypes.c_void_p * 2)(a, b)
    ok = lambda **kw: [kw.get("L", two()), two(), two(), two(), two(), 64, 64, 1, two(), 64, two(), None]
    assert lib.hic_rle_decode_idct_u8_indexed_pair(*ok(L=two(b=None))) == _lib.HIC_ERR_ARG
    assert "plane 1: null pointer" in _lib.last_error()
    assert lib.hic_rle_decode_idct_u8_indexed_pair(*ok(L=two(b=ctypes.c_void_p((1 << 20) + 8)))) == _lib.HIC_ERR_ARG
    assert "16-byte aligned" in _lib.last_error()
    bad_table = ok()
    bad_table[7] = 5
    assert lib.hic_rle_decode_idct_u8_indexed_pair(*bad_table) == _lib.HIC_ERR_ARG


def test_knob_defaults_and_ranges():
    """The launch defaults the measurements chose (hic_get_knob reports the effective
    value; no GPU call): encode_order 6 = XCD-major workgroups + odd unit rows
    bottom-up (profiles/r04/enc_order_xcd); out-of-range values are refused."""
    assert _lib.get_knob("encode_order") == 6
    assert _lib.get_knob("dct_path") == _lib.DCT_PATH_F64 == 1
    with _lib.knobs(encode_order=2):
        assert _lib.get_knob("encode_order") == 2
    assert _lib.get_knob("encode_order") == 6
    for bad in (8, 3, 1):  # odd: the stacked-unit order was removed in round 5
        with pytest.raises(ValueError):
            _lib.set_knob("encode_order", bad)
    with _lib.knobs(dct_path=_lib.DCT_PATH_EXACT):
        assert _lib.get_knob("dct_path") == 0
    for bad in (3, 4, 5, -2):  # 3 / 4: the packed and two-lane kernels, removed in round 5
        assert _lib.load().hic_set_knob(0, bad) == _lib.HIC_ERR_ARG
    for retired in (9, 10, 11, 12, 14, 15):  # retired knobs: any value but the default is refused
        assert _lib.load().hic_set_knob(retired, 0) == _lib.HIC_ERR_ARG
    # resetting every knob to its default works (-1 on a retired knob is a no-op)
    for k in range(16):
        assert _lib.load().hic_set_knob(k, -1) == _lib.HIC_OK, k


def _names(d, prefix):
    return sorted(k[len(prefix):] for k in d if k.startswith(prefix))


def test_huffman_tables_and_bits_golden(golden_codec):
    """Host Huffman (byte-compatible with huffman.py) on the reference's own DC / RLE
    streams reproduces its tables and bit strings."""
    g = golden_codec
    for name in _names(g, "bs_"):
        for ch in ("lum", "cr", "cb"):
            streams = {"dc": g["dc_%s_%s" % (ch, name)], "av": g["acv_%s_%s" % (ch, name)],
                       "al": g["acl_%s_%s" % (ch, name)]}
            for kind, key in (("dc", "dc"), ("av", "av"), ("al", "al")):
                keys = streams[key]
                tree = huffman.HuffmanTree.construct_from_counts(*huffman.first_appearance_counts(keys))
                table = tree.encode_table()
                assert [v for v, _ in table] == g["%shv_%s_%s" % (kind, ch, name)].tolist(), (name, ch, kind)
                assert [c for _, c in table] == g["%shc_%s_%s" % (kind, ch, name)].tolist(), (name, ch, kind)
                bits = tree.encode_keys(keys)
                assert bits == str(g["%sb_%s_%s" % (kind, ch, name)]), (name, ch, kind)
                # decode side: rebuild from the table, decode the bits
                dec = huffman.HuffmanTree.construct_from_coding(table)
                assert dec.decode_data(bits) == keys.tolist()
                # the slow generic path agrees with the vectorised one
                slow = huffman.HuffmanTree.construct_from_data(keys.tolist())
                assert slow.encode_table() == table and slow.encode_data() == bits


def test_huffman_reference_unit_cases():
    # huffmantest.py
    t = huffman.HuffmanTree.construct_from_data([0, 0, 0, 0, 0])
    assert len(t.leaves) == 1 and t.encode_data() == "11111"
    t = huffman.HuffmanTree.construct_from_data([0, 0, 0, 1])
    assert t.root.frequency == 4 and t.root.left.value == 1 and t.root.right.value == 0
    data = [1, 2, 2, 3, 3, 3, 4, 4, 4, 4]
    t = huffman.HuffmanTree.construct_from_data(data)
    out = t.encode_data()
    assert out == "001" + ("000" * 2) + ("01" * 3) + ("1" * 4)
    assert t.decode_data(out) == data
    t = huffman.HuffmanTree.construct_from_data([("A", 0), ("B", 1), ("B", 0)], key_func=lambda x: x[0])
    assert t.root.left.value == "A" and t.root.right.value == "B"


def test_iohelper_reference_cases():
    # iohelpertest.py
    assert iohelper.bin_string(3) == "11"
    assert iohelper.padded_bs_2_bytes("101") == b"\x05\xa0"
    assert iohelper.padded_bytes_2_bs(bytearray(b"\x05\xa0")) == "101"
    for s in ["01", "0000", "1010000", "00000", "000111", "00000001", "000001", "0000001", "10010110",
              "0" * 777 + "1"] + [bin(i)[2:] for i in range(1, 5000, 37)]:
        assert iohelper.padded_bytes_2_bs(iohelper.padded_bs_2_bytes(s)) == s
    with pytest.raises(AssertionError):
        iohelper.bin_string_as_bytes("0")


def test_utils_reference_cases():
    # utilstest.py
    assert utils.group_tuples([1, 2, 3, 4], 2) == [(1, 2), (3, 4)]
    with pytest.raises(AssertionError):
        utils.group_tuples([1, 2, 3], 2)
    for n, b in [[0, 0], [1, 1], [2, 2], [3, 2], [4, 3], [100, 7], [-60, 6], [-1, 1]]:
        assert utils.num_bits_for_int(n) == b
    assert utils.differences([1, 5, 12, 0]) == [1, 4, 7, -12]
    assert utils.invert_differences([1, 1, 1, 1]) == [1, 2, 3, 4]
    assert utils.group_by([1, 2, 2, 3, 3, 3])[3] == [3, 3, 3]
    assert utils.flatten([[1, 2], [3, 4]]) == [1, 2, 3, 4]
    assert utils.img_as_list(np.array([[1, 2], [3, 4]])) == [1, 2, 3, 4]
    assert utils.dict_map({"a": 1, "b": 2}, lambda k, v: k + str(v)) == {"a": "a1", "b": "b2"}
    assert utils.is_gray(np.array([[1, 2], [2, 3]])) and not utils.is_gray(np.array([[1, 2]]))
    with pytest.raises(RuntimeError):
        utils.first([1, 2], lambda x: x < 0)


def test_transform_host_helpers(golden_tables):
    # transformtest.py:21-53,70-120,195-211
    sq = np.array([[1, 2], [3, 4]])
    sp = transform.split_matrix(sq, 1)
    assert len(sp) == 4 and [b[0][0] for b in sp] == [1, 2, 3, 4]
    sp = transform.split_matrix(np.arange(1, 10).reshape(3, 3), 2)
    assert len(sp) == 4 and np.sum(sp[0]) == 12 and np.sum(sp[3]) == 9
    blocks = np.array([[[1, 2], [7, 8]], [[3, 4], [9, 10]], [[5, 6], [11, 12]],
                       [[13, 14], [0, 0]], [[15, 16], [0, 0]], [[17, 18], [0, 0]]])
    assert np.array_equiv(transform.merge_blocks(blocks, (4, 6)),
                          [[1, 2, 3, 4, 5, 6], [7, 8, 9, 10, 11, 12], [13, 14, 15, 16, 17, 18], [0] * 6])
    m = np.random.default_rng(0).integers(0, 256, (8, 12))
    assert np.array_equiv(transform.merge_blocks(transform.split_matrix(m, 4), m.shape), m)
    assert transform.zigzag(np.arange(1, 10).reshape(3, 3)) == [1, 4, 2, 3, 5, 7, 8, 6, 9]
    assert np.array_equiv(transform.izigzag(np.array([1, 4, 2, 3, 5, 7, 8, 6, 9]), (3, 3)),
                          np.arange(1, 10).reshape(3, 3))
    m = np.random.default_rng(1).integers(0, 256, (17, 19))
    assert np.array_equiv(transform.izigzag(transform.zigzag(m), m.shape), m)
    for n in (2, 3, 4, 8):
        order = [y * n + x for y, x in transform._zigzag_indices(np.zeros((n, n)))]
        assert order == golden_tables["zz%d" % n].tolist()
    assert transform.dc_component(np.array([[1, 2], [3, 4]])) == 1
    assert transform.ac_components(np.array([[[1, 2], [3, 4]], [[5, 6], [7, 8]]])) == [3, 2, 4, 7, 6, 8]


def test_container_roundtrip(tmp_path):
    payloads = ([hicimage.PayloadStringP(hicimage.TupP, [hicimage.TupP(5, "10"), hicimage.TupP(-3, "0")])] * 9
                + [hicimage.BitStringP("1011")] * 9 + [hicimage.TupP(16, 24), hicimage.TupP(8, 12)])
    img = hicimage.HicImage.jpeg_image(payloads)
    back = hicimage.HicImage.from_bytes(img.byte_stream())
    assert all(a == b for a, b in zip(img.payloads, back.payloads))
    path = str(tmp_path / "x.hic")
    img.write_file(path)
    again = hicimage.HicImage.from_file(path)
    assert all(a == b for a, b in zip(img.payloads, again.payloads))


def test_shard_plan_and_stitch():
    for H, world in ((4320, 8), (4320 * 8, 8), (33, 2), (250, 3), (97, 5)):
        p = sharding.plan(H, world)
        assert p[0][0] == 0 and p[-1][1] == H
        assert all(a[1] == b[0] for a, b in zip(p, p[1:]))
        assert all(r0 % 16 == 0 for r0, _ in p)
    with pytest.raises(ValueError):
        sharding.plan(16, 2)
    s = np.array([[3, 1, 5, 6], [63, 0, 1, 1], [10, 1, 2, 3]])
    assert sharding.stitch_host(s, 0).tolist() == [0, 0, 0, 0]
    assert sharding.stitch_host(s, 1).tolist() == [3, 0, 1, 6]
    assert sharding.stitch_host(s, 2).tolist() == [66, 1, 1, 1]


def test_bitstring_packed_matches_string_form():
    """BitStringP.from_packed (the GPU packer's output) gives the same payload and
    container bytes as the '0'/'1' string form (iohelper.padded_bs_2_bytes)."""
    import numpy as np
    rng = np.random.default_rng(7)
    for nbits in [0, 1, 3, 7, 8, 9, 15, 16, 17, 64, 1001]:
        bits = rng.integers(0, 2, nbits).astype(np.uint8)
        packed = np.packbits(bits) if nbits else np.zeros(0, np.uint8)
        s = "".join("1" if b else "0" for b in bits)
        a, b = hicimage.BitStringP.from_packed(packed, nbits), hicimage.BitStringP(s)
        assert a.byte_stream == b.byte_stream == iohelper.padded_bs_2_bytes(s), nbits
        assert a.payload == s and a == b


def test_container_bytes_match_reference():
    """The reference's own container bytes (tests/golden/hicimage_cases.npz, written
    by hiccup.hicimage under this Python): our loader reads them (the class
    reference hiccup.hicimage.TupP and numpy scalars, nothing else), re-serialises
    them byte for byte, and the tables built here from the same planes are the
    same bytes (hicimage.py:117-121, codec.py:304-334)."""
    import numpy as np
    import pickle
    import oracle.oracle as orc
    from hiccup_amd import codec
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "hicimage_cases.npz"))
    assert int(g["pickle_protocol"]) == pickle.DEFAULT_PROTOCOL
    for i in list(range(9)) + [18, 19]:
        raw = bytes(g["payload_%02d" % i])
        p = (hicimage.TupP if i >= 18 else hicimage.PayloadStringP).from_bytes(raw)
        assert p.byte_stream == raw, i
    assert hicimage.PlainStringP.from_bytes(bytes(g["settings_0"])).payload == "JPEG"
    for c, ch in enumerate(("lum", "cr", "cb")):
        plane = g["in_" + ch].astype(np.int32)
        zz = orc.zigzag_blocks(orc.split_blocks(plane)).astype(np.int64)
        dc = orc.dpcm(zz[:, 0])
        L, V = orc.rle_encode(zz[:, 1:].reshape(-1), 15)
        for j, (keys, kt) in enumerate(((dc, np.int32), (V, int), (L, int))):
            uniq, counts = huffman.first_appearance_counts(keys)
            tree = huffman.HuffmanTree.construct_from_counts(uniq, counts)
            assert codec.huffman_encode(tree, kt).byte_stream == bytes(g["payload_%02d" % (3 * j + c)]), (ch, j)


def test_container_refuses_foreign_pickles():
    import pickle
    evil = pickle.dumps({"type": os.system, "data": []})
    with pytest.raises(pickle.UnpicklingError):
        hicimage.PayloadStringP.from_bytes(evil)


def test_fused_colour_arithmetic_exhaustive():
    """encode.hip's dot4 restatement of RGB2YCrCb equals the oracle on all 2^24
    RGB triples (tools/check/colour_dot4.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "colour_dot4", os.path.join(os.path.dirname(__file__), "..", "tools", "check", "colour_dot4.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.check()


def test_decode_colour_arithmetic_exhaustive():
    """color.hip's decode colour arithmetic (packed biased pyrUp sums, v_dot2 per
    channel) equals the oracle's pyrUp rounding and YCrCb2RGB on every input
    (tools/check/colour_decode_dot2.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "colour_decode_dot2", os.path.join(os.path.dirname(__file__), "..", "tools", "check", "colour_decode_dot2.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.check()


def test_wire_views_are_byte_views_of_the_tensor():
    """sharding._wire: every point-to-point transfer moves a uint8 view (torch's
    NCCL process group refuses int16); a receive into the view lands in the tensor."""
    import torch
    from hiccup_amd import sharding
    t = torch.arange(12, dtype=torch.int16).reshape(3, 4)
    w = sharding._wire(t)
    assert w.dtype == torch.uint8 and w.shape == (3, 8) and w.data_ptr() == t.data_ptr()
    w.copy_(sharding._wire(torch.full((3, 4), -2, dtype=torch.int16)))
    assert int(t.sum()) == -24
    d = torch.arange(5, dtype=torch.int32)
    assert sharding._wire(d[1:4]).numel() == 12
    b = torch.zeros(7, dtype=torch.uint8)
    assert sharding._wire(b) is b
    with pytest.raises(ValueError):
        sharding._wire(t[:, ::2])


def _ref_padded_bytes_2_bs(b):
    """iohelper.py:51-56 restated with bitstring's semantics: the first byte read
    as a signed int p, the whole buffer shifted left 8 bits (zero fill, same
    length), then ``bin[:-p-8]``."""
    p = b[0] - 256 if b[0] >= 128 else b[0]
    bits = "".join(format(x, "08b") for x in b)
    shifted = bits[8:] + "0" * 8
    return shifted[:-p - 8]


def test_padded_bytes_every_pad_byte():
    """padded_bytes_2_bs and BitStringP.from_bytes (which keeps the bits packed for
    the GPU decoder) agree with the reference's slicing for every pad byte,
    including the signed and out-of-range ones a foreign file could hold."""
    rng = np.random.default_rng(5)
    for nbody in range(0, 5):
        body = bytes(rng.integers(0, 256, nbody, dtype=np.uint8).tolist())
        for pad in range(256):
            b = bytes([pad]) + body
            want = _ref_padded_bytes_2_bs(b)
            assert iohelper.padded_bytes_2_bs(b) == want, (nbody, pad)
            bsp = hicimage.BitStringP.from_bytes(b)
            packed, nbits = bsp.packed_bits()
            assert nbits == len(want), (nbody, pad)
            assert np.unpackbits(np.asarray(packed, np.uint8))[:nbits].tolist() == [int(c) for c in want]
            assert bsp.payload == want
            # re-serialising gives what the reference writes for those bits
            assert bsp.byte_stream == iohelper.padded_bs_2_bytes(want), (nbody, pad)


def _walk_flat(child, leaves, bits):
    """decode_data over the flat arrays hic_huffman_decode takes (the kernel's
    semantics, restated bit by bit)."""
    out, node = [], 0
    for ch in bits:
        c = child[2 * node + (0 if ch == "1" else 1)]
        if c == -1:
            raise AttributeError("missing child")
        if c < 0:
            out.append(leaves[-2 - c].value)
            node = 0
        else:
            node = c
    return out


def test_huffman_flat_tree_matches_walk(golden_codec):
    """HuffmanTree.flat() (the decode kernel's tree) decodes the golden bit strings
    to the golden keys, for trees rebuilt from the tables and built from the data."""
    g = golden_codec
    for name in _names(g, "bs_"):
        for ch in ("lum", "cr", "cb"):
            for kind, key in (("dc", "dc"), ("av", "acv"), ("al", "acl")):
                keys = g["%s_%s_%s" % (key, ch, name)]
                table = list(zip(g["%shv_%s_%s" % (kind, ch, name)].tolist(),
                                 g["%shc_%s_%s" % (kind, ch, name)].tolist()))
                bits = str(g["%sb_%s_%s" % (kind, ch, name)])
                for tree in (huffman.HuffmanTree.construct_from_coding(table),
                             huffman.HuffmanTree.construct_from_counts(*huffman.first_appearance_counts(keys))):
                    child, leaves = tree.flat()
                    assert child.dtype == np.int32 and child.size % 2 == 0
                    assert _walk_flat(child.tolist(), leaves, bits) == keys.tolist()
                    # the decode's output sizing: no key takes fewer bits than this
                    assert tree.min_code_length() == min(len(c) for _, c in table)
                    assert len(keys) <= max(len(bits) // tree.min_code_length(), 1)
    # a one-leaf encoding tree: its empty '0' side is a missing child
    t = huffman.HuffmanTree.construct_from_data([7, 7, 7])
    child, leaves = t.flat()
    assert child.tolist() == [-2, -1] and leaves[0].value == 7
    with pytest.raises(AttributeError):
        _walk_flat(child.tolist(), leaves, "10")
    with pytest.raises(AttributeError):
        t.decode_data("10")


def test_native_codebook_golden(golden_codec):
    """CodeBook (hic_huffman_build, the native heapq tree codec.jpeg_encode uses)
    reproduces the reference's tables on its own DC / RLE streams, and FlatCodes
    (hic_huffman_from_codes, jpeg_decode's tree) decodes its bit strings."""
    g = golden_codec
    for name in _names(g, "bs_"):
        for ch in ("lum", "cr", "cb"):
            for kind, key in (("dc", "dc"), ("av", "acv"), ("al", "acl")):
                keys = g["%s_%s_%s" % (key, ch, name)]
                table = list(zip(g["%shv_%s_%s" % (kind, ch, name)].tolist(),
                                 g["%shc_%s_%s" % (kind, ch, name)].tolist()))
                cb = huffman.CodeBook(*huffman.first_appearance_counts(keys))
                assert cb.encode_table() == table, (name, ch, kind)
                bits = str(g["%sb_%s_%s" % (kind, ch, name)])
                flat = huffman.FlatCodes.from_table(table)
                if len(table) < 2:  # a one-code table has an unused '0' side: the reference's tree
                    assert flat is None
                    continue
                assert _walk_flat(flat.child.tolist(), [huffman.HuffmanTree.Node.leaf(int(v), 0)
                                                        for v in flat.values], bits) == keys.tolist()
                assert flat.minlen == min(len(c) for _, c in table)


@pytest.mark.parametrize("kind", ["uniform", "geometric", "equal_counts", "many_leaves"])
def test_native_trees_match_heapq(kind):
    """The native trees == the node-object trees (heapq, huffman.py:60-79), ties
    included: equal counts in every arrangement, and more than 2500 leaves (CPython's
    heapify switches to its cache-friendly order there; the heap it builds is the
    same).  FlatCodes == construct_from_coding + flat() on the resulting tables."""
    rng = np.random.default_rng({"uniform": 1, "geometric": 2, "equal_counts": 3, "many_leaves": 4}[kind])
    for _ in range(25 if kind != "many_leaves" else 4):
        n = int(rng.integers(1, 4000))
        if kind == "uniform":
            keys = rng.integers(-int(rng.integers(1, 60)), 60, n)
        elif kind == "geometric":
            keys = rng.geometric(0.3, n) * rng.choice([-1, 1], n)
        elif kind == "equal_counts":
            keys = np.repeat(rng.integers(-500, 500, max(1, n // 7)), int(rng.integers(1, 8)))
        else:
            keys = rng.permutation(np.repeat(np.arange(-1500, 1700), 1 + np.arange(3200) % 3))
        uniq, counts = huffman.first_appearance_counts(keys)
        ref = huffman.HuffmanTree.construct_from_counts(uniq, counts)
        cb = huffman.CodeBook(uniq, counts)
        table = ref.encode_table()
        assert cb.encode_table() == table
        lo, nb = min(uniq), max(uniq) - min(uniq) + 1
        for a, b in zip(ref.code_table(lo, nb), cb.code_table(lo, nb)):
            np.testing.assert_array_equal(a, b)
        flat = huffman.FlatCodes.from_table(table)
        if len(uniq) == 1:
            assert flat is None
            continue
        dec = huffman.HuffmanTree.construct_from_coding(table)
        child, leaves = dec.flat()
        np.testing.assert_array_equal(flat.child, child)
        assert flat.nnodes == child.size // 2
        assert flat.values.tolist() == [l.value for l in leaves]
        assert flat.minlen == dec.min_code_length()


def test_native_flat_codes_refuses_irregular_tables():
    """Tables that are not a complete prefix code of int32 values stay with the
    reference's own construction (FlatCodes.from_table -> None); a repeated code
    keeps its last value, as the reference's dict does."""
    for table in ([(5, "1")], [(5, "1"), (6, "01")], [(5, "1"), (6, "0"), (7, "10")], [(5, "1"), (6, "0x")],
                  [(5, ""), (6, "0")], [(None, "1"), (6, "0")], [(2 ** 31, "1"), (6, "0")], [(1.0, "1"), (6, "0")]):
        assert huffman.FlatCodes.from_table(table) is None, table
    f = huffman.FlatCodes.from_table([(5, "1"), (6, "0"), (9, "1")])
    assert f.values.tolist() == [9, 6] and f.child.tolist() == [-2, -3]
    f = huffman.FlatCodes.from_table([(np.int64(-3), "11"), (4, "10"), (True, "0")])
    assert f.values.tolist() == [1, -3, 4] and f.minlen == 1
    with pytest.raises(ValueError):
        huffman.CodeBook([], [])


def test_rle_workspace_covers_scan_partitions():
    """hic_rle_workspace_bytes (rle.hip) holds, for any channel size and record
    density (one record per 64-block tile, or per 32-block half tile as the fused
    encoder's chroma writes them), the records (3 int64), the offsets (2 int64) and
    the scan's hand-off granules: 3 per 256-record partition + the failure granule
    (k_rle_scan16b, kScan16T = 256 in the product build)."""
    lib = _lib.load()
    for n in (1, 63, 64, 65, 4095, 32400, 129600, 518400, 4194304):
        have = lib.hic_rle_workspace_bytes(n, 64)
        for rpt in (1, 2):
            nrec = -(-n * rpt // 64)
            need = (5 * nrec + 3 * -(-nrec // 256) + 1) * 8
            assert have >= need, (n, rpt, have, need)


@pytest.mark.parametrize("H,W", [(1024, 16), (2048, 16), (1024, 48), (48, 16), (16, 1040), (1088, 1920),
                                 (2160, 3840), (4320, 7680)])
def test_rle_rows_workspace_covers_segment_records(H, W):
    """a whole image's fused encoder with a ragged last strip
    (hic_encode420_seg_u8) writes one record per strip segment of every block row:
    rows x ceil(W / 512) of them, far more than the 64-block tiles of a narrow, tall
    image.  hic_rle_rows_workspace_bytes covers those records, their offsets and the
    scan's granules, and the Encoder sizes its workspaces with it (and the library
    refuses a smaller one, tested on the GPU)."""
    from hiccup_amd import pipeline
    lib = _lib.load()
    fused, rpt = pipeline.encoder_layout(H, W)
    for k, (h, w, rowb) in {"lum": (H, W, W // 8), "cr": (H // 2, W // 2, W // 16)}.items():
        n = (h // 8) * (w // 8)
        nrec = (n // rowb) * -(-rowb // (64 // rpt[k]))
        need = (5 * nrec + 3 * -(-nrec // 256) + 1) * 8
        have = lib.hic_rle_rows_workspace_bytes(n, rowb, rpt[k])
        assert have >= need and have >= lib.hic_rle_workspace_bytes(n, 64), (k, have, need)
    if W <= 48 and H >= 1024:  # the case the advisor found: the tile-sized workspace is too small
        n = (H // 8) * (W // 8)
        assert lib.hic_rle_workspace_bytes(n, 64) < lib.hic_rle_rows_workspace_bytes(n, W // 8, 1)


def test_stream_gather_record_layout_past_2gib():
    """a stream gather's landing zone takes the SHARDS' RLE record
    layout.  At 32768^2 the whole image (3.2 GB of RGB) cannot run the fused kernel
    while its 8 row shards can (their chroma records are 32-block half tiles); the
    wire segments are sized with the shards' layout, and every rank makes the same
    fused decision (all shards fusable), so the ranges agree across ranks."""
    from hiccup_amd import pipeline
    H = W = 32768
    assert pipeline.encoder_layout(H, W)[0] is False
    rows = sharding.plan(H, 8)
    lay = [pipeline.encoder_layout(H, W, rr) for rr in rows]
    assert all(f for f, _ in lay)
    assert all(r == {"lum": 1, "cr": 2, "cb": 2} for _, r in lay)
    ranges = sharding.block_ranges(H, W, 8)
    wr = sharding.wire_ranges(ranges, lay[0][1], sharding.records_aligned(ranges, lay[0][1]))
    lib = _lib.load()
    for k in sharding.CHANNELS:
        for (b0, b1), (o0, o1) in zip(ranges[k], wr[k]):
            n = b1 - b0
            nrec = -(-n * lay[0][1][k] // 64)
            assert o1 - o0 == (lib.hic_wire_bytes(n, sharding.TABLE_OF[k]) + -(-nrec * sharding.REC_BYTES // 16) * 16
                               + sharding.TRAILER_BYTES)
    # a ragged image whose last shard cannot fuse: one decision for all (the chain)
    rows = sharding.plan(4328, 4)
    assert not all(pipeline.encoder_layout(4328, 7680, rr)[0] for rr in rows)


def test_jpeg_decode_gc_pause_is_shared():
    """jpeg_decode pauses the process-wide cyclic collector; calls
    that overlap (nested or on other threads) share one pause, the collector stays
    off until the last ends, and its state from before the first returns."""
    import gc
    import threading
    from hiccup_amd import codec
    assert gc.isenabled()
    inside, release = threading.Event(), threading.Event()

    def other():
        with codec._gc_paused():
            inside.set()
            release.wait(10)

    t = threading.Thread(target=other)
    t.start()
    assert inside.wait(10)
    with codec._gc_paused():
        assert not gc.isenabled()
    assert not gc.isenabled()  # the other call still runs
    release.set()
    t.join(10)
    assert gc.isenabled()
    gc.disable()
    try:
        with codec._gc_paused():
            pass
        assert not gc.isenabled()  # a collector the caller had off stays off
    finally:
        gc.enable()


def test_pinned_staging_chunks():
    """the pinned staging buffers are capped (two of _CHUNK bytes,
    round 6); larger copies go in _CHUNK pieces that tile the copy exactly (int32 /
    float64 aligned)."""
    from hiccup_amd import device
    assert device._staging_lock is not None
    for n in [device._PIN_MIN, device._CHUNK - 8, device._CHUNK, device._CHUNK + 4, 5 * device._CHUNK + 12]:
        ch = device._chunks(n)
        assert ch[0][0] == 0 and sum(c for _, c in ch) == n
        assert all(o1 == o0 + c0 for (o0, c0), (o1, _) in zip(ch, ch[1:]))
        assert all(c <= device._CHUNK and o % 8 == 0 for o, c in ch)
