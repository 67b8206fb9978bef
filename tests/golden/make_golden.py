"""Generate the golden parity fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

This script is test infrastructure.  It runs only in the build container (where
the read-only reference checkout lives at /root/reference); the GPU box never
runs it and never sees the reference.  The fixtures it writes are plain data
(inputs + the reference's outputs) saved with ``np.savez_compressed`` and
loadable with ``allow_pickle=False``.

How the reference is imported
-----------------------------
``hiccup.transform`` / ``hiccup.codec`` import ``cv2``, ``pywt``, ``rawpy`` and
``bitstring`` at module load.  None of those packages exists in this image and
none of them is *called* by the functions pinned here (dct_channel,
inv_dct_channel, dct2, idct2, zigzag, jpeg_quantize, run_length_coding,
decode_run_length, differential_coding, jpeg_encode's DC/RLE/Huffman stages).
We register EMPTY module objects under those four names so the import
succeeds; every number below is computed by the reference's own Python code on
top of the real numpy 2.2 / scipy 1.15 (pocketfft) in this container.

The colour conversion / pyrDown inputs for the Lenna planes cannot come from
the reference (it calls OpenCV, which is absent): they are produced by this
repo's own restatement of OpenCV's fixed-point formulas (oracle/oracle.py) and
are marked "parity unpinned" in DESIGN.md.  The DCT / quantize / RLE outputs on
those planes ARE the reference's.

Run:  python tests/golden/make_golden.py      (takes ~2-3 minutes)
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.dont_write_bytecode = True
for _name in ("cv2", "pywt", "rawpy", "bitstring"):
    sys.modules.setdefault(_name, types.ModuleType(_name))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

import hiccup.settings as settings  # noqa: E402
import hiccup.model as model  # noqa: E402
import hiccup.transform as transform  # noqa: E402
import hiccup.quantization as qz  # noqa: E402
import hiccup.codec as codec  # noqa: E402

settings.DEBUG = False
LUM = model.QTables.JPEG_LUMINANCE
CHR = model.QTables.JPEG_CHROMINANCE


def out(name):
    return os.path.join(HERE, name)


def zigzag_tables():
    d = {}
    for n in (1, 2, 3, 4, 5, 8):
        idx = transform._zigzag_indices(np.zeros((n, n)))
        d["zz%d" % n] = np.array([y * n + x for (y, x) in idx], dtype=np.int32)
    # a non-square case, the reference's zigzag accepts any 2-D array
    idx = transform._zigzag_indices(np.zeros((3, 5)))
    d["zz3x5"] = np.array([y * 5 + x for (y, x) in idx], dtype=np.int32)
    d["lum_table"] = qz.table[LUM].astype(np.int32)
    d["chr_table"] = qz.table[CHR].astype(np.int32)
    np.savez_compressed(out("tables.npz"), **d)


def tie_blocks(rng, count, table_id):
    """Random 8x8 uint8 blocks forced onto exact quantizer ties at (4,4)/(2,2).

    (4,4): b44 = 2*sum(x_mn s_m s_n), s = [+,-,-,+,+,-,-,+] (x = pixel-128), an
    integer; the lum quantizer (68) ties when b44 % 68 == 34.
    (2,2): b22 = 2(A+B) + sqrt2 (A-B+C); forcing A-B+C = 0 makes it rational.
    """
    s = np.array([1, -1, -1, 1, 1, -1, -1, 1])
    s44 = np.outer(s, s)
    c = np.array([1, 3, -3, -1, -1, -3, 3, 1])  # pattern of cos(pi(2m+1)/8) classes
    cls = np.outer(np.abs(c), np.abs(c))  # 1 -> c1c1 (A), 9 -> c3c3 (B), 3 -> cross (C)
    sign = np.outer(np.sign(c), np.sign(c))
    blocks = []
    while len(blocks) < count:
        x = rng.integers(-128, 128, (8, 8))
        kind = len(blocks) % 2
        if kind == 0:
            b44 = 2 * int(np.sum(x * s44))
            if table_id == 0 and b44 % 68 != 34:
                # nudge pixel (0,0) (s44 = +1) by the needed amount if possible
                need = (34 - b44 % 68) // 2
                if -128 <= x[0, 0] + need < 128:
                    x[0, 0] += need
                else:
                    continue
        else:
            A = int(np.sum(x * sign * (cls == 1)))
            B = int(np.sum(x * sign * (cls == 9)))
            C = int(np.sum(x * sign * (cls == 3)))
            adj = A - B + C  # remove via a class-A pixel with sign +1: (0,0)
            if not (-128 <= x[0, 0] - adj < 128):
                continue
            x[0, 0] -= adj
        blocks.append(x + 128)
    return np.array(blocks, dtype=np.uint8)


def transform_cases():
    rng = np.random.default_rng(1234)
    planes = {
        "r256_lum": (rng.integers(0, 256, (256, 256), dtype=np.uint8), LUM),
        "r256_chr": (rng.integers(0, 256, (256, 256), dtype=np.uint8), CHR),
        "odd37x53_lum": (rng.integers(0, 256, (37, 53), dtype=np.uint8), LUM),
        "odd37x53_chr": (rng.integers(0, 256, (37, 53), dtype=np.uint8), CHR),
        "odd13x200_lum": (rng.integers(0, 256, (13, 200), dtype=np.uint8), LUM),
        "tiny1x1_lum": (np.array([[200]], dtype=np.uint8), LUM),
        "tiny3x9_chr": (rng.integers(0, 256, (3, 9), dtype=np.uint8), CHR),
        "const128_lum": (np.full((120, 80), 128, np.uint8), LUM),
        "const0_lum": (np.zeros((120, 80), np.uint8), LUM),
        "const1_lum": (np.ones((120, 80), np.uint8), LUM),
        "const255_chr": (np.full((64, 64), 255, np.uint8), CHR),
        "extreme_lum": ((np.indices((64, 64)).sum(0) % 2 * 255).astype(np.uint8), LUM),
        "grad_lum": ((np.add.outer(np.arange(96), np.arange(160)) % 256).astype(np.uint8), LUM),
    }
    ties_l = tie_blocks(rng, 512, 0)  # (512, 8, 8)
    ties_c = tie_blocks(rng, 256, 1)
    # lay tie blocks out as a plane: 8 rows of blocks
    planes["ties_lum"] = (ties_l.reshape(8, 64, 8, 8).swapaxes(1, 2).reshape(64, 512), LUM)
    planes["ties_chr"] = (ties_c.reshape(8, 32, 8, 8).swapaxes(1, 2).reshape(64, 256), CHR)
    d = {}
    for name, (plane, table) in planes.items():
        q = transform.dct_channel(plane, table)
        rec = transform.inv_dct_channel(q, table)
        d["in_" + name] = plane
        d["q_" + name] = np.asarray(q).astype(np.int32)
        d["rec_" + name] = np.asarray(rec).astype(np.uint8)
        d["tab_" + name] = np.int32(0 if table == LUM else 1)
    # inverse on arbitrary (not DCT-produced) coefficient planes: wrap/trunc path
    for name, shape, table, lo, hi in (("rand_coef_lum", (64, 72), LUM, -60, 60),
                                      ("rand_coef_chr", (40, 24), CHR, -40, 40),
                                      ("rand_coef_odd", (21, 35), LUM, -8, 8)):
        c = rng.integers(lo, hi, shape).astype(np.int32)
        d["icin_" + name] = c
        d["icout_" + name] = np.asarray(transform.inv_dct_channel(c, table)).astype(np.uint8)
        d["ictab_" + name] = np.int32(0 if table == LUM else 1)
    # raw dct2/idct2 on single blocks (float64 bit patterns)
    blk = rng.integers(-512, 512, (64, 8, 8))
    d["dct2_in"] = blk.astype(np.int64)
    d["dct2_out"] = np.array([transform.dct2(b) for b in blk])
    d["idct2_out"] = np.array([transform.idct2(b) for b in d["dct2_out"]])
    np.savez_compressed(out("transform_cases.npz"), **d)
    print("transform cases:", len(planes))


def rle_pack(rl):
    return (np.array([r.length for r in rl], dtype=np.int64),
            np.array([r.value for r in rl], dtype=np.int64))


def rle_cases():
    rng = np.random.default_rng(99)
    cases = [
        ("t_run_length", transform.zigzag(np.array([
            [99, -59, 0, 7, 0, 0, 0, 0], [0] * 8, [0] * 8, [0] * 8,
            [12, -2, 0, 0, 0, 0, 0, 0], [0] * 8, [0] * 8, [0] * 8])), 15),
        ("t_trivial", [2, 3, 4], 15),
        ("t_too_long", [0] * 17 + [1], 15),
        ("t_sym00_a", [0, 0, 5], 15),
        ("t_sym00_b", [0, 0, 5, 0, 0], 15),
        ("t_max_len", [0, 0, 0, 0, 0, 1], 15),
        ("t_consec", [0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0], 15),
        ("t_break_plus_1", [0, 0, 0, 0, 0, 1], 4),
        ("t_max_double", [-1, 0, 0, 0, 0, 1, 2], 4),
        ("t_accidental", [0] * 14 + [31], 15),
        ("e_empty", [], 15),
        ("e_single_zero", [0], 15),
        ("e_single_val", [-7], 15),
        ("e_all_zero", [0] * 100, 15),
        ("e_run15", [0] * 15 + [3], 15),
        ("e_run30", [0] * 30 + [3], 15),
        ("e_run31", [0] * 31 + [7], 15),
        ("e_run44", [0] * 44 + [9, 0, 0], 15),
        ("e_maxlen1", [0, 0, 3, 0, 4, 0, 0], 1),
        ("e_nosplit", [0] * 40 + [5, 0, 0, 6], 0),
    ]
    for i, (dens, n, ml) in enumerate([(0.02, 5000, 15), (0.1, 5000, 15), (0.5, 5000, 15),
                                       (0.9, 5000, 15), (0.05, 3000, 4), (0.3, 3000, 7),
                                       (0.01, 20000, 15), (0.05, 4000, 0)]):
        vals = rng.integers(-300, 300, n)
        vals[vals == 0] = 1
        mask = rng.random(n) < dens
        arr = np.where(mask, vals, 0)
        if i % 2:
            arr[-37:] = 0
        cases.append(("rnd%d" % i, arr.tolist(), ml))
    d = {}
    for name, arr, ml in cases:
        rl = codec.run_length_coding(np.array(arr, dtype=np.int64), max_len=(ml if ml else None))
        L, V = rle_pack(rl)
        dec = codec.decode_run_length(rl, len(arr))
        d["in_" + name] = np.array(arr, dtype=np.int64)
        d["ml_" + name] = np.int64(ml)
        d["len_" + name] = L
        d["val_" + name] = V
        d["dec_" + name] = np.array(dec, dtype=np.int64)
    # decode-side edge cases straight from codectest
    rl = [codec.RunLength(value=0, length=14), codec.RunLength(value=31, length=0)]
    d["dec_accidental"] = np.array(codec.decode_run_length(rl, 15), dtype=np.int64)
    np.savez_compressed(out("rle_cases.npz"), **d)
    print("rle cases:", len(cases))


def huff_pack(payload_string):
    vals = np.array([p.numbers[0] for p in payload_string.payloads], dtype=np.int64)
    codes = np.array([p.numbers[1] for p in payload_string.payloads], dtype=np.str_)
    return vals, codes


def codec_cases():
    rng = np.random.default_rng(7)
    cases = [
        ("t_encode", 8, [[1, 2], [3, 4]], [[5, 6], [7, 8]], [[9, 10], [11, 12]]),
        ("t_inverse", 2, [[1, 2, 11, 22], [3, 4, 33, 44]], [[5, 6, 55, 66], [7, 8, 77, 88]],
         [[9, 10, 99, 1010], [11, 12, 1111, 1212]]),
        ("t_inner_zeros", 2, [[1, 0, 0, 22], [3, 0, 33, 44]], [[5, 6, 0, 66], [7, 8, 77, 88]],
         [[9, 0, 99, 1010], [11, 12, 1111, 1212]]),
        ("t_end_zeros", 2, [[1, 2, 11, 0], [3, 0, 33, 0]], [[5, 6, 55, 0], [7, 8, 77, 0]],
         [[9, 10, 99, 0], [11, 12, 1111, 0]]),
        ("t_zero_blocks", 2, [[0, 0, 11, 0], [0, 0, 0, 0]], [[0, 0, 55, 0], [0, 0, 0, 0]],
         [[9, 10, 99, 1010], [11, 12, 1111, 1212]]),
    ]
    # DCT-produced coefficient planes (the realistic input of jpeg_encode)
    for i, (h, w) in enumerate([(32, 48), (24, 40), (20, 28)]):
        y = transform.dct_channel(rng.integers(0, 256, (h, w), dtype=np.uint8), LUM)
        cr = transform.dct_channel(rng.integers(90, 170, (h // 2, w // 2), dtype=np.uint8), CHR)
        cb = transform.dct_channel(rng.integers(100, 140, (h // 2, w // 2), dtype=np.uint8), CHR)
        cases.append(("dct%d" % i, 8, y, cr, cb))
    d = {}
    for name, bs, y, cr, cb in cases:
        settings.JPEG_BLOCK_SIZE = bs
        ci = model.CompressedImage(np.array(y), np.array(cr), np.array(cb))
        hic = codec.jpeg_encode(ci)
        p = hic.payloads
        d["bs_" + name] = np.int64(bs)
        for k, ch in enumerate(("lum", "cr", "cb")):
            d["in_%s_%s" % (ch, name)] = np.asarray(ci.as_dict[ch]).astype(np.int64)
            blocks = transform.split_matrix(ci.as_dict[ch], bs)
            d["dc_%s_%s" % (ch, name)] = np.array(codec.differential_coding(blocks), dtype=np.int64)
            L, V = rle_pack(codec.run_length_coding(transform.ac_components(blocks)))
            d["acl_%s_%s" % (ch, name)] = L
            d["acv_%s_%s" % (ch, name)] = V
            for j, kind in enumerate(("dch", "avh", "alh")):
                vals, codes = huff_pack(p[3 * j + k])
                d["%sv_%s_%s" % (kind, ch, name)] = vals
                d["%sc_%s_%s" % (kind, ch, name)] = codes
            for j, kind in enumerate(("dcb", "avb", "alb")):
                d["%s_%s_%s" % (kind, ch, name)] = np.array(p[9 + 3 * j + k].payload, dtype=np.str_)
        d["shape0_" + name] = np.array(p[18].numbers, dtype=np.int64)
        d["shape1_" + name] = np.array(p[19].numbers, dtype=np.int64)
        try:
            dec = codec.jpeg_decode(hic)
        except AssertionError:
            # the reference's jpeg_decode asserts (utils.group_tuples) whenever a
            # plane is not a multiple of the block size: record the failure
            d["decfail_" + name] = np.int64(1)
            continue
        d["decfail_" + name] = np.int64(0)
        for ch in ("lum", "cr", "cb"):
            d["dec_%s_%s" % (ch, name)] = np.asarray(dec.as_dict[ch]).astype(np.float64)
    settings.JPEG_BLOCK_SIZE = 8
    np.savez_compressed(out("codec_cases.npz"), **d)
    print("codec cases:", len(cases))


def lenna():
    from PIL import Image
    import oracle.oracle as orc
    rgb = np.asarray(Image.open(os.path.join(REF, "resources/Lenna.png")).convert("RGB"))
    y, cr, cb = orc.rgb_to_ycrcb(rgb)
    crd, cbd = orc.pyr_down(cr), orc.pyr_down(cb)
    d = {"rgb": rgb, "y": y, "cr": crd, "cb": cbd}
    for ch, plane, table in (("y", y, LUM), ("cr", crd, CHR), ("cb", cbd, CHR)):
        q = transform.dct_channel(plane, table)
        d["q_" + ch] = np.asarray(q).astype(np.int16)
        d["rec_" + ch] = np.asarray(transform.inv_dct_channel(q, table)).astype(np.uint8)
        blocks = transform.split_matrix(q, 8)
        d["dc_" + ch] = np.array(codec.differential_coding(blocks), dtype=np.int32)
        if ch != "y":
            L, V = rle_pack(codec.run_length_coding(transform.ac_components(blocks)))
            d["acl_" + ch] = L.astype(np.int32)
            d["acv_" + ch] = V.astype(np.int32)
    # luminance RLE on the top 256 rows (the reference's RLE is quadratic)
    blocks = transform.split_matrix(d["q_y"][:256].astype(np.int32), 8)
    L, V = rle_pack(codec.run_length_coding(transform.ac_components(blocks)))
    d["acl_y256"] = L.astype(np.int32)
    d["acv_y256"] = V.astype(np.int32)
    np.savez_compressed(out("lenna.npz"), **d)
    print("lenna done")


def hicimage_cases():
    """The reference's container payload bytes (hicimage.py:31-121): the nine
    Huffman tables (PayloadStringP: a pickle naming the payload CLASS), the two
    shape TupPs and the settings PlainStringP of jpeg_encode on codec case
    inputs.  BitStringP bytes need the absent ``bitstring`` package, so they are not
    recorded here (their format is pinned by iohelpertest.py's vectors)."""
    import hiccup.hicimage as hicimage
    rng = np.random.default_rng(11)
    d = {}
    settings.JPEG_BLOCK_SIZE = 8
    y = transform.dct_channel(rng.integers(0, 256, (32, 48), dtype=np.uint8), LUM)
    cr = transform.dct_channel(rng.integers(90, 170, (16, 24), dtype=np.uint8), CHR)
    cb = transform.dct_channel(rng.integers(100, 140, (16, 24), dtype=np.uint8), CHR)
    hic = codec.jpeg_encode(model.CompressedImage(y, cr, cb))
    for k, ch in enumerate(("lum", "cr", "cb")):
        d["in_" + ch] = np.asarray(hic is not None and {"lum": y, "cr": cr, "cb": cb}[ch]).astype(np.int64)
    for i in list(range(9)) + [18, 19]:
        d["payload_%02d" % i] = np.frombuffer(hic.payloads[i].byte_stream, dtype=np.uint8)
    d["settings_0"] = np.frombuffer(hic.settings[0].byte_stream, dtype=np.uint8)
    d["pickle_protocol"] = np.int64(__import__("pickle").DEFAULT_PROTOCOL)
    assert isinstance(hic.payloads[0], hicimage.PayloadStringP)
    np.savez_compressed(out("hicimage_cases.npz"), **d)
    print("hicimage cases:", len(d))


if __name__ == "__main__":
    which = sys.argv[1:] or ["tables", "transform", "rle", "codec", "lenna", "hicimage"]
    if "hicimage" in which:
        hicimage_cases()
    if "tables" in which:
        zigzag_tables()
    if "transform" in which:
        transform_cases()
    if "rle" in which:
        rle_cases()
    if "codec" in which:
        codec_cases()
    if "lenna" in which:
        lenna()
