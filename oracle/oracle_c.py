"""ctypes wrapper of the C oracle (oracle/hiccup_oracle.c -> oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY (checker + CPU baseline); see hiccup_oracle.c's header
for the reference file:line each function restates.  The C oracle is what the
GPU box uses to check full-size (4K/8K) planes bit-exactly, since the
reference itself never leaves the build container.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_i64 = ctypes.c_int64
_vp = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.orc_dct_channel.argtypes = [_vp, _i64, _i64, _i64, ctypes.c_int, _vp]
        L.orc_dct_channel_mt.argtypes = [_vp, _i64, _i64, _i64, ctypes.c_int, _vp, ctypes.c_int]
        L.orc_inv_dct_channel.argtypes = [_vp, _i64, _i64, ctypes.c_int, _vp]
        L.orc_zigzag_indices.argtypes = [ctypes.c_int, ctypes.c_int, _vp]
        L.orc_zigzag_blocks.argtypes = [_vp, _i64, _i64, ctypes.c_int, _vp]
        L.orc_zigzag_blocks.restype = _i64
        L.orc_dpcm.argtypes = [_vp, _i64, _vp]
        L.orc_rle_encode.argtypes = [_vp, _i64, _i64, _vp, _vp, _i64]
        L.orc_rle_encode.restype = _i64
        L.orc_rle_decode.argtypes = [_vp, _vp, _i64, _i64, _vp, _i64]
        L.orc_rle_decode.restype = _i64
        L.orc_rgb_to_ycrcb.argtypes = [_vp, _i64, _vp, _vp, _vp]
        L.orc_ycrcb_to_rgb.argtypes = [_vp, _vp, _vp, _i64, _vp]
        L.orc_pyr_down.argtypes = [_vp, _i64, _i64, _vp, _i64, _i64]
        L.orc_pyr_up.argtypes = [_vp, _i64, _i64, _vp, _i64, _i64]
        L.orc_dct2.argtypes = [_vp, _vp]
        L.orc_idct2.argtypes = [_vp, _vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def dct_channel(plane, table_id, threads=1):
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    out = np.empty((H, W), np.int32)
    if threads > 1:
        lib().orc_dct_channel_mt(_p(plane), H, W, W, table_id, _p(out), threads)
    else:
        lib().orc_dct_channel(_p(plane), H, W, W, table_id, _p(out))
    return out


def inv_dct_channel(coef, table_id):
    coef = np.ascontiguousarray(coef, dtype=np.int32)
    H, W = coef.shape
    out = np.empty((H, W), np.uint8)
    lib().orc_inv_dct_channel(_p(coef), H, W, table_id, _p(out))
    return out


def dct2(block):
    b = np.ascontiguousarray(block, dtype=np.int64)
    out = np.empty((8, 8), np.float64)
    lib().orc_dct2(_p(b), _p(out))
    return out


def idct2(block):
    b = np.ascontiguousarray(block, dtype=np.float64)
    out = np.empty((8, 8), np.float64)
    lib().orc_idct2(_p(b), _p(out))
    return out


def zigzag_indices(h, w=None):
    w = h if w is None else w
    out = np.empty(h * w, np.int32)
    lib().orc_zigzag_indices(h, w, _p(out))
    return out


def zigzag_blocks(raster, n=8):
    raster = np.ascontiguousarray(raster, dtype=np.int32)
    H, W = raster.shape
    nblk = (-(-H // n)) * (-(-W // n))
    out = np.empty((nblk, n * n), np.int32)
    lib().orc_zigzag_blocks(_p(raster), H, W, n, _p(out))
    return out


def dpcm(dc):
    dc = np.ascontiguousarray(dc, dtype=np.int32)
    out = np.empty_like(dc)
    lib().orc_dpcm(_p(dc), len(dc), _p(out))
    return out


def rle_encode(arr, max_len=15):
    arr = np.ascontiguousarray(arr, dtype=np.int32)
    cap = len(arr) + 1 + (len(arr) // max(1, max_len or 1) if max_len else 0) + 1
    L = np.empty(cap, np.int32)
    V = np.empty(cap, np.int32)
    n = lib().orc_rle_encode(_p(arr), len(arr), max_len or 0, _p(L), _p(V), cap)
    assert n >= 0
    return L[:n].copy(), V[:n].copy()


def rle_decode(lengths, values, length):
    L = np.ascontiguousarray(lengths, dtype=np.int32)
    V = np.ascontiguousarray(values, dtype=np.int32)
    cap = int(np.sum(L.astype(np.int64) + 1)) + max(0, int(length))
    out = np.empty(max(cap, 1), np.int32)
    n = lib().orc_rle_decode(_p(L), _p(V), len(L), length, _p(out), cap)
    assert n >= 0
    return out[:n].copy()


def rgb_to_ycrcb(rgb):
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    y, cr, cb = (np.empty((H, W), np.uint8) for _ in range(3))
    lib().orc_rgb_to_ycrcb(_p(rgb), H * W, _p(y), _p(cr), _p(cb))
    return y, cr, cb


def ycrcb_to_rgb(y, cr, cb):
    y, cr, cb = (np.ascontiguousarray(a, dtype=np.uint8) for a in (y, cr, cb))
    H, W = y.shape
    out = np.empty((H, W, 3), np.uint8)
    lib().orc_ycrcb_to_rgb(_p(y), _p(cr), _p(cb), H * W, _p(out))
    return out


def pyr_down(plane, dst_shape=None):
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    DH, DW = dst_shape if dst_shape is not None else (H // 2, W // 2)
    out = np.empty((DH, DW), np.uint8)
    lib().orc_pyr_down(_p(plane), H, W, _p(out), DH, DW)
    return out


def pyr_up(plane, dst_shape=None):
    plane = np.ascontiguousarray(plane, dtype=np.uint8)
    H, W = plane.shape
    DH, DW = dst_shape if dst_shape is not None else (2 * H, 2 * W)
    out = np.empty((DH, DW), np.uint8)
    lib().orc_pyr_up(_p(plane), H, W, _p(out), DH, DW)
    return out


def encode_plane(coef_raster, max_len=15):
    """Front half of codec.jpeg_encode for one channel (codec.py:287-301):
    returns (dc_diffs, ac_rle_lengths, ac_rle_values)."""
    zz = zigzag_blocks(coef_raster, 8)
    dc = dpcm(zz[:, 0].copy())
    L, V = rle_encode(zz[:, 1:].reshape(-1), max_len)
    return dc, L, V
