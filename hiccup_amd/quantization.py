"""JPEG table quantization (mirrors hiccup/quantization.py:14-94).

``jpeg_quantize`` / ``invert_jpeg_quantize`` run on the GPU (hic_quantize_f64 /
hic_dequantize_i32): IEEE float64 divide, round half to even, int32 -- exactly
``np.round(np.divide(b, T)).astype(int32)`` (quantization.py:47-52,80-81).
The fused channel path (transform.dct_channel) never calls these; they are the
reference's block-level helpers.  ``round_quantize`` / ``deadzone_quantize`` are
the reference's generic numpy one-liners and stay host-side; the wavelet
subband helpers belong to the out-of-scope HIC scheme.
"""
import numpy as np
import torch

from . import _lib, device, model

table = {
    model.QTables.JPEG_LUMINANCE: np.array([
        [16, 11, 10, 16, 24, 40, 51, 61],
        [12, 12, 14, 19, 26, 58, 60, 55],
        [14, 13, 16, 24, 40, 57, 69, 56],
        [14, 17, 22, 29, 51, 87, 80, 62],
        [18, 22, 37, 56, 68, 109, 103, 77],
        [24, 35, 55, 64, 81, 104, 113, 92],
        [49, 64, 78, 87, 103, 121, 120, 101],
        [72, 92, 95, 98, 112, 100, 103, 99]]),
    model.QTables.JPEG_CHROMINANCE: np.array(
        [[17, 18, 24, 47] + [99] * 4, [18, 21, 26, 66] + [99] * 4,
         [24, 26, 56] + [99] * 5, [47, 66] + [99] * 6] + [[99] * 8] * 4),
}

all_tables = set(table.keys())


def _as_blocks(block):
    b = np.asarray(block, dtype=np.float64)
    if b.shape[-2:] != (8, 8):
        raise ValueError("JPEG quantization tables are 8x8: got blocks of shape %s" % (b.shape,))
    return b


def jpeg_quantize(block, option):
    """round_half_even(block / T) as int32, for one 8x8 block or a stack of them."""
    b = _as_blocks(block)
    dev = device.to_device(b.reshape(-1, 64))
    out = device.empty(dev.shape, torch.int32)
    _lib.call("hic_quantize_f64", device.ptr(dev), dev.shape[0], model.table_id(option), device.ptr(out),
              device.stream_ptr())
    return device.to_host(out).reshape(b.shape)


def invert_jpeg_quantize(block, option):
    """block * T (quantization.py:55-57) for integer-valued blocks."""
    b = np.asarray(block)
    if b.shape[-2:] != (8, 8):
        raise ValueError("JPEG quantization tables are 8x8: got blocks of shape %s" % (b.shape,))
    if not np.issubdtype(b.dtype, np.integer):
        if not np.all(np.mod(b, 1) == 0):
            raise ValueError("invert_jpeg_quantize expects integer-valued coefficients")
    dev = device.to_device(b.astype(np.int32).reshape(-1, 64))
    out = device.empty(dev.shape, torch.int64)
    _lib.call("hic_dequantize_i32", device.ptr(dev), dev.shape[0], model.table_id(option), device.ptr(out),
              device.stream_ptr())
    r = device.to_host(out).reshape(b.shape)
    return r if np.issubdtype(b.dtype, np.integer) else r.astype(np.float64)


def round_quantize(block):
    return np.round(block).astype(np.int32)


def deadzone_quantize(block, div):
    return round_quantize(np.divide(block, div))


def subband_quantize(subbands, multiplier=1):
    raise NotImplementedError("the wavelet (HIC) scheme is out of scope (DESIGN.md)")


def subband_invert_quantize(subbands, multiplier=1):
    raise NotImplementedError("the wavelet (HIC) scheme is out of scope (DESIGN.md)")


def quality_threshold_value(vals, q_factor=1):
    s = sorted(vals)
    keep = int(np.ceil(len(vals) * q_factor))
    return s[len(vals) - keep]
