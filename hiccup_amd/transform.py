"""Block transforms (mirrors hiccup/transform.py:17-277).

Channel-level operations run on the GPU through the C-ABI:

* ``dct_channel``    -> hic_dct_quant_u8   (transform.py:182-193)
* ``inv_dct_channel``-> hic_dequant_idct_u8 (transform.py:169-179)
* ``dct2`` / ``idct2`` on 8x8 blocks -> hic_dct2_f64 / hic_idct2_f64 (transform.py:67-103)
* ``down_sample`` / ``up_sample`` -> hic_pyr_down_u8 / hic_pyr_up_u8 (transform.py:151-166)

``pad_matrix`` / ``split_matrix`` / ``merge_blocks`` / ``zigzag`` / ``izigzag`` /
``dc_component`` / ``ac_components`` / ``force_merge`` are the reference's
small host-side reshaping helpers with identical results; the encode/decode
paths never use them (the GPU kernels do blocking, zig-zag and cropping
themselves).  Wavelet / effect helpers belong to out-of-scope subsystems.
"""
import numpy as np
import torch

from . import _lib, device, model

_OUT_OF_SCOPE = "the wavelet (HIC) scheme and image effects are out of scope (DESIGN.md)"


# ---------------------------------------------------------------- host helpers
def pad_matrix(matrix, N):
    """transform.py:17-30: zero-pad each dimension up to a multiple of N."""
    x, y = matrix.shape
    if x % N == 0 and y % N == 0:
        return matrix
    result = np.zeros((x + (N - x % N) % N, y + (N - y % N) % N), dtype=matrix.dtype)
    result[:x, :y] = matrix
    return result


def split_matrix(matrix, N):
    """transform.py:33-42: (nblk, N, N) blocks in raster block order."""
    m = pad_matrix(np.asarray(matrix), N)
    h, w = m.shape
    return m.reshape(h // N, N, -1, N).swapaxes(1, 2).reshape(-1, N, N)


def merge_blocks(blocks, shape):
    """transform.py:45-64: reassemble raster-ordered blocks and crop to shape."""
    y, x = shape
    num, N, _ = blocks.shape
    if y * x != num * N * N:
        assert y * x < num * N * N
        y, x = -(-y // N) * N, -(-x // N) * N
    out = blocks.reshape(y // N, x // N, N, N).swapaxes(1, 2).reshape(y, x)
    return np.array(out[:shape[0], :shape[1]])


def _zigzag_order(h, w):
    order = []
    for s in range(h + w - 1):
        ys = range(max(0, s - (w - 1)), min(s, h - 1) + 1)
        ys = ys if s % 2 == 0 else reversed(ys)
        order.extend((yy, s - yy) for yy in ys)
    return order


def _zigzag_indices(matrix):
    """transform.py:106-124: (row, col) pairs in the transposed zig-zag order."""
    h, w = np.shape(matrix)[:2]
    return _zigzag_order(h, w)


def zigzag(matrix):
    m = np.asarray(matrix)
    flat = np.array([y * m.shape[1] + x for (y, x) in _zigzag_order(*m.shape)], dtype=np.int64)
    return m.reshape(-1)[flat].tolist()


def izigzag(arr, shape):
    mat = np.zeros(shape)
    for v, (y, x) in zip(arr, _zigzag_order(*shape)):
        mat[y][x] = v
    return mat


def dc_component(block):
    return block[0][0]


def ac_components(blocks):
    b = np.asarray(blocks)
    n = b.shape[-1]
    flat = np.array([y * n + x for (y, x) in _zigzag_order(n, n)], dtype=np.int64)
    return b.reshape(len(b), n * n)[:, flat[1:]].reshape(-1).tolist()


def force_merge(lu, c1, c2):
    """transform.py:269-277: crop luminance to the chroma shape, stack 3 channels."""
    shape = c1.shape
    assert shape == c2.shape
    lu = lu[:shape[0], :shape[1]]
    return np.dstack([lu, c1, c2])


# ---------------------------------------------------------------- GPU paths
def _check_block_size(block_size):
    if block_size != 8:
        raise ValueError("the JPEG quantization tables are 8x8: block_size must be 8 (got %r)" % (block_size,))


def _as_u8_plane(channel):
    ch = np.asarray(channel)
    if ch.ndim != 2:
        raise ValueError("expected a 2-D channel, got shape %s" % (ch.shape,))
    if ch.dtype != np.uint8:
        if ch.size and (ch.min() < 0 or ch.max() > 255 or not np.all(np.mod(ch, 1) == 0)):
            raise ValueError("dct_channel expects 8-bit pixel values")
        ch = ch.astype(np.uint8)
    return ch


def _as_i32_plane(channel):
    ch = np.asarray(channel)
    if ch.ndim != 2:
        raise ValueError("expected a 2-D channel, got shape %s" % (ch.shape,))
    if not np.issubdtype(ch.dtype, np.integer):
        if ch.size and not np.all(np.mod(ch, 1) == 0):
            raise ValueError("inv_dct_channel expects integer-valued coefficients")
    if ch.size and (ch.min() < -(1 << 31) or ch.max() >= (1 << 31)):
        raise ValueError("coefficients out of int32 range")
    return ch.astype(np.int32)


def _as_i32_plane_device(channel):
    """_as_i32_plane's checks and result, as an int32 device tensor (large float
    planes are checked and cast on the GPU, device.to_device_i32)."""
    ch = np.asarray(channel)
    if ch.ndim != 2:
        raise ValueError("expected a 2-D channel, got shape %s" % (ch.shape,))
    return device.to_device_i32(ch, "inv_dct_channel expects integer-valued coefficients",
                                "coefficients out of int32 range")


def dct_channel_device(plane_dev, table_id, layout=_lib.LAYOUT_RASTER_I32, out=None, stream=None):
    """Device-resident forward transform: uint8 (H, W) CUDA tensor -> coefficients."""
    H, W = plane_dev.shape
    if out is None:
        if layout == _lib.LAYOUT_RASTER_I32:
            out = device.empty((H, W), torch.int32)
        elif layout == _lib.LAYOUT_RASTER_I16:
            out = device.empty((H, W), torch.int16)
        else:
            out = device.empty((-(-H // 8) * -(-W // 8), 64), torch.int16)
    _lib.call("hic_dct_quant_u8", device.ptr(plane_dev), H, W, plane_dev.stride(0), table_id, layout,
              device.ptr(out), device.stream_ptr(stream))
    return out


def inv_dct_channel_device(coef_dev, H, W, table_id, layout=_lib.LAYOUT_RASTER_I32, out=None, stream=None):
    """Device-resident inverse transform -> uint8 (H, W) CUDA tensor."""
    if out is None:
        out = device.empty((H, W), torch.uint8)
    _lib.call("hic_dequant_idct_u8", device.ptr(coef_dev), layout, H, W, table_id, device.ptr(out), out.stride(0),
              device.stream_ptr(stream))
    return out


def dct_channel(channel, quantization_table, block_size=8):
    """transform.py:182-193: uint8 H x W -> int32 H x W quantized DCT coefficients."""
    _check_block_size(block_size)
    plane = device.to_device(_as_u8_plane(channel))
    out = dct_channel_device(plane, model.table_id(quantization_table))
    return device.to_host(out)


def inv_dct_channel(channel, quantization_table, block_size=8):
    """transform.py:169-179: coefficients H x W -> uint8 H x W pixels."""
    _check_block_size(block_size)
    coef = _as_i32_plane_device(channel)
    H, W = coef.shape
    out = inv_dct_channel_device(coef, H, W, model.table_id(quantization_table))
    return device.to_host(out)


def dct2(matrix):
    """transform.py:67-84 for 8x8 blocks (or a stack of them): float64, bit-exact."""
    m = np.asarray(matrix, dtype=np.float64)
    if m.shape[-2:] != (8, 8):
        raise NotImplementedError("dct2 is implemented for 8x8 blocks (the JPEG block size)")
    dev = device.to_device(m.reshape(-1, 64))
    out = device.empty(dev.shape, torch.float64)
    _lib.call("hic_dct2_f64", device.ptr(dev), dev.shape[0], device.ptr(out), device.stream_ptr())
    return device.to_host(out).reshape(m.shape)


def idct2(matrix):
    """transform.py:87-103 for 8x8 blocks: float64, includes the /256."""
    m = np.asarray(matrix, dtype=np.float64)
    if m.shape[-2:] != (8, 8):
        raise NotImplementedError("idct2 is implemented for 8x8 blocks (the JPEG block size)")
    dev = device.to_device(m.reshape(-1, 64))
    out = device.empty(dev.shape, torch.float64)
    _lib.call("hic_idct2_f64", device.ptr(dev), dev.shape[0], device.ptr(out), device.stream_ptr())
    return device.to_host(out).reshape(m.shape)


def _as_u8_image(matrix):
    m = np.asarray(matrix)
    if m.dtype != np.uint8 or m.ndim != 2:
        raise ValueError("pyrUp/pyrDown are implemented for 2-D uint8 planes (cv2 8U)")
    return m


def down_sample(matrix, factor=2):
    """transform.py:160-166: cv2.pyrDown(matrix, dstsize=(x // factor, y // factor))."""
    m = _as_u8_image(matrix)
    y, x = m.shape
    dh, dw = y // factor, x // factor
    src = device.to_device(m)
    out = device.empty((dh, dw), torch.uint8)
    _lib.call("hic_pyr_down_u8", device.ptr(src), y, x, device.ptr(out), dh, dw, device.stream_ptr())
    return device.to_host(out)


def up_sample(matrix, factor=2):
    """transform.py:151-157: cv2.pyrUp(matrix, dstsize=(x * factor, y * factor))."""
    m = _as_u8_image(matrix)
    y, x = m.shape
    dh, dw = y * factor, x * factor
    src = device.to_device(m)
    out = device.empty((dh, dw), torch.uint8)
    _lib.call("hic_pyr_up_u8", device.ptr(src), y, x, device.ptr(out), dh, dw, device.stream_ptr())
    return device.to_host(out)


# ---------------------------------------------------------------- out of scope
def wavelet_split_resolutions(channel, wavelet, levels=3):
    raise NotImplementedError(_OUT_OF_SCOPE)


def linearize_subband(subbands):
    raise NotImplementedError(_OUT_OF_SCOPE)


def subband_view(pyramid):
    raise NotImplementedError(_OUT_OF_SCOPE)


def wavelet_merge_resolutions(pyramid, wavelet):
    raise NotImplementedError(_OUT_OF_SCOPE)


def threshold(arr, thresh, replace=0):
    raise NotImplementedError(_OUT_OF_SCOPE)


def threshold_channel_by_quality(parts, q_factor=1):
    raise NotImplementedError(_OUT_OF_SCOPE)


def high_pass(img, ksize=3):
    raise NotImplementedError(_OUT_OF_SCOPE)


def low_pass(img, k=(3, 3)):
    raise NotImplementedError(_OUT_OF_SCOPE)


def salt_pepper(img, prob=.01):
    raise NotImplementedError(_OUT_OF_SCOPE)
