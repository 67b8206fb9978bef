"""Channel orchestration (mirrors hiccup/compression.py:16-56), JPEG flavour.

``jpeg_compression``: RGB -> YCrCb + 4:2:0 pyrDown (hic_rgb_to_ycrcb420, one
fused kernel) -> three hic_dct_quant_u8 launches (luminance / chrominance
tables) -> CompressedImage of int32 coefficient planes.
``jpeg_decompression``: three hic_dequant_idct_u8 launches -> fused pyrUp +
crop + YCrCb->RGB (hic_ycrcb420_to_rgb).
Colour / pyramid kernels restate OpenCV 8U and are parity-unpinned.
"""
import numpy as np
import torch

from . import _lib, device, model, settings, transform, utils

_OUT_OF_SCOPE = "the wavelet (HIC) scheme is out of scope (DESIGN.md)"


def _check_block():
    if settings.JPEG_BLOCK_SIZE != 8:
        raise ValueError("the JPEG quantization tables are 8x8: settings.JPEG_BLOCK_SIZE must be 8")


def ycrcb420_device(rgb_dev, stream=None):
    """RGB (H, W, 3) uint8 device tensor -> (Y (H, W), Cr, Cb (H//2, W//2)) device tensors."""
    H, W = rgb_dev.shape[:2]
    y = device.empty((H, W), torch.uint8)
    cr = device.empty((H // 2, W // 2), torch.uint8)
    cb = device.empty((H // 2, W // 2), torch.uint8)
    _lib.call("hic_rgb_to_ycrcb420", device.ptr(rgb_dev), H, W, device.ptr(y), device.ptr(cr), device.ptr(cb),
              device.stream_ptr(stream))
    return y, cr, cb


def jpeg_compression(rgb_image):
    """compression.py:16-39: H x W x 3 uint8 -> CompressedImage(int32 planes)."""
    utils.debug_msg("Starting JPEG compression")
    _check_block()
    rgb = np.asarray(rgb_image)
    if rgb.ndim != 3 or rgb.shape[2] != 3 or rgb.dtype != np.uint8:
        raise ValueError("jpeg_compression expects an H x W x 3 uint8 image")
    y, cr, cb = ycrcb420_device(device.to_device(rgb))
    planes = {
        "lum": transform.dct_channel_device(y, 0),
        "cr": transform.dct_channel_device(cr, 1),
        "cb": transform.dct_channel_device(cb, 1),
    }
    return model.CompressedImage.from_dict(dict((k, device.to_host(v)) for k, v in planes.items()))


def jpeg_decompression(d):
    """compression.py:42-56: CompressedImage -> (2h) x (2w) x 3 uint8 RGB."""
    _check_block()
    lum = transform._as_i32_plane_device(d.luminance_component)
    cr = transform._as_i32_plane_device(d.red_chrominance_component)
    cb = transform._as_i32_plane_device(d.blue_chrominance_component)
    assert cr.shape == cb.shape  # transform.force_merge
    H, W = lum.shape
    h, w = cr.shape
    if 2 * h > H or 2 * w > W:
        raise ValueError("luminance plane smaller than the up-sampled chroma planes")
    y = transform.inv_dct_channel_device(lum, H, W, 0)
    crp = transform.inv_dct_channel_device(cr, h, w, 1)
    cbp = transform.inv_dct_channel_device(cb, h, w, 1)
    rgb = device.empty((2 * h, 2 * w, 3), torch.uint8)
    _lib.call("hic_ycrcb420_to_rgb", device.ptr(y), y.stride(0), device.ptr(crp), device.ptr(cbp), h, w,
              device.ptr(rgb), device.stream_ptr())
    return device.to_host(rgb)


def encode(rgb_image):
    """Convenience: compression.jpeg_compression then codec.jpeg_encode."""
    from . import codec
    return codec.jpeg_encode(jpeg_compression(rgb_image))


def decode(hic_image):
    """Convenience: codec.jpeg_decode then compression.jpeg_decompression."""
    from . import codec
    return jpeg_decompression(codec.jpeg_decode(hic_image))


def wavelet_compression(rgb_image):
    raise NotImplementedError(_OUT_OF_SCOPE)


def wavelet_decompression(channels):
    raise NotImplementedError(_OUT_OF_SCOPE)
