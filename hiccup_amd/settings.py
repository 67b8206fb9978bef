"""Runtime configuration (mirrors hiccup/settings.py:10-23).

Mutable module globals, read at call time exactly like the reference:
``codec.jpeg_encode`` / ``jpeg_decode`` use ``JPEG_BLOCK_SIZE``; the wavelet
knobs exist for API compatibility only (the wavelet scheme is out of scope).
"""
from . import model

DEBUG = True

WAVELET = model.Wavelet.DAUBECHIE
WAVELET_QUALITY_FACTOR = 1
WAVELET_SUBBAND_QUANTIZATION_MULTIPLIER = 1
WAVELET_THRESHOLD = 5
WAVELET_NUM_LEVELS = 3
WAVELET_TILES = 8

JPEG_BLOCK_SIZE = 8


def JPEG_BLOCK_SHAPE():
    return JPEG_BLOCK_SIZE, JPEG_BLOCK_SIZE
