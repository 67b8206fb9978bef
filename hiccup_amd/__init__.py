"""hiccup_amd -- MI355X-native drop-in for hiccup's 8x8 DCT / quantize / zig-zag /
DC-DPCM / RLE encode path and its inverse.

Modules mirror the reference's own (nhomble/hiccup @ /root/reference/hiccup):
``transform``, ``quantization``, ``codec``, ``compression``, ``model``,
``settings``, ``utils``, ``huffman``, ``hicimage``, ``iohelper``.  Every
channel-level operation runs in hand-written gfx950 HIP kernels reached through
the C-ABI in ``include/hiccup_hip.h`` (``_lib``); there is no CPU fallback.
``pipeline`` is the device-resident batch encoder used by ``bench.py`` and
``sharding`` the multi-GPU (one process per GPU, RCCL) tile-sharded encoder.
"""
__version__ = "0.1.0"
