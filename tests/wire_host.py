"""Host restatement of the gather's wire format (hiccup_amd/csrc/wire.hip), for the
CPU gloo tests of the stream gather.  Test infrastructure: the GPU kernels are
pinned to it by tests/test_gpu_codec.py::test_wire_pack_unpack."""
import numpy as np

BLOCK_BITS = 16 + 63 * 13  # 835
TILE_BYTES = 1672 * 4      # 1670 words + 2 words of padding


def wire_bytes(nblk):
    return 0 if nblk <= 0 else -(-nblk // 64) * TILE_BYTES


def _fields():
    return np.array([16] + [13] * 63)


def pack(blocks):
    """(n, 64) int16 zig-zag blocks -> uint8 wire bytes (LSB-first bit stream per tile)."""
    blocks = np.asarray(blocks, dtype=np.int16)
    n = blocks.shape[0]
    nt = -(-n // 64)
    full = np.zeros((nt * 64, 64), np.int64)
    full[:n] = blocks
    ac = full[:, 1:]
    if np.any(ac < -4096) or np.any(ac > 4095):
        raise ValueError("AC value outside 13 bits")
    widths = _fields()
    masked = np.where(np.arange(64) == 0, full & 0xFFFF, full & 0x1FFF)
    bits = []
    for j, nb in enumerate(widths):
        bits.append((masked[:, j:j + 1] >> np.arange(nb)) & 1)
    stream = np.concatenate(bits, axis=1).reshape(nt, 64 * BLOCK_BITS).astype(np.uint8)
    tiles = np.zeros((nt, TILE_BYTES * 8), np.uint8)
    tiles[:, :64 * BLOCK_BITS] = stream
    return np.packbits(tiles, axis=1, bitorder="little").reshape(-1)


def unpack(wire, nblk):
    """The inverse: wire bytes -> (nblk, 64) int16 blocks."""
    nt = -(-nblk // 64)
    bits = np.unpackbits(np.asarray(wire, np.uint8)[:nt * TILE_BYTES].reshape(nt, TILE_BYTES), axis=1,
                         bitorder="little")[:, :64 * BLOCK_BITS].reshape(nt * 64, BLOCK_BITS).astype(np.int64)
    out = np.zeros((nt * 64, 64), np.int64)
    pos = 0
    for j, nb in enumerate(_fields()):
        v = (bits[:, pos:pos + nb] << np.arange(nb)).sum(axis=1)
        out[:, j] = (v ^ (1 << (nb - 1))) - (1 << (nb - 1))
        pos += nb
    return out[:nblk].astype(np.int16)
