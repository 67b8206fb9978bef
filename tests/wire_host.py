"""Host restatement of the gather's wire format (hiccup_amd/csrc/wire.hip), for the
CPU gloo tests of the stream gather.  Test infrastructure: the GPU kernels are
pinned to it by tests/test_gpu_codec.py::test_wire_pack_unpack."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "check"))
import wire_widths  # noqa: E402

WIDTHS = [wire_widths.widths(wire_widths.LUM), wire_widths.widths(wire_widths.CHROMA)]
TABLE_OF = {"lum": 0, "cr": 1, "cb": 1}


def block_bits(table):
    return sum(WIDTHS[table])


def tile_bytes(table):
    return -(-2 * block_bits(table) // 4) * 4 * 4  # 2 * bits words, rounded up to 4 words


def wire_bytes(nblk, table):
    return 0 if nblk <= 0 else -(-nblk // 64) * tile_bytes(table)


def pack(blocks, table):
    """(n, 64) int16 zig-zag blocks -> uint8 wire bytes (LSB-first bit stream per tile)."""
    blocks = np.asarray(blocks, dtype=np.int16)
    n = blocks.shape[0]
    nt = -(-n // 64)
    full = np.zeros((nt * 64, 64), np.int64)
    full[:n] = blocks
    bits = []
    for j, nb in enumerate(WIDTHS[table]):
        col = full[:, j]
        if np.any(col < -(1 << (nb - 1))) or np.any(col >= (1 << (nb - 1))):
            raise ValueError("slot %d value outside %d bits" % (j, nb))
        bits.append(((col[:, None] & ((1 << nb) - 1)) >> np.arange(nb)) & 1)
    bb = block_bits(table)
    stream = np.concatenate(bits, axis=1).reshape(nt, 64 * bb).astype(np.uint8)
    tiles = np.zeros((nt, tile_bytes(table) * 8), np.uint8)
    tiles[:, :64 * bb] = stream
    return np.packbits(tiles, axis=1, bitorder="little").reshape(-1)


def unpack(wire, nblk, table):
    """The inverse: wire bytes -> (nblk, 64) int16 blocks."""
    nt = -(-nblk // 64)
    tb, bb = tile_bytes(table), block_bits(table)
    bits = np.unpackbits(np.asarray(wire, np.uint8)[:nt * tb].reshape(nt, tb), axis=1,
                         bitorder="little")[:, :64 * bb].reshape(nt * 64, bb).astype(np.int64)
    out = np.zeros((nt * 64, 64), np.int64)
    pos = 0
    for j, nb in enumerate(WIDTHS[table]):
        v = (bits[:, pos:pos + nb] << np.arange(nb)).sum(axis=1)
        out[:, j] = (v ^ (1 << (nb - 1))) - (1 << (nb - 1))
        pos += nb
    return out[:nblk].astype(np.int16)


def random_blocks(rng, n, table):
    """Blocks with every slot anywhere in its width's range (half zeros)."""
    w = np.array(WIDTHS[table])
    lo, hi = -(1 << (w - 1)), (1 << (w - 1))
    b = (rng.random((n, 64)) * (hi - lo) + lo).astype(np.int64)
    b[rng.random((n, 64)) < 0.5] = 0
    return b.astype(np.int16)
