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


def tile_records(zz, per, M=15, base_blk=0):
    """Host restatement of the RLE tile records (rle_core.h tile_record16 /
    tile_record16_half): (n, 64) zig-zag blocks -> int64 [ceil(n / per), 3] with
    `per` blocks per record (64: full tiles, 32: the fused kernel's chroma half
    tiles); AC element j of block b sits at stream position (base_blk + b) * 63 + j.
      [0] position of the record's first nonzero AC (-1: none)
      [1] position of its last nonzero AC (-1: none)
      [2] symbols of every nonzero but the first: 1 + run // M each, runs counted
          across the record's blocks (codec.py:55-99 splits runs >= M)."""
    zz = np.asarray(zz)
    n = zz.shape[0]
    nrec = -(-n // per)
    out = np.zeros((nrec, 3), np.int64)
    for r in range(nrec):
        pos = np.flatnonzero(zz[r * per:(r + 1) * per, 1:].reshape(-1) != 0)
        if len(pos) == 0:
            out[r] = (-1, -1, 0)
            continue
        g0 = (base_blk + r * per) * 63
        gaps = np.diff(pos) - 1
        out[r] = (g0 + pos[0], g0 + pos[-1], len(gaps) + int((gaps // M).sum()))
    return out


def rebase(rec, shift):
    """hic_rle_records_rebase: positions (>= 0) moved by `shift`, counts kept."""
    out = rec.copy()
    for c in (0, 1):
        out[:, c] = np.where(rec[:, c] >= 0, rec[:, c] + shift, rec[:, c])
    return out
