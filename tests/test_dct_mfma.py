"""The integer-MFMA forward DCT (k_dct_mfma), pinned on the CPU.

tools/check/dct_mfma.py holds the constant matrices, the exactness proof and a
bit-level numpy emulation of the kernel's integer arithmetic (digit products,
the two truncating shifts, R >> 19, the flag test).  These tests
  * re-run the proof and diff the generated header (dct_mfma_tables.h);
  * run the emulation against the oracle (the reference's pocketfft restatement,
    pinned to golden vectors by test_oracle_golden.py): every unflagged
    coefficient equals the reference's, the DC comes back as the exact pixel sum,
    and the luminance (4,4) slot is flagged exactly at its ties.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools", "check"))
sys.path.insert(0, REPO)
import dct_mfma as M  # noqa: E402
from oracle import oracle as O  # noqa: E402

HEADER = os.path.join(REPO, "hiccup_amd", "csrc", "dct_mfma_tables.h")


def test_header_matches_proof(tmp_path):
    out = tmp_path / "h.h"
    M.emit(str(out))
    assert out.read_text() == open(HEADER).read(), \
        "dct_mfma_tables.h differs from tools/check/dct_mfma.py --emit: regenerate it"


def test_window_covers_bound():
    o, L, m = M.windows()
    assert m < 0.5 + 1e-3            # EA + EQ below one half R unit (2^-20)
    assert o - 1 > m and L - o > m   # both sides of the flag window
    assert L <= 4                    # flags stay rare (~L 2^-19 per slot)
    M.bounds_ok()                    # int32 accumulators and R


def test_limbs_roundtrip():
    for t in range(2):
        A, _ = M.amatrix(t)
        for z in range(64):
            for a in A[z]:
                d = M.limbs(a)
                assert all(-128 <= x <= 127 for x in d)
                assert sum(x << (8 * k) for k, x in enumerate(d)) == a


def _blocks(kind, n, rng):
    if kind == "random":
        return rng.integers(0, 256, (n, 8, 8))
    if kind == "constant":
        return np.repeat(rng.integers(0, 256, (n, 1, 1)), 64).reshape(n, 8, 8)
    if kind == "levels":
        return rng.choice([0, 64, 128, 192, 255], (n, 8, 8))
    if kind == "extreme":
        return rng.choice([0, 255], (n, 8, 8))
    if kind == "ramp":
        i, j = np.meshgrid(np.arange(8), np.arange(8), indexing="ij")
        a, b, c = (rng.integers(-16, 17, (n, 1, 1)) for _ in range(3))
        return np.clip(a * i + b * j + 128 + c, 0, 255)
    raise ValueError(kind)


@pytest.mark.parametrize("table", [0, 1])
@pytest.mark.parametrize("kind", ["random", "constant", "levels", "extreme", "ramp"])
def test_emulation_matches_oracle(table, kind):
    rng = np.random.default_rng(11 + table * 7 + len(kind))
    n = 20000
    p = _blocks(kind, n, rng)
    x = (p - 128).reshape(n, 64)
    o, L, _ = M.windows()
    q, fr, R = M.emulate(x, table, int(round(o * 2 ** 13)))
    ref = np.round(O.dct2((p - 128).astype(np.float64)) / O.TABLES[table]).astype(np.int64).reshape(n, 64)[:, M.ZZ]
    X = (R[:, 0] - (1 << 18)) >> 17
    assert np.array_equal(X, x.sum(1)), "DC row must return the exact pixel sum"
    q[:, 0] = M.dc_quant(X, int(O.TABLES[table][0, 0]))
    assert np.array_equal(q[:, 0], ref[:, 0])
    flag = fr < L
    flag[:, 0] = False
    if table == 0:
        # (4,4) luminance: y/T = K/34, flagged exactly at a tie
        y44 = O.dct2((p - 128).astype(np.float64))[:, 4, 4] / 68.0
        tie = np.abs(np.abs(y44 - np.floor(y44)) - 0.5) < 1e-9
        assert np.array_equal(flag[:, M.Z44], tie)
    bad = (q != ref) & ~flag
    assert not bad.any(), "unflagged mismatch at slots %s" % np.nonzero(bad.any(0))[0]
    other = flag.copy()
    if table == 0:
        other[:, M.Z44] = False
    if kind == "random":
        assert other.any(1).mean() < 2e-3   # ~62 * 3 * 2^-19 per block
