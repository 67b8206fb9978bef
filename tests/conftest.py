import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


def load_golden(name):
    """Golden fixtures are plain arrays: never unpickle anything."""
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden_transform():
    return load_golden("transform_cases.npz")


@pytest.fixture(scope="session")
def golden_rle():
    return load_golden("rle_cases.npz")


@pytest.fixture(scope="session")
def golden_codec():
    return load_golden("codec_cases.npz")


@pytest.fixture(scope="session")
def golden_tables():
    return load_golden("tables.npz")


@pytest.fixture(scope="session")
def golden_lenna():
    return load_golden("lenna.npz")
