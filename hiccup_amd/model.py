"""Enumerations and the CompressedImage container (mirrors hiccup/model.py:9-74)."""
import enum

import numpy as np


class Compression(enum.Enum):
    JPEG = "JPEG"
    HIC = "HIC"


class Coefficient(enum.Enum):
    DC = "DC"
    AC = "AC"


class QTables(enum.Enum):
    JPEG_LUMINANCE = "jpeg standard luminance"
    JPEG_CHROMINANCE = "jpeg standard chrominance"


class Wavelet(enum.Enum):
    DAUBECHIE = "db1"
    HAAR = "haar"
    COIF = "coif1"
    SYM = "sym2"


def table_id(option):
    """QTables -> the C-ABI table id (HIC_TABLE_*)."""
    if option == QTables.JPEG_LUMINANCE:
        return 0
    if option == QTables.JPEG_CHROMINANCE:
        return 1
    raise KeyError(option)


class CompressedImage:
    """Three coefficient planes (model.py:38-74): luminance, red and blue chroma."""

    @classmethod
    def from_dict(cls, d):
        assert len(d) == 3
        return cls(d["lum"], d["cr"], d["cb"])

    def __init__(self, lum, cr, cb):
        self.luminance_component = lum
        self.red_chrominance_component = cr
        self.blue_chrominance_component = cb

    @property
    def shape(self):
        return self.luminance_component.shape, self.red_chrominance_component.shape

    @property
    def as_dict(self):
        return {"lum": self.luminance_component,
                "cr": self.red_chrominance_component,
                "cb": self.blue_chrominance_component}

    def __eq__(self, other):
        if type(self) != type(other):
            return False
        return all(np.array_equiv(a, b) for a, b in zip(
            (self.luminance_component, self.red_chrominance_component, self.blue_chrominance_component),
            (other.luminance_component, other.red_chrominance_component, other.blue_chrominance_component)))
