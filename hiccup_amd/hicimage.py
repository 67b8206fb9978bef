"""HIC container (mirrors hiccup/hicimage.py:14-183), JPEG flavour.

Host-side "next" row: the payload list jpeg_encode
returns.  Serialisation uses pickle of plain tuples/bytes of THIS package's own
objects only (never loads foreign files with anything but this format).
"""
import pickle

import numpy as np

from . import iohelper as io
from . import model, utils


class Payload:
    @classmethod
    def from_bytes(cls, b):
        raise NotImplementedError

    @property
    def byte_stream(self):
        raise NotImplementedError


class TupP(Payload):
    """A pair: a shape, or one Huffman table entry (value, code)."""

    @classmethod
    def from_bytes(cls, b):
        t = pickle.loads(b)
        return cls(t[0], t[1])

    def __init__(self, n1, n2):
        self.n1 = n1
        self.n2 = n2

    def __eq__(self, other):
        return type(self) == type(other) and self.n1 == other.n1 and self.n2 == other.n2

    @property
    def numbers(self):
        return self.n1, self.n2

    @property
    def byte_stream(self):
        return pickle.dumps((self.n1, self.n2))


class BitStringP(Payload):
    """Huffman-coded data as a '0'/'1' string, stored byte-padded.  A stream packed
    on the GPU (from_packed) keeps its bytes; the string is made on first use."""

    @classmethod
    def from_bytes(cls, b):
        return cls(io.padded_bytes_2_bs(b))

    @classmethod
    def from_packed(cls, packed, nbits):
        """packed: uint8 array, nbits bits MSB-first (hic_huffman_pack's output)."""
        obj = cls(None)
        obj._packed, obj._nbits = np.asarray(packed, dtype=np.uint8), int(nbits)
        return obj

    def __init__(self, string):
        self._payload = string
        self._packed = None
        self._nbits = None

    @property
    def payload(self):
        if self._payload is None:
            bits = np.unpackbits(self._packed[:-(-self._nbits // 8)])[:self._nbits]
            self._payload = (bits + ord("0")).astype(np.uint8).tobytes().decode("ascii")
        return self._payload

    def __eq__(self, other):
        return type(self) == type(other) and self.payload == other.payload

    @property
    def byte_stream(self):
        if self._payload is None:  # io.padded_bs_2_bytes on the packed bits
            padding = 8 - self._nbits % 8
            body = self._packed[:self._nbits // 8 + 1] if self._nbits % 8 else self._packed[:self._nbits // 8]
            body = np.concatenate([body, np.zeros(1 if padding == 8 else 0, np.uint8)])
            return bytes([padding]) + body.tobytes()
        return io.padded_bs_2_bytes(self.payload)


class PlainStringP(Payload):
    ENCODING = "ascii"

    @classmethod
    def from_bytes(cls, b):
        return cls(b.decode(cls.ENCODING))

    def __init__(self, string):
        self.payload = string

    def __eq__(self, other):
        return type(self) == type(other) and self.payload == other.payload

    @property
    def byte_stream(self):
        return self.payload.encode(encoding=self.ENCODING)


class PayloadStringP(Payload):
    """A group of payloads of one type (a Huffman table)."""

    _TYPES = {"TupP": TupP, "BitStringP": BitStringP, "PlainStringP": PlainStringP}

    @classmethod
    def from_bytes(cls, b):
        d = pickle.loads(b)
        t = cls._TYPES[d["type"]]
        return cls(t, [t.from_bytes(x) for x in d["data"]])

    def __init__(self, t, payloads):
        self.t = t
        self.payloads = payloads

    def __eq__(self, other):
        return type(self) == type(other) and self.t == other.t and self.payloads == other.payloads

    @property
    def byte_stream(self):
        return pickle.dumps({"type": self.t.__name__, "data": [p.byte_stream for p in self.payloads]})


class HicImage:
    @classmethod
    def from_bytes(cls, raw_data):
        t = model.Compression(PlainStringP.from_bytes(raw_data[0]).payload)
        if t != model.Compression.JPEG:
            raise NotImplementedError("the wavelet (HIC) scheme is out of scope")
        huffs = [PayloadStringP.from_bytes(b) for b in raw_data[1:10]]
        data = [BitStringP.from_bytes(b) for b in raw_data[10:19]]
        shapes = [TupP.from_bytes(b) for b in raw_data[19:21]]
        return cls.jpeg_image(huffs + data + shapes)

    @classmethod
    def jpeg_image(cls, payloads):
        return cls(model.Compression.JPEG, [PlainStringP(model.Compression.JPEG.value)], payloads)

    @classmethod
    def wavelet_image(cls, payloads):
        raise NotImplementedError("the wavelet (HIC) scheme is out of scope")

    @classmethod
    def from_file(cls, path):
        with open(path, "rb") as f:
            raw = pickle.load(f)
        assert raw is not None
        return cls.from_bytes(raw)

    def __init__(self, hic_type, settings, payloads):
        self.hic_type = hic_type
        self.settings = settings
        self._payloads = payloads

    def write_file(self, path):
        utils.debug_msg("Writing HIC file to: " + path)
        with open(path, "wb") as f:
            pickle.dump(self.byte_stream(), f)

    @property
    def payloads(self):
        return self._payloads

    def byte_stream(self):
        return [p.byte_stream for p in self.settings + self.payloads]
