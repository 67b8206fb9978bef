"""HIC container (mirrors hiccup/hicimage.py:14-183), JPEG flavour.

Host-side "next" row: the payload list jpeg_encode
returns.  Byte format = the reference's: a Huffman table (PayloadStringP) is a
pickle of {"type": <the payload CLASS>, "data": [...]} whose class reference reads
``hiccup.hicimage.TupP`` (hicimage.py:117-121), so files written here load in the
reference and the reference's files load here (pinned byte-for-byte by
tests/golden/hicimage_cases.npz).  Loading never runs arbitrary pickles: a
restricted unpickler admits only the three payload classes (as the reference
names them, or by this module's name) and numpy's scalar reconstruction (the
reference's DC tables hold numpy integers).
"""
import io as _bio
import pickle

import numpy as np

from . import iohelper as io
from . import model, utils

_REF_MODULE = "hiccup.hicimage"  # the module the reference's pickles name


class _SafeUnpickler(pickle.Unpickler):
    _NUMPY = {("numpy._core.multiarray", "scalar"), ("numpy.core.multiarray", "scalar"), ("numpy", "dtype")}

    def find_class(self, module, name):
        if module in (_REF_MODULE, __name__) and name in _PAYLOAD_TYPES:
            return _PAYLOAD_TYPES[name]
        if (module, name) in self._NUMPY:
            return super().find_class(module, name)
        raise pickle.UnpicklingError("refusing to load %s.%s from a HIC file" % (module, name))


def _loads(b):
    return _SafeUnpickler(_bio.BytesIO(bytes(b))).load()


class _RefPickler(pickle._Pickler):
    """Writes this module's payload classes as the reference names them."""

    def save_global(self, obj, name=None):
        if isinstance(obj, type) and _PAYLOAD_TYPES.get(obj.__name__) is obj:
            self.save(_REF_MODULE)
            self.save(obj.__name__)
            self.write(pickle.STACK_GLOBAL)
            self.memoize(obj)
            return
        super().save_global(obj, name)


def _dumps(obj):
    f = _bio.BytesIO()
    _RefPickler(f, protocol=pickle.DEFAULT_PROTOCOL).dump(obj)
    return f.getvalue()


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
        t = _loads(b)
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
        """io.padded_bytes_2_bs's bits, kept packed (the '0'/'1' string is made on
        first use of .payload): byte 0 = pad length p, then the body, whose last p
        bits are padding."""
        b = bytes(b)
        if len(b) == 0:  # padded_bytes_2_bs indexes byte 0
            raise IndexError("index out of range")
        n = io.padded_bits_length(len(b), b[0])
        body = np.zeros(-(-n // 8), dtype=np.uint8)  # bits past the body are zero
        m = min(body.size, len(b) - 1)
        body[:m] = np.frombuffer(b[1:1 + m], dtype=np.uint8)
        return cls.from_packed(body, n)

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

    def packed_bits(self):
        """(uint8 array, nbits): the bits MSB-first, as hic_huffman_decode reads them."""
        if self._packed is None:
            bits = np.frombuffer(self._payload.encode("ascii"), dtype=np.uint8) - ord("0")
            return np.packbits(bits), bits.size
        return self._packed, self._nbits

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
            if padding != 8:  # the pad bits are zero (bytes read from a file may carry others)
                body = body.copy()
                body[-1] &= (0xFF << padding) & 0xFF
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

    @classmethod
    def from_bytes(cls, b):
        d = _loads(b)
        t = d["type"] if isinstance(d["type"], type) else _PAYLOAD_TYPES[d["type"]]  # (round-1 files: a name)
        return cls(t, [t.from_bytes(x) for x in d["data"]])

    def __init__(self, t, payloads):
        self.t = t
        self.payloads = payloads

    def __eq__(self, other):
        return type(self) == type(other) and self.t == other.t and self.payloads == other.payloads

    @property
    def byte_stream(self):
        return _dumps({"type": self.t, "data": [p.byte_stream for p in self.payloads]})


_PAYLOAD_TYPES = {"TupP": TupP, "BitStringP": BitStringP, "PlainStringP": PlainStringP}


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
            raw = _loads(f.read())
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
