"""Bit-string <-> bytes helpers (mirrors hiccup/iohelper.py:20-56) without the
``bitstring`` package (absent from this image).  Same byte format: one leading
byte holding the pad length p (1..8), then the bits, then p zero bits."""


def open_raw_img(path):
    raise NotImplementedError("raw camera images need rawpy (absent); out of scope")


def bin_string(i):
    return bin(i)[2:]


def bin_string_as_bytes(s):
    assert len(s) > 0 and len(s) % 8 == 0
    return int(s, 2).to_bytes(len(s) // 8, "big")


def padded_bs_2_bytes(s):
    padding = 8 - (len(s) % 8)
    bits = s + "0" * padding
    return bytes([padding]) + (int(bits, 2).to_bytes(len(bits) // 8, "big") if bits else b"")


def padded_bits_length(nbytes, pad_byte):
    """How many bits padded_bytes_2_bs keeps of an nbytes-byte buffer whose first
    byte is pad_byte: iohelper.py:51-56 reads it as a SIGNED 8-bit int p, shifts the
    whole buffer left by 8 bits (zero fill) and slices ``bin[:-p-8]`` -- Python
    slice semantics, so p >= -8 drops p + 8 bits from the end while p < -8 keeps
    the first -p - 8.  Bits past the body read as zero."""
    p = pad_byte - 256 if pad_byte >= 128 else pad_byte
    total, stop = 8 * nbytes, -p - 8
    return max(0, total + stop) if stop < 0 else min(stop, total)


def padded_bytes_2_bs(bites):
    bites = bytes(bites)
    body = bites[1:]
    n = padded_bits_length(len(bites), bites[0])
    bits = bin(int.from_bytes(body, "big"))[2:].zfill(8 * len(body)) if body else ""
    return (bits + "0" * 8)[:n]
