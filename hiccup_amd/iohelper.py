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


def padded_bytes_2_bs(bites):
    bites = bytes(bites)
    padding = bites[0]
    body = bites[1:]
    bits = bin(int.from_bytes(body, "big"))[2:].zfill(8 * len(body)) if body else ""
    return bits[:len(bits) - padding]
