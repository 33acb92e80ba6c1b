"""Helpers to turn golden records back into images / key lists (tests only)."""
import numpy as np


def keys_of(golden_lib, name):
    return [bytes.fromhex(h) for h in golden_lib["key_sets"][name]]


def image_of(rec):
    """Rebuild a serialized image from {header_hex, image_len, bits}."""
    img = bytearray(rec["image_len"])
    hdr = bytes.fromhex(rec["header_hex"])
    img[:len(hdr)] = hdr
    if rec["image_len"] > 28 and rec["bits"]:
        bits = np.zeros((rec["image_len"] - 28) * 8, dtype=np.uint8)
        bits[np.asarray(rec["bits"], dtype=np.int64)] = 1
        img[28:] = np.packbits(bits, bitorder="little").tobytes()
    return bytes(img)


def words_of_bits(m, bits):
    w = np.zeros(max((m + 63) // 64, 1), dtype=np.uint64)
    if bits:
        b = np.asarray(bits, dtype=np.uint64)
        np.bitwise_or.at(w, (b >> np.uint64(6)).astype(np.int64), np.uint64(1) << (b & np.uint64(63)))
    return w


def pack(keys):
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        offs[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
    buf = np.frombuffer(b"".join(keys) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, offs
