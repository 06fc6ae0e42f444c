"""Integer codecs of Hivemall's ``utils/codec`` package (upstream
core/src/main/java/hivemall/utils/codec/{VariableByteCodec,ZigZagLEB128Codec,DeflateCodec}.java).

* VariableByte = unsigned LEB128: 7 value bits per byte, least significant group first, the
  high bit set on every byte but the last.
* ZigZag LEB128 = signed integers mapped to unsigned by zigzag (0, -1, 1, -2, ... -> 0, 1, 2,
  3, ...) and then VariableByte-encoded; small magnitudes of either sign take one byte.
* Deflate = zlib stream (``deflate`` / ``inflate`` SQL functions in ``tools``), used with
  Base91 (``utils/base91.py``) for model strings.

Vectorised over numpy arrays; scalar helpers round-trip one value.
"""
from __future__ import annotations

import zlib

import numpy as np


def zigzag_encode(v: np.ndarray | int, bits: int = 64):
    """Signed -> unsigned zigzag mapping for ``bits``-wide integers."""
    if isinstance(v, (int, np.integer)):
        v = int(v)
        return ((v << 1) ^ (v >> (bits - 1))) & ((1 << bits) - 1)
    a = np.asarray(v, dtype=np.int64)
    return ((a << 1) ^ (a >> 63)).view(np.uint64)


def zigzag_decode(u: np.ndarray | int):
    if isinstance(u, (int, np.integer)):
        u = int(u)
        return (u >> 1) ^ -(u & 1)
    a = np.asarray(u, dtype=np.uint64)
    return ((a >> np.uint64(1)).astype(np.int64)) ^ (-(a & np.uint64(1)).astype(np.int64))


def vbyte_encode(values) -> bytes:
    """Unsigned LEB128 of a sequence of non-negative integers (< 2^64)."""
    out = bytearray()
    for v in np.asarray(values, dtype=np.uint64).tolist():
        if v < 0:
            raise ValueError("vbyte_encode: negative value (use zigzag_leb128_encode)")
        while v >= 0x80:
            out.append((v & 0x7F) | 0x80)
            v >>= 7
        out.append(v)
    return bytes(out)


def vbyte_decode(data: bytes, count: int | None = None) -> np.ndarray:
    """Decode ``count`` values (all when None) from unsigned LEB128 bytes."""
    vals = []
    cur = shift = 0
    for b in data:
        cur |= (b & 0x7F) << shift
        if b & 0x80:
            shift += 7
            if shift > 63:
                raise ValueError("vbyte_decode: value wider than 64 bits")
        else:
            vals.append(cur)
            cur = shift = 0
            if count is not None and len(vals) == count:
                break
    if shift:
        raise ValueError("vbyte_decode: truncated input")
    return np.array(vals, dtype=np.uint64)


def zigzag_leb128_encode(values) -> bytes:
    return vbyte_encode(zigzag_encode(np.asarray(values, dtype=np.int64)))


def zigzag_leb128_decode(data: bytes, count: int | None = None) -> np.ndarray:
    return zigzag_decode(vbyte_decode(data, count))


def deflate_codec(data: bytes, level: int = -1) -> bytes:
    return zlib.compress(data, level)


def inflate_codec(data: bytes) -> bytes:
    return zlib.decompress(data)
