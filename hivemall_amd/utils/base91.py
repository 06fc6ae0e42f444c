"""basE91 codec (Joachim Henke's algorithm; Hivemall hivemall.utils.codec.Base91, used to
ship tree models as printable strings: Deflate -> Base91)."""
from __future__ import annotations

_ENC = ('ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789'
        '!#$%&()*+,./:;<=>?@[]^_`{|}~"')
_DEC = {c: i for i, c in enumerate(_ENC)}


def encode(data: bytes) -> str:
    b = n = 0
    out = []
    for byte in data:
        b |= byte << n
        n += 8
        if n > 13:
            v = b & 8191
            if v > 88:
                b >>= 13
                n -= 13
            else:
                v = b & 16383
                b >>= 14
                n -= 14
            out.append(_ENC[v % 91])
            out.append(_ENC[v // 91])
    if n:
        out.append(_ENC[b % 91])
        if n > 7 or b > 90:
            out.append(_ENC[b // 91])
    return "".join(out)


def decode(s: str) -> bytes:
    v = -1
    b = n = 0
    out = bytearray()
    for ch in s:
        if ch not in _DEC:
            continue
        c = _DEC[ch]
        if v < 0:
            v = c
        else:
            v += c * 91
            b |= v << n
            n += 13 if (v & 8191) > 88 else 14
            while n > 7:
                out.append(b & 255)
                b >>= 8
                n -= 8
            v = -1
    if v + 1:
        out.append((b | v << n) & 255)
    return bytes(out)
