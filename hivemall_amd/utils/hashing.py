"""MurmurHash3 / ``mhash`` (bit-exact with Hivemall's hivemall.utils.hashing.MurmurHash3).

Reference: core/src/main/java/hivemall/utils/hashing/MurmurHash3.java and
core/src/main/java/hivemall/ftvec/hashing/MurmurHash3UDF.java:
MurmurHash3_x86_32 over the UTF-8 bytes, seed 0x9747b28c, ``h % num_features`` with Java
remainder semantics, negatives shifted into range, result starting from 1.

The batch paths run in the native host library (``csrc/host/hashing.cpp``) and, for device
resident string buffers, in the gfx950 kernel ``csrc/kernels/mhash.hip``.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np

DEFAULT_SEED = 0x9747B28C
DEFAULT_NUM_FEATURES = 1 << 24


def pack_strings(strs: Sequence[str]) -> tuple[bytes, np.ndarray]:
    """Concatenate UTF-8 encodings; returns (buffer, int64 offsets of length n+1)."""
    enc = [s.encode("utf-8") if isinstance(s, str) else bytes(s) for s in strs]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        np.cumsum(np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc)), out=off[1:])
    return b"".join(enc), off


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF


def murmurhash3_x86_32_py(data: bytes, seed: int = DEFAULT_SEED) -> int:
    """Pure-Python reference (used by tests to cross-check the native + HIP paths)."""
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h1 = seed & 0xFFFFFFFF
    n = len(data)
    nb = n // 4
    for i in range(nb):
        k1 = int.from_bytes(data[4 * i:4 * i + 4], "little")
        k1 = (k1 * c1) & 0xFFFFFFFF
        k1 = _rotl(k1, 15)
        k1 = (k1 * c2) & 0xFFFFFFFF
        h1 ^= k1
        h1 = _rotl(h1, 13)
        h1 = (h1 * 5 + 0xE6546B64) & 0xFFFFFFFF
    tail = data[4 * nb:]
    k1 = 0
    if len(tail) >= 3:
        k1 ^= tail[2] << 16
    if len(tail) >= 2:
        k1 ^= tail[1] << 8
    if len(tail) >= 1:
        k1 ^= tail[0]
        k1 = (k1 * c1) & 0xFFFFFFFF
        k1 = _rotl(k1, 15)
        k1 = (k1 * c2) & 0xFFFFFFFF
        h1 ^= k1
    h1 ^= n
    h1 ^= h1 >> 16
    h1 = (h1 * 0x85EBCA6B) & 0xFFFFFFFF
    h1 ^= h1 >> 13
    h1 = (h1 * 0xC2B2AE35) & 0xFFFFFFFF
    h1 ^= h1 >> 16
    return h1


def to_signed32(h: int) -> int:
    return h - (1 << 32) if h & 0x80000000 else h


def mhash_reduce(h_unsigned: int, num_features: int) -> int:
    s = to_signed32(h_unsigned)
    r = int(np.fmod(s, num_features))  # Java % truncates toward zero
    if r < 0:
        r += num_features
    return r + 1


def murmurhash3(data: str | bytes, seed: int = DEFAULT_SEED) -> int:
    """Signed 32-bit MurmurHash3_x86_32 of a string's UTF-8 bytes."""
    from .. import _native

    b = data.encode("utf-8") if isinstance(data, str) else data
    buf = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
    return to_signed32(int(_native.host().hm_murmur3(buf.ctypes.data, len(b), seed)))


def mhash(word: str, num_features: int = DEFAULT_NUM_FEATURES, seed: int = DEFAULT_SEED) -> int:
    """``mhash(word [, num_features])`` — murmurhash3 INT value starting from 1."""
    return int(mhash_batch([word], num_features, seed)[0])


def mhash_batch(words: Iterable[str], num_features: int = DEFAULT_NUM_FEATURES,
                seed: int = DEFAULT_SEED) -> np.ndarray:
    from .. import _native

    words = list(words)
    buf, off = pack_strings(words)
    out = np.empty(len(words), dtype=np.int32)
    if words:
        b = np.frombuffer(buf, dtype=np.uint8) if buf else np.zeros(1, np.uint8)
        _native.host().hm_mhash_batch(b.ctypes.data, off.ctypes.data, len(words), seed,
                                      int(num_features), out.ctypes.data)
    return out


def murmur3_batch(words: Iterable[str], seed: int = DEFAULT_SEED) -> np.ndarray:
    from .. import _native

    words = list(words)
    buf, off = pack_strings(words)
    out = np.empty(len(words), dtype=np.uint32)
    if words:
        b = np.frombuffer(buf, dtype=np.uint8) if buf else np.zeros(1, np.uint8)
        _native.host().hm_murmur3_batch(b.ctypes.data, off.ctypes.data, len(words), seed,
                                        out.ctypes.data)
    return out.view(np.int32)


def mhash_device(words: Iterable[str], num_features: int = DEFAULT_NUM_FEATURES,
                 seed: int = DEFAULT_SEED, device="cuda") -> "torch.Tensor":
    """Batched mhash on the GPU (csrc/kernels/hashing.hip): strings are packed on the host,
    copied once, and hashed by the gfx950 kernel (bytes staged in LDS).  ``num_features <= 0``
    returns the raw signed 32-bit hashes.  Bit-exact with :func:`mhash_batch`."""
    import torch

    from .. import _native

    words = list(words)
    buf, off = pack_strings(words)
    dev = torch.device(device)
    out = torch.empty(len(words), dtype=torch.int32, device=dev)
    if not words:
        return out
    b = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy() if buf else np.zeros(16, np.uint8))
    # pad so the kernel's 16-B staging loads never run past the allocation
    b = torch.cat([b, torch.zeros(16, dtype=torch.uint8)]).to(dev)
    o = torch.from_numpy(off.astype(np.int64)).to(dev)
    rc = _native.hip().hm_mhash(_native.ptr(b), _native.ptr(o), len(words), seed, int(num_features),
                                _native.ptr(out), _native.stream_of(dev))
    _native.check(rc, "hm_mhash")
    return out


def _register():
    import ctypes as C

    from .. import _native
    _native.register_hip("hm_mhash", [_native.c_p, _native.c_p, _native.c_i64, C.c_uint32, C.c_int32,
                                      _native.c_p, _native.c_p])


_register()
