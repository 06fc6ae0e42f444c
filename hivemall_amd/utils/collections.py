"""Primitive collections (upstream
core/src/main/java/hivemall/utils/collections/{BoundedPriorityQueue,
maps/Int2FloatOpenHashTable,maps/Int2LongOpenHashTable,lists/IntArrayList,
lists/FloatArrayList,lists/DoubleArrayList}.java and utils/lang/HalfFloat.java).

The device engines keep models in dense hashed HBM tables, so these containers serve the host
side (model-table assembly, top-k over candidate streams, fp16 model strings).  The hash
tables are open-addressing with linear probing over numpy arrays (no per-entry objects, like
upstream's "without boxing" tables) and expose vectorised ``get_many`` / ``put_many``
(SIMD-friendly bulk probes) next to the scalar API; capacity is a power of two and grows
at 0.7 load.
"""
from __future__ import annotations

import heapq
from typing import Any, Callable, Iterator

import numpy as np

_EMPTY = np.iinfo(np.int64).min


class BoundedPriorityQueue:
    """Keeps the ``capacity`` largest elements (by ``key``) seen so far; ``offer`` returns
    whether the element was kept (upstream ``BoundedPriorityQueue`` with a natural-order
    comparator).  ``sorted()`` lists them largest first; ties keep insertion order."""

    def __init__(self, capacity: int, key: Callable[[Any], Any] | None = None):
        if capacity <= 0:
            raise ValueError("capacity must be positive")
        self.capacity = int(capacity)
        self.key = key or (lambda x: x)
        self._h: list = []
        self._n = 0

    def offer(self, e) -> bool:
        k = self.key(e)
        self._n += 1
        item = (k, -self._n, e)
        if len(self._h) < self.capacity:
            heapq.heappush(self._h, item)
            return True
        if k > self._h[0][0]:
            heapq.heapreplace(self._h, item)
            return True
        return False

    def peek(self):
        """The smallest kept element (the next one to be evicted)."""
        return self._h[0][2] if self._h else None

    def poll(self):
        return heapq.heappop(self._h)[2] if self._h else None

    def __len__(self):
        return len(self._h)

    def sorted(self) -> list:
        return [e for _, _, e in sorted(self._h, key=lambda t: (t[0], t[1]), reverse=True)]

    def clear(self):
        self._h.clear()


def _mix64(k: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser: spreads sequential keys over the table."""
    with np.errstate(over="ignore"):
        z = k.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


class _OpenHashTable:
    VALUE_DTYPE: Any = np.float32

    def __init__(self, capacity: int = 16, default_value=0):
        cap = 16
        while cap < capacity / 0.7:
            cap <<= 1
        self.keys = np.full(cap, _EMPTY, dtype=np.int64)
        self.vals = np.zeros(cap, dtype=self.VALUE_DTYPE)
        self.size = 0
        self.default_value = default_value

    def _slot(self, key: int) -> int:
        mask = self.keys.size - 1
        i = int(_mix64(np.array([key]))[0]) & mask
        while True:
            k = self.keys[i]
            if k == key or k == _EMPTY:
                return i
            i = (i + 1) & mask

    def _grow(self):
        ok = self.keys != _EMPTY
        ks, vs = self.keys[ok], self.vals[ok]
        self.keys = np.full(self.keys.size * 2, _EMPTY, dtype=np.int64)
        self.vals = np.zeros(self.keys.size, dtype=self.VALUE_DTYPE)
        self.size = 0
        self.put_many(ks, vs)

    def put(self, key: int, value) -> None:
        key = int(key)
        if key == _EMPTY:
            raise ValueError("reserved key")
        i = self._slot(key)
        if self.keys[i] == _EMPTY:
            self.keys[i] = key
            self.size += 1
        self.vals[i] = value
        if self.size > 0.7 * self.keys.size:
            self._grow()

    def get(self, key: int, default=None):
        i = self._slot(int(key))
        if self.keys[i] == _EMPTY:
            return self.default_value if default is None else default
        return self.vals[i].item()

    def __contains__(self, key) -> bool:
        return self.keys[self._slot(int(key))] != _EMPTY

    def __len__(self):
        return self.size

    def _probe(self, keys: np.ndarray, insert: bool) -> np.ndarray:
        """Slot of every key (-1: absent).  The native bulk probe (csrc/host/hashing.cpp
        ``hm_oht_probe``: sequential inserts, OpenMP lookups) when the host library is loaded,
        else vectorised numpy rounds: each resolves the keys whose slot holds them (or is
        empty), the rest advance one slot."""
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        try:
            from .. import _native
            lib = _native.host()
        except Exception:   # noqa: BLE001 - no host library: the numpy rounds below
            lib = None
        if lib is not None and keys.size:
            out = np.empty(keys.size, dtype=np.int64)
            self.size += int(lib.hm_oht_probe(self.keys.ctypes.data, self.keys.size, keys.ctypes.data,
                                              keys.size, out.ctypes.data, int(insert)))
            return out
        return self._probe_np(keys, insert)

    def _probe_np(self, keys: np.ndarray, insert: bool) -> np.ndarray:
        """Duplicate new keys in one batch are inserted once (the first claimant claims the
        slot, the others then find it)."""
        mask = self.keys.size - 1
        pos = (_mix64(keys) & np.uint64(mask)).astype(np.int64)
        out = np.full(keys.size, -1, dtype=np.int64)
        todo = np.arange(keys.size)
        while todo.size:
            p = pos[todo]
            k = self.keys[p]
            hit = k == keys[todo]
            empty = k == _EMPTY
            other = ~hit & ~empty                   # slot owned by another key: advance
            out[todo[hit]] = p[hit]
            done = hit.copy()
            if empty.any():
                ei = np.flatnonzero(empty)
                if insert:
                    # one claimant per empty slot this round; the losers re-probe the slot
                    _, first = np.unique(p[ei], return_index=True)
                    w = ei[first]
                    self.keys[p[w]] = keys[todo[w]]
                    self.size += w.size
                    out[todo[w]] = p[w]
                    done[w] = True
                else:
                    done[ei] = True                 # absent: out stays -1
            adv = todo[other]
            pos[adv] = (pos[adv] + 1) & mask
            todo = todo[~done]
        return out

    def put_many(self, keys, values) -> None:
        keys = np.asarray(keys, dtype=np.int64)
        values = np.broadcast_to(np.asarray(values, dtype=self.VALUE_DTYPE), keys.shape)
        while self.size + keys.size > 0.7 * self.keys.size:
            self._grow()
        slots = self._probe(keys, insert=True)
        self.vals[slots] = values          # last write wins for duplicate keys

    def get_many(self, keys, default=None) -> np.ndarray:
        keys = np.asarray(keys, dtype=np.int64)
        slots = self._probe(keys, insert=False)
        d = self.default_value if default is None else default
        out = np.full(keys.size, d, dtype=self.VALUE_DTYPE)
        ok = slots >= 0
        out[ok] = self.vals[slots[ok]]
        return out

    def items(self) -> Iterator[tuple[int, Any]]:
        ok = np.flatnonzero(self.keys != _EMPTY)
        for i in ok:
            yield int(self.keys[i]), self.vals[i].item()

    def to_arrays(self) -> tuple[np.ndarray, np.ndarray]:
        ok = self.keys != _EMPTY
        order = np.argsort(self.keys[ok], kind="stable")
        return self.keys[ok][order], self.vals[ok][order]


class Int2FloatOpenHashTable(_OpenHashTable):
    VALUE_DTYPE = np.float32


class Int2LongOpenHashTable(_OpenHashTable):
    """Key -> int64 offset (upstream FFM model store: V(feature, field) key -> HeapBuffer
    offset).  Resolves the SQL fused join-predict's integer keys to model rows
    (sql/fused.py ``_join_index``)."""
    VALUE_DTYPE = np.int64

    def get_many(self, keys, default=None) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        d = self.default_value if default is None else default
        try:
            from .. import _native
            lib = _native.host()
        except Exception:   # noqa: BLE001 - no host library: the generic path
            lib = None
        if lib is None or not keys.size:
            return super().get_many(keys, default)
        out = np.empty(keys.size, dtype=np.int64)
        lib.hm_oht_get_i64(self.keys.ctypes.data, self.vals.ctypes.data, self.keys.size, keys.ctypes.data,
                           keys.size, int(d), out.ctypes.data)
        return out


class Long2DoubleOpenHashTable(_OpenHashTable):
    VALUE_DTYPE = np.float64


# ------------------------------------------------------------------------------ HalfFloat
def float_to_half_bits(x, rounding: str = "nearest") -> np.ndarray:
    """IEEE binary16 bit patterns (uint16) of ``x`` (upstream ``HalfFloat.floatToHalfFloat``).
    ``rounding="nearest"`` is round-to-nearest-even; ``"truncate"`` drops the low mantissa
    bits (the table-driven conversion).  Which one upstream's tables implement is parity
    unpinned (no upstream fixture offline); both keep |x| <= 65504 finite."""
    a = np.asarray(x, dtype=np.float32)
    if rounding == "nearest":
        return a.astype(np.float16).view(np.uint16)
    if rounding != "truncate":
        raise ValueError(rounding)
    b = a.view(np.uint32).astype(np.uint64)
    sign = ((b >> 16) & 0x8000).astype(np.uint16)
    exp = ((b >> 23) & 0xFF).astype(np.int64) - 127 + 15
    man = (b & 0x7FFFFF).astype(np.uint64)
    out = np.zeros(a.shape, dtype=np.uint16)
    nan = np.isnan(a)
    inf = np.isinf(a) | (~nan & (exp >= 31))
    norm = ~nan & ~inf & (exp > 0)
    sub = ~nan & ~inf & (exp <= 0) & (exp > -11)
    out[norm] = ((exp[norm].astype(np.uint64) << 10) | (man[norm] >> 13)).astype(np.uint16)
    m = man[sub] | 0x800000
    sh = (14 - exp[sub]).astype(np.uint64)
    out[sub] = (m >> sh).astype(np.uint16)
    out[inf] = 0x7C00
    out[nan] = 0x7E00
    return out | sign


def half_bits_to_float(h) -> np.ndarray:
    """uint16 binary16 bit patterns -> float32 (``HalfFloat.halfFloatToFloat``, exact)."""
    return np.asarray(h, dtype=np.uint16).view(np.float16).astype(np.float32)


HALF_FLOAT_MAX = 65504.0


def is_representable_as_half(x: float) -> bool:
    """``HalfFloat.isRepresentable``: finite and within ±65504."""
    return bool(np.isfinite(x) and abs(x) <= HALF_FLOAT_MAX)
