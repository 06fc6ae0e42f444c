"""Feature-vector data plane: Hivemall feature strings -> CSR / padded-ELL tensors.

Hivemall feature grammar (reference core/src/main/java/hivemall/model/FeatureValue.java,
hivemall/fm/Feature.java):

* ``"name:value"`` — numeric feature (split at the FIRST ``:``);
* ``"name"``       — value 1.0;
* ``"field:index:value"`` — FFM form;
* features may also be int/bigint arrays (value 1.0).

Integer names are used as indices directly.  Non-integer names are dictionary-encoded
(exact, collision-free, and reversible so model tables carry the original names) or,
with ``-feature_hashing``, hashed with ``mhash``.  Parsing runs in the native host library.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import numpy as np

from .. import _native
from .hashing import DEFAULT_SEED, pack_strings
from .options import UDFArgumentException


@dataclass
class CSR:
    indptr: np.ndarray   # int64 [n+1]
    idx: np.ndarray      # int64 [nnz]
    val: np.ndarray      # float32 [nnz]
    fld: np.ndarray | None = None  # int32 [nnz] (FFM only)

    @property
    def n_rows(self) -> int:
        return len(self.indptr) - 1

    @property
    def nnz(self) -> int:
        return int(self.indptr[-1])

    def row(self, i):
        s, e = self.indptr[i], self.indptr[i + 1]
        return self.idx[s:e], self.val[s:e]

    def max_row_nnz(self) -> int:
        return int(np.diff(self.indptr).max()) if self.n_rows else 0

    def to_ell(self, width: int | None = None, pad_idx: int = -1):
        """Padded-ELL [n, width] (idx int32, val f32, fld int32|None)."""
        n = self.n_rows
        w = width if width is not None else max(1, self.max_row_nnz())
        lens = np.diff(self.indptr)
        if (lens > w).any():
            raise ValueError(f"row nnz {int(lens.max())} exceeds ELL width {w}")
        idx = np.full((n, w), pad_idx, dtype=np.int32)
        val = np.zeros((n, w), dtype=np.float32)
        fld = np.zeros((n, w), dtype=np.int32) if self.fld is not None else None
        rows = np.repeat(np.arange(n), lens)
        cols = np.arange(self.nnz) - np.repeat(self.indptr[:-1], lens)
        idx[rows, cols] = self.idx
        val[rows, cols] = self.val
        if fld is not None:
            fld[rows, cols] = self.fld
        return idx, val, fld

    def to_dense(self, dims: int) -> np.ndarray:
        out = np.zeros((self.n_rows, dims), dtype=np.float32)
        rows = np.repeat(np.arange(self.n_rows), np.diff(self.indptr))
        ok = (self.idx >= 0) & (self.idx < dims)
        np.add.at(out, (rows[ok], self.idx[ok]), self.val[ok])
        return out


def _is_intlike_rows(rows) -> bool:
    for r in rows:
        if r is None:
            continue
        if isinstance(r, np.ndarray):
            return np.issubdtype(r.dtype, np.integer)
        for x in r:
            return isinstance(x, (int, np.integer)) and not isinstance(x, bool)
    return False


class FeatureEncoder:
    """Encodes rows of Hivemall features to integer indices.

    mode: ``"auto"`` (integers as-is, other names dictionary-encoded above ``int_base``),
    ``"int"`` (names must be integers), ``"dict"`` (every name dictionary-encoded),
    ``"hash"`` (``mhash`` into ``num_features``, 1-based like upstream).
    """

    def __init__(self, mode: str = "auto", num_features: int = 1 << 24, int_base: int | None = None,
                 seed: int = DEFAULT_SEED):
        self.mode = mode
        self.num_features = int(num_features)
        self.seed = seed
        self.int_base = int_base
        self._dict = None
        self.saw_strings = False

    # ---------------------------------------------------------------- dictionary
    def _d(self):
        if self._dict is None:
            lib = _native.host()
            self._dict = lib.hm_dict_new()
        return self._dict

    def __del__(self):
        if getattr(self, "_dict", None) is not None:
            try:
                _native.host().hm_dict_free(self._dict)
            except Exception:
                pass
            self._dict = None

    def vocab_size(self) -> int:
        if self._dict is None:
            return 0
        return int(_native.host().hm_dict_size(self._dict))

    def vocab(self) -> list[str]:
        if self._dict is None:
            return []
        lib = _native.host()
        n = self.vocab_size()
        tot = lib.hm_dict_dump(self._dict, None, None)
        buf = np.zeros(max(1, tot), dtype=np.uint8)
        off = np.zeros(n + 1, dtype=np.int64)
        lib.hm_dict_dump(self._dict, buf.ctypes.data, off.ctypes.data)
        b = buf.tobytes()
        return [b[off[i]:off[i + 1]].decode("utf-8") for i in range(n)]

    # ---------------------------------------------------------------- encode
    def _encode_packed(self, b: np.ndarray, off: np.ndarray, indptr: np.ndarray, add_new: bool,
                       shown) -> CSR:
        nnz = int(indptr[-1])
        idx = np.empty(nnz, dtype=np.int64)
        val = np.empty(nnz, dtype=np.float32)
        mode = {"int": 0, "dict": 1, "hash": 2, "auto": 3}[self.mode]
        d = self._d() if mode in (1, 3) else None
        base = self.int_base if self.int_base is not None else self.num_features
        bad = _native.host().hm_parse_features(b.ctypes.data, off.ctypes.data, nnz, mode, d,
                                               1 if add_new else 0, self.num_features, self.seed,
                                               int(base), idx.ctypes.data, val.ctypes.data)
        if bad >= 0:
            raise UDFArgumentException(f"malformed feature: '{shown(bad)}'")
        if mode in (1, 3) and self.vocab_size() > 0:
            self.saw_strings = True
        return CSR(indptr, idx, val)

    def encode(self, rows: Sequence, add_new: bool = True) -> CSR:
        from ..io.ingest import arrow_buffers, is_arrow_like, to_arrow_lists

        if is_arrow_like(rows):
            # Arrow list<string> column: parsed straight from its buffers (no Python object per
            # feature; a SQL feature_hashing / add_bias result arrives this way)
            data, so, lo = arrow_buffers(to_arrow_lists(rows))
            indptr = np.ascontiguousarray(lo, dtype=np.int64)
            if int(indptr[-1]) == 0:
                return CSR(indptr, np.zeros(0, np.int64), np.zeros(0, np.float32))
            b = np.ascontiguousarray(data) if len(data) else np.zeros(1, np.uint8)
            so = np.ascontiguousarray(so, dtype=np.int64)
            return self._encode_packed(b, so, indptr, add_new,
                                       lambda k: bytes(b[so[k]:so[k + 1]]).decode("utf-8", "replace"))
        rows = [([] if r is None else r) for r in rows]
        lens = np.fromiter((len(r) for r in rows), dtype=np.int64, count=len(rows))
        indptr = np.zeros(len(rows) + 1, dtype=np.int64)
        np.cumsum(lens, out=indptr[1:])
        nnz = int(indptr[-1])
        if nnz == 0:
            return CSR(indptr, np.zeros(0, np.int64), np.zeros(0, np.float32))
        if _is_intlike_rows(rows):
            idx = np.concatenate([np.asarray(r, dtype=np.int64) for r in rows if len(r)])
            return CSR(indptr, idx, np.ones(nnz, dtype=np.float32))
        flat = [str(x) for r in rows for x in r]
        buf, off = pack_strings(flat)
        b = np.frombuffer(buf, dtype=np.uint8) if buf else np.zeros(1, np.uint8)
        return self._encode_packed(b, off, indptr, add_new, lambda k: flat[k])

    def decode(self, ids: np.ndarray) -> list:
        """Map indices back to feature names (ints stay ints)."""
        ids = np.asarray(ids)
        if self.mode == "hash" or self._dict is None:
            return [int(i) for i in ids]
        voc = self.vocab()
        base = 0 if self.mode == "dict" else (self.int_base if self.int_base is not None else self.num_features)
        out = []
        for i in ids:
            i = int(i)
            if self.mode == "dict":
                out.append(voc[i] if 0 <= i < len(voc) else i)
            elif i >= base and i - base < len(voc):
                out.append(voc[i - base])
            else:
                out.append(i)
        return out


class _LazyStrings:
    """``flat[k]`` of a packed string buffer (error messages only)."""

    def __init__(self, b, off):
        self.b, self.off = b, off

    def __getitem__(self, k):
        return bytes(self.b[self.off[k]:self.off[k + 1]]).decode("utf-8", "replace")


def parse_ffm_rows(rows: Sequence, num_features: int, num_fields: int, hash_ints: bool = False,
                   seed: int = DEFAULT_SEED) -> CSR:
    """Parse rows of ``field:index[:value]`` strings (FFM input; Python lists or an Arrow
    list<string> column, the latter straight from its buffers)."""
    from ..io.ingest import arrow_buffers, is_arrow_like, to_arrow_lists

    if is_arrow_like(rows):
        data, off, lo = arrow_buffers(to_arrow_lists(rows))
        indptr = np.ascontiguousarray(lo, dtype=np.int64)
        off = np.ascontiguousarray(off, dtype=np.int64)
        b = np.ascontiguousarray(data) if len(data) else np.zeros(1, np.uint8)
        flat = _LazyStrings(b, off)
    else:
        rows = [([] if r is None else r) for r in rows]
        lens = np.fromiter((len(r) for r in rows), dtype=np.int64, count=len(rows))
        indptr = np.zeros(len(rows) + 1, dtype=np.int64)
        np.cumsum(lens, out=indptr[1:])
        flat = None
    nnz = int(indptr[-1])
    fld = np.empty(nnz, dtype=np.int32)
    idx = np.empty(nnz, dtype=np.int32)
    val = np.empty(nnz, dtype=np.float32)
    if nnz:
        if flat is None:
            flat = [str(x) for r in rows for x in r]
            buf, off = pack_strings(flat)
            b = np.frombuffer(buf, dtype=np.uint8) if buf else np.zeros(1, np.uint8)
        bad = _native.host().hm_parse_ffm_features(b.ctypes.data, off.ctypes.data, nnz,
                                                   int(num_features), int(num_fields),
                                                   1 if hash_ints else 0, seed, fld.ctypes.data,
                                                   idx.ctypes.data, val.ctypes.data)
        if bad >= 0:
            raise UDFArgumentException(f"malformed FFM feature: '{flat[bad]}' "
                                       f"(expected field:index[:value], field < {num_fields})")
    return CSR(indptr, idx.astype(np.int64), val, fld)


def parse_feature(s: str) -> tuple[str, float]:
    """Split one ``name[:value]`` feature string (pure Python helper for UDFs)."""
    s = str(s)
    p = s.find(":")
    if p < 0:
        return s, 1.0
    return s[:p], float(s[p + 1:])
