"""Training-matrix containers and matrix builders (upstream
core/src/main/java/hivemall/math/matrix/{Matrix,DenseMatrix2d,RowMajorDenseMatrix2d,
ColumnMajorDenseMatrix2d,CSRMatrix,CSCMatrix,DoKMatrix}.java and
math/matrix/builders/{MatrixBuilder,RowMajorDenseMatrixBuilder,ColumnMajorDenseMatrixBuilder,
CSRMatrixBuilder,CSCMatrixBuilder,DoKMatrixBuilder}.java).

Upstream learners that need the whole training set (RF, GBT, SLIM) buffer rows into a
``MatrixBuilder`` in ``process()`` and hand the built ``Matrix`` to the algorithm in
``close()``.  Here the containers are numpy-backed on the host and move to the device in one
copy (``to_torch``):

* ``CSRMatrix``   row access (online learners, SpMV ``X @ w``);
* ``CSCMatrix``   column access (coordinate descent, SLIM);
* ``DoKMatrix``   incremental assembly by (row, col) key;
* ``DenseMatrix2d`` row- or column-major dense storage (the tree engines read column-major
  bins, so ``row_major=False`` is the layout they consume without a transpose).

Rows are fed to a builder as Hivemall feature strings (``"i:v"``, bare ``"i"`` = 1.0), as
``(index, value)`` pairs, or as a dense list of floats.  Duplicate (row, col) entries are
summed, as upstream's builders do.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

from typing import Iterable, Sequence

import numpy as np


class Matrix(ABC):
    """Common read interface (upstream ``hivemall.math.matrix.Matrix``)."""

    n_rows: int
    n_cols: int

    @property
    def shape(self) -> tuple[int, int]:
        return (self.n_rows, self.n_cols)

    @abstractmethod
    def nnz(self) -> int:
        ...

    @abstractmethod
    def get(self, i: int, j: int, default: float = 0.0) -> float:
        ...

    @abstractmethod
    def row(self, i: int) -> tuple[np.ndarray, np.ndarray]:
        """(column indices, values) of the non-zeros of row ``i``."""
        ...

    @abstractmethod
    def to_dense(self) -> np.ndarray:
        ...

    @abstractmethod
    def matvec(self, x: np.ndarray) -> np.ndarray:
        ...

    @abstractmethod
    def to_csr(self) -> "CSRMatrix":
        ...

    def to_torch(self, device=None, dtype=None):
        """Dense tensor (dense layouts) or ``torch.sparse_csr_tensor`` (sparse layouts)."""
        import torch

        c = self.to_csr()
        dt = dtype or torch.float32
        return torch.sparse_csr_tensor(torch.from_numpy(c.indptr), torch.from_numpy(c.indices),
                                       torch.from_numpy(c.values).to(dt), size=self.shape,
                                       device=device)


class DenseMatrix2d(Matrix):
    """Dense matrix, row-major (``RowMajorDenseMatrix2d``) or column-major
    (``ColumnMajorDenseMatrix2d``)."""

    def __init__(self, data, row_major: bool = True, dtype=np.float64):
        a = np.asarray(data, dtype=dtype)
        if a.ndim != 2:
            raise ValueError("DenseMatrix2d needs a 2-D array")
        self.row_major = row_major
        self.data = np.ascontiguousarray(a) if row_major else np.asfortranarray(a)
        self.n_rows, self.n_cols = a.shape

    def nnz(self) -> int:
        return int(np.count_nonzero(self.data))

    def get(self, i, j, default=0.0):
        if not (0 <= i < self.n_rows and 0 <= j < self.n_cols):
            return default
        return float(self.data[i, j])

    def row(self, i):
        r = self.data[i]
        nz = np.flatnonzero(r)
        return nz, r[nz]

    def column(self, j) -> np.ndarray:
        return self.data[:, j]

    def to_dense(self):
        return np.array(self.data)

    def matvec(self, x):
        return self.data @ np.asarray(x, dtype=self.data.dtype)

    def to_csr(self):
        return CSRMatrix.from_dense(self.data)

    def to_torch(self, device=None, dtype=None):
        import torch

        t = torch.from_numpy(np.ascontiguousarray(self.data))
        return t.to(device=device, dtype=dtype or torch.float32)


def _coo_to_compressed(major: np.ndarray, minor: np.ndarray, vals: np.ndarray, n_major: int):
    """Sort (major, minor), sum duplicates, and return (indptr, minor, vals)."""
    order = np.lexsort((minor, major))
    major, minor, vals = major[order], minor[order], vals[order]
    if len(major):
        new = np.ones(len(major), dtype=bool)
        new[1:] = (major[1:] != major[:-1]) | (minor[1:] != minor[:-1])
        starts = np.flatnonzero(new)
        vals = np.add.reduceat(vals, starts)
        major, minor = major[starts], minor[starts]
    indptr = np.zeros(n_major + 1, dtype=np.int64)
    np.cumsum(np.bincount(major, minlength=n_major), out=indptr[1:])
    return indptr, minor.astype(np.int32), vals


class CSRMatrix(Matrix):
    """Compressed sparse rows (upstream ``CSRMatrix``: rowPointers, columnIndices, values)."""

    def __init__(self, indptr, indices, values, n_cols: int):
        self.indptr = np.asarray(indptr, dtype=np.int64)
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)
        self.n_rows = len(self.indptr) - 1
        self.n_cols = int(n_cols)
        if self.indptr[-1] != len(self.indices) or len(self.indices) != len(self.values):
            raise ValueError("CSRMatrix: indptr / indices / values lengths disagree")
        if len(self.indices) and (self.indices.min() < 0 or self.indices.max() >= self.n_cols):
            raise ValueError("CSRMatrix: column index out of range")

    @classmethod
    def from_coo(cls, rows, cols, vals, shape):
        indptr, ind, v = _coo_to_compressed(np.asarray(rows, np.int64), np.asarray(cols, np.int64),
                                            np.asarray(vals, np.float64), shape[0])
        return cls(indptr, ind, v, shape[1])

    @classmethod
    def from_dense(cls, a):
        a = np.asarray(a)
        r, c = np.nonzero(a)
        return cls.from_coo(r, c, a[r, c], a.shape)

    def nnz(self):
        return int(self.indptr[-1])

    def row_ids(self) -> np.ndarray:
        return np.repeat(np.arange(self.n_rows, dtype=np.int64), np.diff(self.indptr))

    def row(self, i):
        s, e = self.indptr[i], self.indptr[i + 1]
        return self.indices[s:e], self.values[s:e]

    def get(self, i, j, default=0.0):
        if not (0 <= i < self.n_rows):
            return default
        cols, vals = self.row(i)
        k = np.searchsorted(cols, j)
        return float(vals[k]) if k < len(cols) and cols[k] == j else default

    def to_dense(self):
        out = np.zeros(self.shape, dtype=self.values.dtype)
        out[self.row_ids(), self.indices] = self.values
        return out

    def matvec(self, x):
        x = np.asarray(x, dtype=np.float64)
        return np.bincount(self.row_ids(), weights=self.values * x[self.indices],
                           minlength=self.n_rows)

    def to_csr(self):
        return self

    def to_csc(self) -> "CSCMatrix":
        indptr, ind, v = _coo_to_compressed(self.indices.astype(np.int64), self.row_ids(),
                                            self.values, self.n_cols)
        return CSCMatrix(indptr, ind, v, self.n_rows)


class CSCMatrix(Matrix):
    """Compressed sparse columns (upstream ``CSCMatrix``)."""

    def __init__(self, indptr, indices, values, n_rows: int):
        self.indptr = np.asarray(indptr, dtype=np.int64)
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)
        self.n_cols = len(self.indptr) - 1
        self.n_rows = int(n_rows)
        if self.indptr[-1] != len(self.indices) or len(self.indices) != len(self.values):
            raise ValueError("CSCMatrix: indptr / indices / values lengths disagree")

    def nnz(self):
        return int(self.indptr[-1])

    def col_ids(self) -> np.ndarray:
        return np.repeat(np.arange(self.n_cols, dtype=np.int64), np.diff(self.indptr))

    def column(self, j) -> tuple[np.ndarray, np.ndarray]:
        s, e = self.indptr[j], self.indptr[j + 1]
        return self.indices[s:e], self.values[s:e]

    def row(self, i):
        hit = self.indices == i
        return self.col_ids()[hit].astype(np.int32), self.values[hit]

    def get(self, i, j, default=0.0):
        if not (0 <= j < self.n_cols):
            return default
        rows, vals = self.column(j)
        k = np.searchsorted(rows, i)
        return float(vals[k]) if k < len(rows) and rows[k] == i else default

    def to_dense(self):
        out = np.zeros(self.shape, dtype=self.values.dtype)
        out[self.indices, self.col_ids()] = self.values
        return out

    def matvec(self, x):
        x = np.asarray(x, dtype=np.float64)
        return np.bincount(self.indices, weights=self.values * x[self.col_ids()],
                           minlength=self.n_rows)

    def to_csr(self):
        indptr, ind, v = _coo_to_compressed(self.indices.astype(np.int64), self.col_ids(),
                                            self.values, self.n_rows)
        return CSRMatrix(indptr, ind, v, self.n_cols)


class DoKMatrix(Matrix):
    """Dictionary-of-keys matrix (upstream ``DoKMatrix``): O(1) set/get by (row, col); the shape
    grows with the largest key set unless fixed at construction."""

    def __init__(self, n_rows: int = 0, n_cols: int = 0):
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        self.data: dict[tuple[int, int], float] = {}

    def set(self, i: int, j: int, v: float) -> None:
        if i < 0 or j < 0:
            raise IndexError("DoKMatrix: negative index")
        if v == 0.0:
            self.data.pop((i, j), None)
        else:
            self.data[(i, j)] = float(v)
        self.n_rows = max(self.n_rows, i + 1)
        self.n_cols = max(self.n_cols, j + 1)

    def add(self, i: int, j: int, v: float) -> None:
        self.set(i, j, self.data.get((i, j), 0.0) + v)

    def get(self, i, j, default=0.0):
        return self.data.get((i, j), default)

    def nnz(self):
        return len(self.data)

    def row(self, i):
        return self.to_csr().row(i)

    def to_csr(self):
        if not self.data:
            return CSRMatrix(np.zeros(self.n_rows + 1, np.int64), [], [], self.n_cols)
        keys = np.array(list(self.data.keys()), dtype=np.int64)
        vals = np.fromiter(self.data.values(), dtype=np.float64, count=len(self.data))
        return CSRMatrix.from_coo(keys[:, 0], keys[:, 1], vals, self.shape)

    def to_dense(self):
        return self.to_csr().to_dense()

    def matvec(self, x):
        return self.to_csr().matvec(x)


def _parse_row(features) -> tuple[np.ndarray, np.ndarray]:
    """A builder row -> (column indices, values)."""
    if features is None:
        return np.zeros(0, np.int64), np.zeros(0, np.float64)
    if isinstance(features, np.ndarray) and features.dtype.kind == "f":
        nz = np.flatnonzero(features)
        return nz, features[nz].astype(np.float64)
    cols, vals = [], []
    for k, f in enumerate(features):
        if f is None:
            continue
        if isinstance(f, str):
            name, sep, v = f.partition(":")
            cols.append(int(name))
            vals.append(float(v) if sep else 1.0)
        elif isinstance(f, (tuple, list)):
            cols.append(int(f[0]))
            vals.append(float(f[1]))
        elif isinstance(f, (float, np.floating)):   # dense row of floats
            if f != 0.0:
                cols.append(k)
                vals.append(float(f))
        else:   # int / bigint feature arrays: index with value 1.0
            cols.append(int(f))
            vals.append(1.0)
    c = np.asarray(cols, dtype=np.int64)
    if len(c) and c.min() < 0:
        raise ValueError("negative feature index")
    return c, np.asarray(vals, dtype=np.float64)


class MatrixBuilder:
    """Row-at-a-time matrix assembly (upstream ``MatrixBuilder.nextRow`` / ``buildMatrix``).

    ``kind``: ``"csr"``, ``"csc"``, ``"dok"``, ``"dense"`` (row-major) or ``"dense_colmajor"``.
    ``n_cols`` fixes the width; otherwise it is 1 + the largest column seen.
    """

    KINDS = ("csr", "csc", "dok", "dense", "dense_colmajor")

    def __init__(self, kind: str = "csr", n_cols: int | None = None):
        if kind not in self.KINDS:
            raise ValueError(f"MatrixBuilder: unknown kind {kind!r}; one of {self.KINDS}")
        self.kind = kind
        self.n_cols = n_cols
        self._rows: list[np.ndarray] = []
        self._cols: list[np.ndarray] = []
        self._vals: list[np.ndarray] = []
        self.n_rows = 0
        self._width = 0

    def next_row(self, features: Sequence | np.ndarray | None) -> "MatrixBuilder":
        c, v = _parse_row(features)
        if features is not None and len(features) and isinstance(
                features[0], (float, np.floating)):   # dense row: its length is the width
            self._width = max(self._width, len(features))
        self._rows.append(np.full(len(c), self.n_rows, dtype=np.int64))
        self._cols.append(c)
        self._vals.append(v)
        self.n_rows += 1
        return self

    def next_rows(self, rows: Iterable) -> "MatrixBuilder":
        for r in rows:
            self.next_row(r)
        return self

    def build(self) -> Matrix:
        r = np.concatenate(self._rows) if self._rows else np.zeros(0, np.int64)
        c = np.concatenate(self._cols) if self._cols else np.zeros(0, np.int64)
        v = np.concatenate(self._vals) if self._vals else np.zeros(0, np.float64)
        width = self.n_cols if self.n_cols is not None else max(
            self._width, int(c.max()) + 1 if len(c) else 0)
        if len(c) and c.max() >= width:
            raise ValueError(f"MatrixBuilder: column {int(c.max())} >= n_cols {width}")
        csr = CSRMatrix.from_coo(r, c, v, (self.n_rows, width))
        if self.kind == "csr":
            return csr
        if self.kind == "csc":
            return csr.to_csc()
        if self.kind == "dok":
            m = DoKMatrix(self.n_rows, width)
            for i, j, x in zip(csr.row_ids().tolist(), csr.indices.tolist(), csr.values.tolist()):
                m.set(i, j, x)
            return m
        return DenseMatrix2d(csr.to_dense(), row_major=(self.kind == "dense"))
