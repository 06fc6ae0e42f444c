"""Integer matrices and math vectors (upstream
core/src/main/java/hivemall/math/matrix/ints/{IntMatrix,AbstractIntMatrix,DoKIntMatrix,
ColumnMajorIntMatrix,ColumnMajorDenseIntMatrix2d}.java and
math/vector/{Vector,DenseVector,SparseVector,VectorProcedure}.java).

Upstream uses the int matrices for co-occurrence counts (SLIM's item-item kNN restriction,
``item_pairs_sampling``) and the vectors as per-row views of the training matrices.  Here
the storage is numpy (int32 counts, float64 values) so a whole matrix moves to HBM in one
``to_torch`` copy; the per-element API mirrors upstream (``get/set/incr``, ``eachInRow`` /
``eachNonZeroInColumn`` as Python iterators).
"""
from __future__ import annotations

from typing import Iterator

import numpy as np


class IntMatrix:
    """Read/write interface of upstream ``IntMatrix``; ``default_value`` is returned for
    absent cells (upstream ``setDefaultValue``)."""

    n_rows: int
    n_cols: int
    default_value: int = 0

    @property
    def shape(self) -> tuple[int, int]:
        return (self.n_rows, self.n_cols)

    def get(self, i: int, j: int) -> int:
        raise NotImplementedError

    def set(self, i: int, j: int, v: int) -> None:
        raise NotImplementedError

    def incr(self, i: int, j: int, delta: int = 1) -> int:
        v = self.get(i, j) + int(delta)
        self.set(i, j, v)
        return v

    def nnz(self) -> int:
        raise NotImplementedError

    def to_dense(self) -> np.ndarray:
        raise NotImplementedError

    def each_in_row(self, i: int, nonzero_only: bool = True) -> Iterator[tuple[int, int]]:
        row = self.to_dense()[i] if i < self.n_rows else np.zeros(self.n_cols, np.int32)
        for j, v in enumerate(row):
            if not nonzero_only or v != 0:
                yield j, int(v)

    def each_nonzero_in_column(self, j: int) -> Iterator[tuple[int, int]]:
        col = self.to_dense()[:, j] if j < self.n_cols else np.zeros(self.n_rows, np.int32)
        for i in np.flatnonzero(col):
            yield int(i), int(col[i])

    def to_torch(self, device=None):
        import torch

        return torch.from_numpy(np.ascontiguousarray(self.to_dense())).to(device)


class DoKIntMatrix(IntMatrix):
    """Dictionary-of-keys int matrix; the shape grows with the largest key (``DoKIntMatrix``).
    Setting a cell to the default value removes it."""

    def __init__(self, n_rows: int = 0, n_cols: int = 0, default_value: int = 0):
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        self.default_value = int(default_value)
        self.data: dict[tuple[int, int], int] = {}

    def get(self, i, j):
        return self.data.get((int(i), int(j)), self.default_value)

    def set(self, i, j, v):
        i, j = int(i), int(j)
        if i < 0 or j < 0:
            raise IndexError("DoKIntMatrix: negative index")
        if int(v) == self.default_value:
            self.data.pop((i, j), None)
        else:
            self.data[(i, j)] = int(v)
        self.n_rows = max(self.n_rows, i + 1)
        self.n_cols = max(self.n_cols, j + 1)

    def nnz(self):
        return len(self.data)

    def to_dense(self):
        out = np.full(self.shape, self.default_value, dtype=np.int32)
        for (i, j), v in self.data.items():
            out[i, j] = v
        return out

    def each_nonzero_in_column(self, j):
        for (i, jj), v in sorted(self.data.items()):
            if jj == j and v != 0:
                yield i, v

    def to_column_major(self) -> "ColumnMajorIntMatrix":
        return ColumnMajorIntMatrix.from_dense(self.to_dense())


class ColumnMajorDenseIntMatrix2d(IntMatrix):
    """Dense int32 matrix stored column by column (``ColumnMajorDenseIntMatrix2d``)."""

    def __init__(self, n_rows: int, n_cols: int, default_value: int = 0):
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)
        self.default_value = int(default_value)
        self.cols = np.full((self.n_cols, self.n_rows), self.default_value, dtype=np.int32)

    @classmethod
    def from_dense(cls, a) -> "ColumnMajorDenseIntMatrix2d":
        a = np.asarray(a, dtype=np.int32)
        m = cls(a.shape[0], a.shape[1])
        m.cols[:] = a.T
        return m

    def get(self, i, j):
        if not (0 <= i < self.n_rows and 0 <= j < self.n_cols):
            return self.default_value
        return int(self.cols[j, i])

    def set(self, i, j, v):
        if not (0 <= i < self.n_rows and 0 <= j < self.n_cols):
            raise IndexError(f"({i}, {j}) outside {self.shape}")
        self.cols[j, i] = v

    def nnz(self):
        return int(np.count_nonzero(self.cols))

    def to_dense(self):
        return self.cols.T.copy()

    def each_nonzero_in_column(self, j):
        c = self.cols[j]
        for i in np.flatnonzero(c):
            yield int(i), int(c[i])


class ColumnMajorIntMatrix(IntMatrix):
    """Read-only compressed-column int matrix (``ColumnMajorIntMatrix``: per-column sorted row
    indices + values)."""

    def __init__(self, colptr, rowidx, values, n_rows: int):
        self.colptr = np.asarray(colptr, dtype=np.int64)
        self.rowidx = np.asarray(rowidx, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.int32)
        self.n_rows, self.n_cols = int(n_rows), len(self.colptr) - 1

    @classmethod
    def from_dense(cls, a) -> "ColumnMajorIntMatrix":
        a = np.asarray(a, dtype=np.int32)
        cols, rows = np.nonzero(a.T)
        ptr = np.zeros(a.shape[1] + 1, np.int64)
        np.add.at(ptr, cols + 1, 1)
        return cls(np.cumsum(ptr), rows, a[rows, cols], a.shape[0])

    def get(self, i, j):
        if not (0 <= j < self.n_cols):
            return self.default_value
        s, e = self.colptr[j], self.colptr[j + 1]
        k = np.searchsorted(self.rowidx[s:e], i)
        if k < e - s and self.rowidx[s + k] == i:
            return int(self.values[s + k])
        return self.default_value

    def set(self, i, j, v):
        raise TypeError("ColumnMajorIntMatrix is read-only (build it with DoKIntMatrix)")

    def nnz(self):
        return int(self.values.size)

    def to_dense(self):
        out = np.zeros(self.shape, dtype=np.int32)
        for j in range(self.n_cols):
            s, e = self.colptr[j], self.colptr[j + 1]
            out[self.rowidx[s:e], j] = self.values[s:e]
        return out

    def each_nonzero_in_column(self, j):
        s, e = self.colptr[j], self.colptr[j + 1]
        for k in range(s, e):
            yield int(self.rowidx[k]), int(self.values[k])


# ------------------------------------------------------------------------------ vectors
class Vector:
    """Upstream ``hivemall.math.vector.Vector``: get/set/incr, ``each(nonzero)``, ``size``."""

    def get(self, i: int, default: float = 0.0) -> float:
        raise NotImplementedError

    def set(self, i: int, v: float) -> None:
        raise NotImplementedError

    def incr(self, i: int, delta: float) -> None:
        self.set(i, self.get(i) + delta)

    def size(self) -> int:
        raise NotImplementedError

    def to_array(self) -> np.ndarray:
        raise NotImplementedError

    def dot(self, other: "Vector") -> float:
        a, b = self.to_array(), other.to_array()
        n = min(a.size, b.size)
        return float(a[:n] @ b[:n])


class DenseVector(Vector):
    def __init__(self, size_or_values):
        if np.isscalar(size_or_values):
            self.values = np.zeros(int(size_or_values), dtype=np.float64)
        else:
            self.values = np.array(size_or_values, dtype=np.float64)

    def get(self, i, default=0.0):
        return float(self.values[i]) if 0 <= i < self.values.size else default

    def set(self, i, v):
        self.values[i] = v

    def size(self):
        return int(self.values.size)

    def to_array(self):
        return self.values

    def each(self, nonzero_only: bool = True):
        for i, v in enumerate(self.values):
            if not nonzero_only or v != 0.0:
                yield i, float(v)

    def clear(self):
        self.values[:] = 0.0


class SparseVector(Vector):
    """Index -> value map (upstream ``SparseVector`` over an ``Int2DoubleOpenHashTable``);
    ``size`` is the largest index + 1."""

    def __init__(self):
        self.data: dict[int, float] = {}

    def get(self, i, default=0.0):
        return self.data.get(int(i), default)

    def set(self, i, v):
        if v == 0.0:
            self.data.pop(int(i), None)
        else:
            self.data[int(i)] = float(v)

    def size(self):
        return max(self.data) + 1 if self.data else 0

    def to_array(self):
        out = np.zeros(self.size(), dtype=np.float64)
        for i, v in self.data.items():
            out[i] = v
        return out

    def each(self, nonzero_only: bool = True):
        for i in sorted(self.data):
            yield i, self.data[i]

    def clear(self):
        self.data.clear()
