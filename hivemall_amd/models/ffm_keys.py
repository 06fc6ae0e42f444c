"""FFM model-table key scheme + the SQL-side prediction path (docs/compat.md O4).

Model table rows ``(model_id, i, Wi, Vi)``:
  * ``i = -1``                          global bias w0 in ``Wi``;
  * ``i = feature``                     linear weight ``Wi`` (``Vi`` NULL);
  * ``i = NF + feature * F + field``    latent vector V[feature, field] in ``Vi`` (``Wi`` NULL),
where NF = number of (hashed) features and F = number of fields.  This mirrors upstream's
FFMStringFeatureMapModel, whose keys address V(feature, field) entries, so prediction is
the documented SQL pattern:

    feature_pairs(features, '-ffm -feature_hashing B -num_fields F') -> (i, j, Xi, Xj)
    JOIN model m1 ON m1.i = t.i  LEFT JOIN model m2 ON m2.i = t.j
    ffm_predict(m1.Wi, m1.Vi, m2.Vi, t.Xi, t.Xj) GROUP BY rowid
"""
from __future__ import annotations

import math

import numpy as np

from ..registry import udaf
from ..utils.features import parse_ffm_rows


def vkey(feature: int, field: int, num_features: int, num_fields: int) -> int:
    return num_features + feature * num_fields + field


def ffm_pair_rows(features, cl):
    """Rows (i, j, xi, xj) of one FFM feature vector (used by ``feature_pairs -ffm``)."""
    nf = (1 << cl["feature_hashing"]) if cl["feature_hashing"] > 0 else (1 << 24)
    F = int(cl["num_fields"])
    csr = parse_ffm_rows([list(features)], nf, F, hash_ints=cl["feature_hashing"] > 0)
    idx, val, fld = csr.idx, csr.val.astype(np.float64), csr.fld
    norm = math.sqrt(float((val * val).sum())) or 1.0
    if not cl.has("no_norm") or not cl["no_norm"]:
        val = val / norm
    if not cl["no_bias"]:
        yield (-1, None, 1.0, None)
    n = len(idx)
    for a in range(n):
        yield (int(idx[a]), None, float(val[a]), None)
    for a in range(n):
        for b in range(a + 1, n):
            yield (vkey(int(idx[a]), int(fld[b]), nf, F), vkey(int(idx[b]), int(fld[a]), nf, F),
                   float(val[a]), float(val[b]))


def ffm_pair_columns(rows: list, cl):
    """``ffm_pair_rows`` for a whole column at once (the LATERAL VIEW batch path): returns
    (source row of every output row, {i, j, xi, xj} arrays), rows in the per-row order.  NULL
    feature lists produce no rows.  ``j`` / ``xj`` are NaN where the per-row path yields NULL
    (the float64 column pandas builds from those rows)."""
    nf = (1 << cl["feature_hashing"]) if cl["feature_hashing"] > 0 else (1 << 24)
    F = int(cl["num_fields"])
    keep = np.asarray([r is not None for r in rows], dtype=bool)
    src = np.nonzero(keep)[0]
    csr = parse_ffm_rows([list(rows[r]) for r in src], nf, F, hash_ints=cl["feature_hashing"] > 0)
    indptr = np.asarray(csr.indptr, dtype=np.int64)
    idx = np.asarray(csr.idx, dtype=np.int64)
    fld = np.asarray(csr.fld, dtype=np.int64)
    val = np.asarray(csr.val, dtype=np.float32).astype(np.float64)
    lens = np.diff(indptr)
    n = len(src)
    if not cl.has("no_norm") or not cl["no_norm"]:
        row_of = np.repeat(np.arange(n), lens)
        norm = np.sqrt(np.bincount(row_of, weights=val * val, minlength=n))
        norm[norm == 0] = 1.0
        val = val / norm[row_of]
    nb = 0 if cl["no_bias"] else 1
    cnt = nb + lens + lens * (lens - 1) // 2
    start = np.zeros(n, dtype=np.int64)
    np.cumsum(cnt[:-1], out=start[1:])
    total = int(cnt.sum())
    I = np.empty(total, dtype=np.int64)
    J = np.full(total, np.nan)
    XI = np.empty(total, dtype=np.float64)
    XJ = np.full(total, np.nan)
    if nb:
        I[start] = -1
        XI[start] = 1.0
    for L in np.unique(lens):
        L = int(L)
        if L == 0:
            continue
        rs = np.nonzero(lens == L)[0]
        base = start[rs] + nb
        fi = indptr[rs][:, None] + np.arange(L)
        ii, vv, ff = idx[fi], val[fi], fld[fi]
        pos = base[:, None] + np.arange(L)
        I[pos] = ii
        XI[pos] = vv
        a, b = np.triu_indices(L, 1)
        if len(a):
            pos = base[:, None] + L + np.arange(len(a))
            I[pos] = nf + ii[:, a] * F + ff[:, b]
            J[pos] = nf + ii[:, b] * F + ff[:, a]
            XI[pos] = vv[:, a]
            XJ[pos] = vv[:, b]
    return np.repeat(src, cnt), {"i": I, "j": J, "xi": XI, "xj": XJ}


@udaf("ffm_predict")
def ffm_predict(Wi, Vi, Vj, Xi, Xj):
    """Σ Wi·Xi over linear/bias rows + Σ <Vi, Vj>·Xi·Xj over pair rows (raw score)."""
    s = 0.0
    for w, vi, vj, xi, xj in zip(Wi, Vi, Vj, Xi, Xj):
        if vi is not None and vj is not None and xj is not None:
            s += float(np.dot(np.asarray(vi, dtype=np.float64), np.asarray(vj, dtype=np.float64))) \
                * float(xi) * float(xj)
        elif w is not None and not (isinstance(w, float) and math.isnan(w)):
            s += float(w) * float(xi)
    return s
