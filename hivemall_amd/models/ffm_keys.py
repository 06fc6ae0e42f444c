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
