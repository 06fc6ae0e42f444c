"""Ensemble UDAFs (upstream core/src/main/java/hivemall/ensemble/
{bagging/VotedAvgUDAF,bagging/WeightVotedAvgUDAF,MaxValueLabelUDAF,MaxRowUDAF,ArgminKLDistanceUDAF}).

``argmin_kld`` is the model-mixing rule of the covariance learners: the argmin of the summed
KL divergence between Gaussians N(w_i, σ_i) is w = Σ(w_i/σ_i) / Σ(1/σ_i) with covariance
1/Σ(1/σ_i).  The same rule runs on the device in ``csrc/kernels/linear.hip`` (replica mixing)
and over RCCL in ``parallel.mix.ModelMixer.argmin_kld``.
"""
from __future__ import annotations

import numpy as np

from ..registry import udaf


@udaf("voted_avg")
def voted_avg(values):
    """Average of the majority-sign values (positive votes vs. negative votes)."""
    v = np.asarray([x for x in values if x is not None], dtype=np.float64)
    if v.size == 0:
        return None
    pos, neg = v[v > 0], v[v <= 0]
    if pos.size > neg.size:
        return float(pos.mean())
    return float(neg.mean()) if neg.size else 0.0


@udaf("weight_voted_avg")
def weight_voted_avg(values):
    """Majority decided by the summed weights of each sign; average of the winning side."""
    v = np.asarray([x for x in values if x is not None], dtype=np.float64)
    if v.size == 0:
        return None
    pos, neg = v[v > 0], v[v <= 0]
    if pos.sum() > -neg.sum():
        return float(pos.mean())
    return float(neg.mean()) if neg.size else 0.0


@udaf("max_label")
def max_label(scores, labels):
    """Label of the maximum score."""
    best, lab = None, None
    for s, l in zip(scores, labels):
        if s is None:
            continue
        if best is None or s > best:
            best, lab = s, l
    return lab


@udaf("maxrow")
def maxrow(scores, *cols):
    """The row (score, cols...) with the maximum score, as a list."""
    best = None
    out = None
    for i, s in enumerate(scores):
        if s is None:
            continue
        if best is None or s > best:
            best = s
            out = [s] + [c[i] for c in cols]
    return out


@udaf("argmin_kld")
def argmin_kld(means, covars):
    """Σ(w/σ)/Σ(1/σ) (the mixed weight); see module doc."""
    m = np.asarray(means, dtype=np.float64)
    c = np.asarray(covars, dtype=np.float64)
    ok = np.isfinite(m) & np.isfinite(c) & (c > 0)
    if not ok.any():
        return None
    inv = 1.0 / c[ok]
    return float((m[ok] * inv).sum() / inv.sum())


def argmin_kld_covar(covars):
    c = np.asarray(covars, dtype=np.float64)
    c = c[np.isfinite(c) & (c > 0)]
    return float(1.0 / (1.0 / c).sum()) if c.size else None
