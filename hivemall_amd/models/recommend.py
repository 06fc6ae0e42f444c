"""``train_slim`` (SLIM, Ning & Karypis ICDM'11) and ``train_kpa`` / ``kpa_predict``
(kernel-expanded Passive-Aggressive).

Reference behaviour: Hivemall recommend/SlimUDTF, classifier/KernelExpansionPassiveAggressiveUDTF,
classifier/KPAPredictUDAF.  Both are small, per-item /
per-example sequential learners and run on the host.
"""
from __future__ import annotations

import math
from collections import defaultdict

import numpy as np
import pandas as pd

from ..registry import udaf
from ..utils.options import opt
from .base import Learner

SLIM_OPTS = [
    opt("l1", None, 0.001, float, "L1 regularization"),
    opt("l2", None, 0.0005, float, "L2 regularization"),
    opt("iters", "iterations", 30, int, "Coordinate-descent sweeps", aliases=("iter",)),
    opt("eps", None, 1e-4, float, "Convergence threshold on the max weight change"),
    opt("disable_cv", None, None, str, "Accepted"),
]


def slim_cd_batched(Gs, bs, l1: float, l2: float, iters: int, eps: float, device=None):
    """Non-negative elastic-net coordinate descent for every item at once, in Gram form.

    Per item the problem is min_w ½||y − Xw||² + ½λ2||w||² + λ1||w||₁, w ≥ 0 with
    G = XᵀX, b = Xᵀy.  A coordinate step is ρ_k = b_k − Σ_{m≠k} G_km w_m,
    w_k = max(0, ρ_k − λ1) / (G_kk + λ2) — the same update and coordinate order as the
    per-item residual loop of upstream SlimUDTF, so the result matches it to rounding.  All
    items (padded to the largest neighbourhood K) advance together: one [items, K] mat-vec
    row per coordinate, on the learner's device; an item stops when its largest change in a
    sweep falls below ``eps`` (the per-item convergence test).  Returns an [items, K] numpy
    array (padding columns are zero).
    """
    n = len(Gs)
    Kmax = max(g.shape[0] for g in Gs)
    out = np.zeros((n, Kmax))
    # items sorted by neighbourhood size and solved in chunks of bounded n_chunk * K_chunk^2 Gram
    # bytes: padding to one item's huge kNN union no longer sizes every item's Gram matrix
    order = np.argsort([g.shape[0] for g in Gs], kind="stable")
    s = 0
    while s < n:
        e = s + 1
        kc = Gs[order[s]].shape[0]
        while e < n:
            k_next = max(kc, Gs[order[e]].shape[0])
            if (e + 1 - s) * k_next * k_next * 8 > _SLIM_CHUNK_BYTES:
                break
            kc = k_next
            e += 1
        idx = order[s:e]
        w = _slim_cd_chunk([Gs[i] for i in idx], [bs[i] for i in idx], l1, l2, iters, eps, device)
        out[idx, :w.shape[1]] = w
        s = e
    return out


_SLIM_CHUNK_BYTES = 256 << 20


def _slim_cd_chunk(Gs, bs, l1: float, l2: float, iters: int, eps: float, device=None):
    import torch

    dev = device if device is not None else torch.device("cpu")
    n = len(Gs)
    K = max(g.shape[0] for g in Gs)
    G = torch.zeros((n, K, K), dtype=torch.float64)
    b = torch.zeros((n, K), dtype=torch.float64)
    for t, (g, v) in enumerate(zip(Gs, bs)):
        m = g.shape[0]
        G[t, :m, :m] = torch.from_numpy(np.asarray(g, dtype=np.float64))
        b[t, :m] = torch.from_numpy(np.asarray(v, dtype=np.float64))
    G, b = G.to(dev), b.to(dev)
    w = torch.zeros((n, K), dtype=torch.float64, device=dev)
    diag = torch.diagonal(G, dim1=1, dim2=2)
    live = diag > 0                                   # sq[k] == 0 columns are skipped
    active = torch.ones(n, dtype=torch.bool, device=dev)
    for _ in range(iters):
        dmax = torch.zeros(n, dtype=torch.float64, device=dev)
        for k in range(K):
            gk = G[:, k, :]
            rho = b[:, k] - (gk * w).sum(1) + diag[:, k] * w[:, k]
            nw = torch.clamp(rho - l1, min=0.0) / (diag[:, k] + l2)
            upd = active & live[:, k]
            nw = torch.where(upd, nw, w[:, k])
            dmax = torch.maximum(dmax, (nw - w[:, k]).abs())
            w[:, k] = nw
        active = active & (dmax >= eps)
        if not bool(active.any()):
            break
    return w.cpu().numpy()


class SLIM(Learner):
    """For every item i: min_w ½||r_i − Σ_j w_j r_j||² + ½λ2||w||² + λ1||w||₁, w ≥ 0, over the
    item's kNN neighbours j (coordinate descent with soft thresholding)."""
    NAME = "train_slim"
    OPTIONS = SLIM_OPTS

    def fit(self, i_col, ri_col, knn_col, j_col, rj_col):
        c = self.cl
        groups: dict = defaultdict(lambda: {"ri": None, "nb": {}})
        for i, ri, knn, j, rj in zip(i_col, ri_col, knn_col, j_col, rj_col):
            g = groups[i]
            if ri is not None:
                g["ri"] = dict(ri)
            if j is not None and rj is not None:
                g["nb"][j] = dict(rj)
            if knn:
                for jj, rr in dict(knn).items():
                    g["nb"].setdefault(jj, dict(rr))
        items, nbl, Gs, bs = [], [], [], []
        for i, g in groups.items():
            ri = g["ri"] or {}
            nbs = [j for j in g["nb"] if j != i]
            if not ri or not nbs:
                continue
            users = sorted(set(ri) | {u for j in nbs for u in g["nb"][j]})
            uix = {u: k for k, u in enumerate(users)}
            y = np.zeros(len(users))
            for u, v in ri.items():
                y[uix[u]] = v
            X = np.zeros((len(users), len(nbs)))
            for col, j in enumerate(nbs):
                for u, v in g["nb"][j].items():
                    X[uix[u], col] = v
            items.append(i)
            nbl.append(nbs)
            Gs.append(X.T @ X)
            bs.append(X.T @ y)
        rows = []
        if items:
            W = slim_cd_batched(Gs, bs, float(c["l1"]), float(c["l2"]), int(c["iters"]),
                                float(c["eps"]), self.device)
            for n, (i, nbs) in enumerate(zip(items, nbl)):
                for k, j in enumerate(nbs):
                    if W[n, k] != 0:
                        rows.append((i, j, float(W[n, k])))
        self.table = pd.DataFrame(rows, columns=["i", "nn", "w"])
        return self

    def model_table(self) -> pd.DataFrame:
        return self.table


KPA_OPTS = [
    opt("pkc", None, 1.0, float, "Constant c of the polynomial kernel (x·x' + c)^2"),
    opt("c", "aggressiveness", 1.0, float, "PA-I aggressiveness"),
    opt("iters", "iterations", 1, int, "Epochs"),
]


def _fv(f):
    s = str(f)
    p = s.find(":")
    return (s, 1.0) if p < 0 else (s[:p], float(s[p + 1:]))


class KPA(Learner):
    """PA-I on the explicit degree-2 polynomial kernel expansion:
    φ(x) = [√c²·1, √(2c)·x_h, x_h², √2·x_h x_k (h<k)]; weights (w0, w1, w2, w3)."""
    NAME = "train_kpa"
    OPTIONS = KPA_OPTS

    def fit(self, features, labels):
        c = self.cl
        pkc = float(c["pkc"])
        self.w0 = 0.0
        self.w1: dict = defaultdict(float)
        self.w2: dict = defaultdict(float)
        self.w3: dict = defaultdict(float)
        s0, s1, s2 = pkc, math.sqrt(2 * pkc), math.sqrt(2)
        for _ in range(int(c["iters"])):
            for feats, lab in zip(features, labels):
                y = 1.0 if float(lab) > 0 else -1.0
                xs = [_fv(f) for f in feats]
                p = self.w0 * s0
                sq = s0 * s0
                for h, x in xs:
                    p += self.w1[h] * s1 * x + self.w2[h] * x * x
                    sq += 2 * pkc * x * x + x ** 4
                for a in range(len(xs)):
                    for b in range(a + 1, len(xs)):
                        (h, xh), (k, xk) = xs[a], xs[b]
                        p += self.w3[(h, k)] * s2 * xh * xk
                        sq += 2 * (xh * xk) ** 2
                loss = max(0.0, 1.0 - y * p)
                if loss <= 0:
                    continue
                eta = min(float(c["c"]), loss / sq) * y
                self.w0 += eta * s0
                for h, x in xs:
                    self.w1[h] += eta * s1 * x
                    self.w2[h] += eta * x * x
                for a in range(len(xs)):
                    for b in range(a + 1, len(xs)):
                        (h, xh), (k, xk) = xs[a], xs[b]
                        self.w3[(h, k)] += eta * s2 * xh * xk
        self.pkc = pkc
        return self

    def model_table(self) -> pd.DataFrame:
        s0, s1, s2 = self.pkc, math.sqrt(2 * self.pkc), math.sqrt(2)
        rows = [(0, None, self.w0 * s0, None, None, None)]
        for h in self.w1:
            rows.append((h, None, None, self.w1[h] * s1, self.w2[h], None))
        for (h, k), v in self.w3.items():
            rows.append((h, k, None, None, None, v * s2))
        return pd.DataFrame(rows, columns=["h", "hk", "w0", "w1", "w2", "w3"])

    def decision_function(self, features) -> np.ndarray:
        tab = self.model_table()
        out = []
        for feats in features:
            xs = [_fv(f) for f in feats]
            out.append(_kpa_score(xs, self))
        return np.asarray(out)


def _kpa_score(xs, m):
    s0, s1, s2 = m.pkc, math.sqrt(2 * m.pkc), math.sqrt(2)
    p = m.w0 * s0
    for h, x in xs:
        p += m.w1.get(h, 0.0) * s1 * x + m.w2.get(h, 0.0) * x * x
    for a in range(len(xs)):
        for b in range(a + 1, len(xs)):
            (h, xh), (k, xk) = xs[a], xs[b]
            p += m.w3.get((h, k), 0.0) * s2 * xh * xk
    return p


@udaf("kpa_predict")
def kpa_predict(xh, xk, w0, w1, w2, w3):
    """Σ over the joined feature_pairs('-kpa') rows: w0 + w1·xh + w2·xh² + w3·xh·xk."""
    s = 0.0
    seen_bias = False
    for a, b, z0, z1, z2, z3 in zip(xh, xk, w0, w1, w2, w3):
        if z0 is not None and not seen_bias and not (isinstance(z0, float) and math.isnan(z0)):
            s += float(z0)
            seen_bias = True
        if b is None:
            if z1 is not None and not (isinstance(z1, float) and math.isnan(z1)):
                s += float(z1) * float(a)
            if z2 is not None and not (isinstance(z2, float) and math.isnan(z2)):
                s += float(z2) * float(a) * float(a)
        elif z3 is not None and not (isinstance(z3, float) and math.isnan(z3)):
            s += float(z3) * float(a) * float(b)
    return s


def register_sql(reg):
    reg("train_slim", lambda: SLIM, n_data_args=5)
    reg("train_kpa", lambda: KPA)
