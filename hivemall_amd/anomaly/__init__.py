"""Anomaly / change-point detection (upstream core/src/main/java/hivemall/
anomaly/{ChangeFinderUDF,ChangeFinder1D,ChangeFinder2D,SDAR1D,SDAR2D,
SingularSpectrumTransformUDF,SingularSpectrumTransform}.java).

Both are streaming functions over an ordered series; they are registered as *vectorised* UDFs
(the executor hands over the whole ordered column) so the SDAR / SST state lives in one
object per call.
"""
from __future__ import annotations

import math

import numpy as np

from ..registry import udf
from ..utils.options import Options, flag, opt

_CF_OPTS = Options([
    opt("k", None, 7, int, "Order of the AR model"),
    opt("r1", None, 0.02, float, "Discounting rate of the outlier stage"),
    opt("r2", None, 0.02, float, "Discounting rate of the change-point stage"),
    opt("T1", None, 7, int, "Smoothing window of the outlier scores"),
    opt("T2", None, 7, int, "Smoothing window of the change-point scores"),
    opt("outlier_threshold", None, -1.0, float, "Outlier threshold (emit is_outlier)"),
    opt("changepoint_threshold", None, -1.0, float, "Change-point threshold"),
    opt("loss_function", None, "hellinger", str, "hellinger | logloss"),
    opt("loss_function1", None, None, str, "Loss of stage 1"),
    opt("loss_function2", None, None, str, "Loss of stage 2")], "changefinder")


class SDAR1D:
    """Sequentially discounting AR model (Yamanishi & Takeuchi 2002)."""

    def __init__(self, r: float, k: int):
        self.r, self.k = r, k
        self.mu = 0.0
        self.C = np.zeros(k + 1)
        self.sigma = 0.0
        self.hist: list[float] = []
        self.n = 0

    def update(self, x: float, loss: str) -> float:
        r, k = self.r, self.k
        if self.n == 0:
            self.mu = x
            self.sigma = 1e-6
        self.mu = (1 - r) * self.mu + r * x
        past = self.hist[::-1]  # x_{t-1}, x_{t-2}, ...
        for j in range(k + 1):
            xj = x if j == 0 else (past[j - 1] if j - 1 < len(past) else self.mu)
            self.C[j] = (1 - r) * self.C[j] + r * (x - self.mu) * (xj - self.mu)
        w = _levinson(self.C)
        xhat = self.mu + sum(w[i] * ((past[i] if i < len(past) else self.mu) - self.mu)
                             for i in range(k))
        prev_sigma = self.sigma
        self.sigma = (1 - r) * self.sigma + r * (x - xhat) ** 2
        self.hist.append(x)
        if len(self.hist) > k:
            self.hist.pop(0)
        self.n += 1
        s2 = max(self.sigma, 1e-12)
        if loss == "logloss":
            return 0.5 * math.log(2 * math.pi * s2) + (x - xhat) ** 2 / (2 * s2)
        # Hellinger distance between the predictive distributions before / after the update
        s1 = max(prev_sigma, 1e-12)
        bc = math.sqrt(2 * math.sqrt(s1 * s2) / (s1 + s2))
        return max(0.0, 2.0 - 2.0 * bc * math.exp(-(x - xhat) ** 2 / (4 * (s1 + s2))))


def _levinson(C: np.ndarray) -> np.ndarray:
    """Solve the Yule-Walker equations Σ_j w_j C_|i-j| = C_{i+1} (Levinson-Durbin)."""
    k = len(C) - 1
    if C[0] <= 0:
        return np.zeros(k)
    a = np.zeros(k)
    e = C[0]
    for i in range(k):
        acc = C[i + 1] - sum(a[j] * C[i - j] for j in range(i))
        kappa = acc / e if e > 0 else 0.0
        kappa = max(-0.999, min(0.999, kappa))
        new = a.copy()
        new[i] = kappa
        for j in range(i):
            new[j] = a[j] - kappa * a[i - 1 - j]
        a = new
        e *= (1 - kappa * kappa)
    return a


class ChangeFinder:
    def __init__(self, options: str | None):
        c = _CF_OPTS.parse(options)
        self.c = c
        l1 = c["loss_function1"] or c["loss_function"]
        l2 = c["loss_function2"] or c["loss_function"]
        self.l1, self.l2 = l1, l2
        self.s1: list = []
        self.s2: list = []
        self.m1 = None
        self.m2 = None

    def _mk(self, dim, r):
        return [SDAR1D(r, self.c["k"]) for _ in range(dim)]

    def step(self, x):
        xs = np.atleast_1d(np.asarray(x, dtype=np.float64))
        if self.m1 is None:
            self.m1 = self._mk(len(xs), self.c["r1"])
            self.m2 = SDAR1D(self.c["r2"], self.c["k"])
        o = float(sum(m.update(float(v), self.l1) for m, v in zip(self.m1, xs)))
        self.s1.append(o)
        y = float(np.mean(self.s1[-self.c["T1"]:]))
        cp_raw = self.m2.update(y, self.l2)
        self.s2.append(cp_raw)
        cp = float(np.mean(self.s2[-self.c["T2"]:]))
        out = [o, cp]
        if self.c["outlier_threshold"] >= 0 or self.c["changepoint_threshold"] >= 0:
            out += [o > self.c["outlier_threshold"] >= 0, cp > self.c["changepoint_threshold"] >= 0]
        return out


@udf("changefinder", vectorized=True)
def changefinder(xs, options=None):
    """Per ordered input: [outlier_score, changepoint_score(, is_outlier, is_changepoint)]."""
    o = options[0] if isinstance(options, (list, tuple, np.ndarray)) else options
    cf = ChangeFinder(o)
    return [cf.step(x) for x in xs]


_SST_OPTS = Options([
    opt("w", "window", 30, int, "Window size"),
    opt("n", "n_past", None, int, "Number of past windows"),
    opt("m", "n_current", None, int, "Number of current windows"),
    opt("g", "current_offset", None, int, "Offset of the current windows"),
    opt("r", "n_component", 3, int, "Rank of the past subspace"),
    opt("k", "n_dim", 5, int, "Rank of the current subspace"),
    opt("th", "threshold", -1.0, float, "Change-point threshold"),
    flag("ika", None, "Use the implicit Krylov approximation",
         inert="SST uses an exact (batched) SVD")], "sst")


@udf("sst", vectorized=True)
def sst(xs, options=None):
    """Singular spectrum transformation score per point: 1 - (largest singular value of
    U_pastᵀ U_current)² between the top-r past and top-k current subspaces."""
    o = options[0] if isinstance(options, (list, tuple, np.ndarray)) else options
    c = _SST_OPTS.parse(o)
    w = c["w"]
    n = c["n"] or w
    m = c["m"] or w
    g = c["g"] if c["g"] is not None else -w
    r, k = c["r"], c["k"]
    x = np.asarray(list(xs), dtype=np.float64)
    out = []
    need = w + n + max(0, -g) + m
    for t in range(len(x)):
        if t + 1 < need:
            out.append([0.0] if c["th"] < 0 else [0.0, False])
            continue
        end = t + 1
        past = np.stack([x[end + g - m - n + i - w + 1: end + g - m - n + i + 1] for i in range(n)], 1)
        cur = np.stack([x[end - m + i - w + 1: end - m + i + 1] for i in range(m)], 1)
        U, _, _ = np.linalg.svd(past, full_matrices=False)
        Q, _, _ = np.linalg.svd(cur, full_matrices=False)
        s = np.linalg.svd(U[:, :r].T @ Q[:, :k], compute_uv=False)
        score = float(1.0 - (s[0] ** 2 if s.size else 0.0))
        out.append([score] if c["th"] < 0 else [score, score > c["th"]])
    return out
