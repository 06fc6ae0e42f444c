"""Synthetic dataset generators with the shapes of the benchmark configs (BASELINE.json).

No network => no real datasets.  Every generator plants a known model so logloss / AUC
have a meaningful floor, and runs with torch ops directly on the target device.

* ``criteo_like``  — Criteo display-ads shape: 39 fields (13 bucketised integer + 26
  categorical) with the published Kaggle-DAC per-field cardinalities, power-law value
  frequencies, hashed into 2^bits feature ids, every value 1.0; labels from a planted FM-style
  logit with a ~20 % positive rate.
* ``criteo_ffm``   — the same shape as ``field:index:value`` triples: explicit field ids and
  log-scaled count values on the 13 integer fields (the headline bench's data).
* ``a9a_like``     — 123 binary features, ~14 nnz/row (libsvm a9a shape).
* ``higgs_like``   — 28 dense float features (HIGGS shape), planted non-linear boundary.
* ``movielens_like`` — implicit feedback triples with MovieLens-20M user/item counts.
"""
from __future__ import annotations

import math

import numpy as np
import torch

# Kaggle Criteo DAC categorical cardinalities (C1..C26); integer fields I1..I13 are
# bucketised (log2 buckets) before hashing, ~64 buckets each.
CRITEO_CAT_CARD = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593,
                   3194, 27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105,
                   142572]
CRITEO_INT_CARD = [64] * 13


def _gen(seed: int, device) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def criteo_like(n_rows: int, hash_bits: int = 20, seed: int = 7, device="cpu",
                zipf_power: float = 3.0, planted_k: int = 4, chunk: int = 1 << 20,
                return_logit: bool = False, model_seed: int = 20240607):
    """Criteo-shaped FFM data on ``device``.

    Returns (idx int32 [n,39], y f32 [n] in {-1,+1}); field of slot j is j, value 1.0.
    ``seed`` selects the rows; the planted model depends only on ``model_seed`` (so shards
    and held-out sets generated with different seeds share one ground truth).
    """
    device = torch.device(device)
    cards = torch.tensor(CRITEO_INT_CARD + CRITEO_CAT_CARD, dtype=torch.float64, device=device)
    F = cards.numel()
    NF = 1 << hash_bits
    gm = _gen(model_seed, device)
    # planted model (hashed tables, same id space)
    w_true = torch.randn(NF, generator=gm, device=device)
    U = torch.randn(NF, planted_k, generator=gm, device=device) * 0.5
    pair_std = math.sqrt(F * (F - 1) / 2 * planted_k * 0.5 ** 4)
    bias = -1.7
    idx_out = torch.empty(n_rows, F, dtype=torch.int32, device=device)
    y_out = torch.empty(n_rows, dtype=torch.float32, device=device)
    logit_out = torch.empty(n_rows, dtype=torch.float32, device=device) if return_logit else None
    g = _gen(seed, device)
    field_salt = (torch.arange(F, device=device, dtype=torch.int64) * 0x9E3779B1) & 0x7FFFFFFF
    for s in range(0, n_rows, chunk):
        e = min(n_rows, s + chunk)
        n = e - s
        u = torch.rand(n, F, generator=g, device=device, dtype=torch.float64)
        v = torch.floor(cards * u.pow(zipf_power)).to(torch.int64)        # power-law values
        h = (v * 0x5BD1E995 + field_salt) & 0x7FFFFFFF                    # mix, no overflow
        h = ((h ^ (h >> 15)) * 0x2545F491) & 0x7FFFFFFF
        ids = (h ^ (h >> 13)) & (NF - 1)
        idx_out[s:e] = ids.to(torch.int32)
        lin = w_true[ids].sum(1)
        Ur = U[ids]                                                        # [n,F,k]
        sv = Ur.sum(1)
        pair = 0.5 * ((sv * sv).sum(1) - (Ur * Ur).sum((1, 2)))
        logit = bias + lin / math.sqrt(F) + 0.7 * pair / pair_std
        p = torch.sigmoid(logit)
        y_out[s:e] = torch.where(torch.rand(n, generator=g, device=device) < p, 1.0, -1.0)
        if logit_out is not None:
            logit_out[s:e] = logit
    if return_logit:
        return idx_out, y_out, logit_out
    return idx_out, y_out


def criteo_ffm(n_rows: int, hash_bits: int = 20, seed: int = 7, device="cpu",
               zipf_power: float = 3.0, planted_k: int = 4, chunk: int = 1 << 20,
               return_logit: bool = False, model_seed: int = 20240607):
    """Criteo-for-FFM rows with explicit fields and values (the ``field:index:value`` triples
    train_ffm parses): the 13 integer fields carry a raw count
    ``c = floor(2^(16 u^2)) - 1`` (u uniform: mostly small counts, a long tail up to 65,535),
    hashed by its log2 bucket (``floor(4 log2(1 + c))``, 64 buckets per field) and valued
    ``log2(2 + c) / 4`` (log-scaled count, in [0.25, 4.25)); the 26 categorical fields draw
    Kaggle-DAC-cardinality power-law ids, value 1.

    The planted logit reads the values the way the model does, after the instance L2 norm
    (scaled so a row of all-ones values gives :func:`criteo_like`'s logit scale).

    Returns (idx int32 [n,39], fld int32 [n,39], val f32 [n,39], y f32 [n] in {-1,+1}) and, with
    ``return_logit``, the planted logit [n]."""
    device = torch.device(device)
    n_int = len(CRITEO_INT_CARD)
    cards = torch.tensor([0.0] * n_int + CRITEO_CAT_CARD, dtype=torch.float64, device=device)
    F = cards.numel()
    NF = 1 << hash_bits
    gm = _gen(model_seed, device)
    w_true = torch.randn(NF, generator=gm, device=device)
    U = torch.randn(NF, planted_k, generator=gm, device=device) * 0.5
    pair_std = math.sqrt(F * (F - 1) / 2 * planted_k * 0.5 ** 4)
    bias = -1.7
    idx_out = torch.empty(n_rows, F, dtype=torch.int32, device=device)
    val_out = torch.empty(n_rows, F, dtype=torch.float32, device=device)
    y_out = torch.empty(n_rows, dtype=torch.float32, device=device)
    logit_out = torch.empty(n_rows, dtype=torch.float32, device=device) if return_logit else None
    fld_out = torch.arange(F, dtype=torch.int32, device=device).expand(n_rows, F).contiguous()
    g = _gen(seed, device)
    field_salt = (torch.arange(F, device=device, dtype=torch.int64) * 0x9E3779B1) & 0x7FFFFFFF
    is_int = torch.arange(F, device=device) < n_int
    for s in range(0, n_rows, chunk):
        e = min(n_rows, s + chunk)
        n = e - s
        u = torch.rand(n, F, generator=g, device=device, dtype=torch.float64)
        cnt = torch.floor(torch.exp2(16.0 * u * u)) - 1.0                  # integer fields: counts
        v = torch.where(is_int, cnt, torch.floor(cards * u.pow(zipf_power)))  # categorical: ids
        key = torch.where(is_int, torch.floor(4.0 * torch.log2(1.0 + v)), v).to(torch.int64)
        h = (key * 0x5BD1E995 + field_salt) & 0x7FFFFFFF
        h = ((h ^ (h >> 15)) * 0x2545F491) & 0x7FFFFFFF
        ids = (h ^ (h >> 13)) & (NF - 1)
        x = torch.where(is_int, 0.25 * torch.log2(2.0 + v), torch.ones_like(v)).to(torch.float32)
        idx_out[s:e] = ids.to(torch.int32)
        val_out[s:e] = x
        xs = x * (math.sqrt(F) / x.norm(dim=1, keepdim=True))              # normalised, mean square 1
        lin = (w_true[ids] * xs).sum(1)
        Ur = U[ids] * xs.unsqueeze(-1)                                     # [n,F,k]
        sv = Ur.sum(1)
        pair = 0.5 * ((sv * sv).sum(1) - (Ur * Ur).sum((1, 2)))
        logit = bias + lin / math.sqrt(F) + 0.7 * pair / pair_std
        p = torch.sigmoid(logit)
        y_out[s:e] = torch.where(torch.rand(n, generator=g, device=device) < p, 1.0, -1.0)
        if logit_out is not None:
            logit_out[s:e] = logit
    if return_logit:
        return idx_out, fld_out, val_out, y_out, logit_out
    return idx_out, fld_out, val_out, y_out


def criteo_like_strings(n_rows: int, hash_bits: int = 20, seed: int = 7):
    """Same data as Hivemall-style FFM feature strings ``field:index:1`` (for SQL/UDTF tests)."""
    idx, y = criteo_like(n_rows, hash_bits, seed, "cpu")
    idx = idx.numpy()
    rows = [[f"{j}:{int(i)}:1" for j, i in enumerate(r)] for r in idx]
    return rows, ((y.numpy() > 0).astype(np.int32))


def a9a_like(n_rows: int = 32561, n_features: int = 123, nnz: int = 14, seed: int = 3,
             model_seed: int = 123):
    """libsvm a9a-shaped binary data: returns (rows as list of int arrays (1-based), labels 0/1).
    The planted model depends only on ``model_seed``; ``seed`` selects the rows."""
    mrng = np.random.default_rng(model_seed)
    w = mrng.normal(0, 1.0, n_features + 1)
    pop = mrng.dirichlet(np.ones(n_features) * 0.3)
    rng = np.random.default_rng(seed)
    rows = []
    ys = np.empty(n_rows, dtype=np.int32)
    for r in range(n_rows):
        k = max(1, int(rng.normal(nnz, 1.5)))
        f = np.unique(rng.choice(n_features, size=min(k, n_features), replace=False, p=pop)) + 1
        rows.append(f.astype(np.int64))
        m = w[f].sum() - 0.8
        ys[r] = 1 if rng.random() < 1.0 / (1.0 + math.exp(-m)) else 0
    return rows, ys


def higgs_like(n_rows: int = 100000, n_features: int = 28, seed: int = 5, device="cpu"):
    """Dense HIGGS-shaped data (28 float features) with a planted non-linear rule."""
    g = _gen(seed, torch.device(device))
    X = torch.randn(n_rows, n_features, generator=g, device=device)
    X[:, 21:] = X[:, 21:].abs() + 0.5 * X[:, :7].abs()                   # "high-level" features
    logit = (1.2 * X[:, 0] * X[:, 1] - 0.8 * X[:, 2] + 0.6 * torch.tanh(2 * X[:, 3])
             + 0.9 * (X[:, 25] > 1.2).float() - 0.5 * X[:, 27] + 0.4 * X[:, 4] ** 2 - 0.4)
    y = (torch.rand(n_rows, generator=g, device=device) < torch.sigmoid(logit)).float()
    return X, y


def movielens_like(n_ratings: int = 20000263, n_users: int = 138493, n_items: int = 27278,
                   seed: int = 11, device="cpu", k: int = 16):
    """Implicit-feedback (user, item) pairs with MovieLens-20M counts; popularity is
    power-law and preferences come from a planted low-rank model."""
    device = torch.device(device)
    g = _gen(seed, device)
    P = torch.randn(n_users, k, generator=g, device=device) * 0.5
    Q = torch.randn(n_items, k, generator=g, device=device) * 0.5
    users = torch.floor(n_users * torch.rand(n_ratings, generator=g, device=device).pow(1.5)).long()
    # candidate items from popularity, accepted by planted affinity
    cand = torch.floor(n_items * torch.rand(n_ratings, 4, generator=g, device=device).pow(2.5)).long()
    score = (P[users].unsqueeze(1) * Q[cand]).sum(-1)
    best = score.argmax(1)
    items = cand.gather(1, best.unsqueeze(1)).squeeze(1)
    return users.int(), items.int()
