"""Similarity / distance / LSH / top-k (upstream core/src/main/java/hivemall/
knn/{similarity,distance,lsh}/*.java, tools/EachTopKUDTF.java).

Row-wise functions take Hivemall feature arrays (``"name:value"`` strings, or plain numeric
arrays for the dense forms).  ``pairwise_cosine`` / ``topk_similar`` are the batched device
paths: an MFMA-backed GEMM (torch.matmul on ROCm -> hipBLASLt) over L2-normalised dense
matrices followed by ``torch.topk``.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..registry import udf, udtf
from ..utils.hashing import murmurhash3


def _fv(x) -> dict:
    """Feature array -> {name: value}."""
    if x is None:
        return {}
    if isinstance(x, dict):
        return {k: float(v) for k, v in x.items()}
    out = {}
    for i, f in enumerate(x):
        if isinstance(f, str):
            p = f.find(":")
            if p < 0:
                out[f] = 1.0
            else:
                out[f[:p]] = float(f[p + 1:])
        elif isinstance(f, (int, np.integer)) and not isinstance(f, bool):
            out[int(f)] = 1.0
        else:
            out[i] = float(f)
    return out


def _dense_pair(a, b):
    if a is not None and len(a) and not isinstance(list(a)[0], str):
        return np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return None


# ------------------------------------------------------------------ similarity
@udf("cosine_similarity", "cosine_sim")
def cosine_similarity(a, b):
    A, B = _fv(a), _fv(b)
    dot = sum(v * B.get(k, 0.0) for k, v in A.items())
    na = math.sqrt(sum(v * v for v in A.values()))
    nb = math.sqrt(sum(v * v for v in B.values()))
    return dot / (na * nb) if na > 0 and nb > 0 else 0.0


@udf("jaccard_similarity")
def jaccard_similarity(a, b, k: int = 128):
    """Jaccard of two feature sets (or of two minhash signature arrays of length k)."""
    if a is None or b is None:
        return 0.0
    if len(a) and isinstance(list(a)[0], (int, np.integer)) and len(a) == len(b) and len(a) == k:
        return float(np.mean(np.asarray(a) == np.asarray(b)))
    A, B = set(_fv(a)), set(_fv(b))
    u = len(A | B)
    return len(A & B) / u if u else 0.0


@udf("angular_similarity")
def angular_similarity(a, b):
    c = max(-1.0, min(1.0, cosine_similarity(a, b)))
    return 1.0 - math.acos(c) / math.pi


@udf("euclid_similarity")
def euclid_similarity(a, b):
    return 1.0 / (1.0 + euclid_distance(a, b))


@udf("distance2similarity")
def distance2similarity(d):
    return 1.0 / (1.0 + float(d))


@udtf("dimsum_mapper", per_row=True, cols=("j", "k", "b_jk"))
def dimsum_mapper(row, col_norms, options=None):
    """DIMSUM all-pairs similarity mapper: emits (j, k, a_ij*a_ik / (|c_j||c_k|)) sampled with
    probability min(1, γ / (|c_j||c_k|)); ``-threshold`` sets γ = 4·log(n)/threshold."""
    import random
    gamma = 1e30
    if options:
        toks = str(options).split()
        if "-threshold" in toks:
            t = float(toks[toks.index("-threshold") + 1])
            gamma = 4.0 * math.log(max(2, len(col_norms))) / t
    R = _fv(row)
    items = sorted(R.items(), key=lambda kv: str(kv[0]))
    rng = random.Random(42)
    for ai, (j, vj) in enumerate(items):
        nj = float(col_norms.get(j, 0.0)) if isinstance(col_norms, dict) else 0.0
        if nj == 0:
            continue
        for k, vk in items[ai + 1:]:
            nk = float(col_norms.get(k, 0.0))
            if nk == 0:
                continue
            p = min(1.0, gamma / (nj * nk))
            if rng.random() < p:
                yield (j, k, vj * vk / (min(math.sqrt(gamma), nj) * min(math.sqrt(gamma), nk)))


# ------------------------------------------------------------------ distance
@udf("euclid_distance")
def euclid_distance(a, b):
    d = _dense_pair(a, b)
    if d is not None:
        return float(np.linalg.norm(d[0] - d[1]))
    A, B = _fv(a), _fv(b)
    keys = set(A) | set(B)
    return math.sqrt(sum((A.get(k, 0.0) - B.get(k, 0.0)) ** 2 for k in keys))


@udf("cosine_distance")
def cosine_distance(a, b):
    return 1.0 - cosine_similarity(a, b)


@udf("angular_distance")
def angular_distance(a, b):
    return 1.0 - angular_similarity(a, b)


@udf("manhattan_distance")
def manhattan_distance(a, b):
    d = _dense_pair(a, b)
    if d is not None:
        return float(np.abs(d[0] - d[1]).sum())
    A, B = _fv(a), _fv(b)
    return sum(abs(A.get(k, 0.0) - B.get(k, 0.0)) for k in set(A) | set(B))


@udf("minkowski_distance")
def minkowski_distance(a, b, p: float):
    p = float(p)
    A, B = _fv(a), _fv(b)
    s = sum(abs(A.get(k, 0.0) - B.get(k, 0.0)) ** p for k in set(A) | set(B))
    return s ** (1.0 / p)


@udf("jaccard_distance")
def jaccard_distance(a, b, k: int = 128):
    return 1.0 - jaccard_similarity(a, b, k)


@udf("hamming_distance")
def hamming_distance(a, b):
    """Bit differences of two ints or of two long arrays (bitsets)."""
    if isinstance(a, (int, np.integer)):
        return bin((int(a) ^ int(b)) & ((1 << 64) - 1)).count("1")
    return sum(bin((int(x) ^ int(y)) & ((1 << 64) - 1)).count("1") for x, y in zip(a, b))


@udf("popcnt")
def popcnt(a):
    if isinstance(a, (int, np.integer)):
        return bin(int(a) & ((1 << 64) - 1)).count("1")
    return sum(bin(int(x) & ((1 << 64) - 1)).count("1") for x in a)


@udf("kld")
def kld(mu1, sigma1, mu2, sigma2):
    """KL divergence between two univariate Gaussians N(mu1, sigma1) || N(mu2, sigma2)
    (sigma = variance)."""
    return 0.5 * (math.log(sigma2 / sigma1) + sigma1 / sigma2 + (mu1 - mu2) ** 2 / sigma2 - 1.0)


# ------------------------------------------------------------------ LSH
def _minhash_values(features, num_hashes: int, key_groups: int, seed0: int = 0):
    F = _fv(features)
    names = [str(k) for k in F]
    sig = []
    for h in range(num_hashes):
        m = None
        for n in names:
            v = murmurhash3(n, seed=seed0 + h) & 0xFFFFFFFF
            if m is None or v < m:
                m = v
        sig.append(m if m is not None else 0)
    return sig


@udf("minhashes")
def minhashes(features, no_weight: bool = False, num_hashes: int = 5, key_groups: int = 2):
    """Minhash signature (``num_hashes`` groups of ``key_groups`` concatenated hashes)."""
    sig = _minhash_values(features, int(num_hashes) * int(key_groups), int(key_groups))
    kg = int(key_groups)
    out = []
    for g in range(int(num_hashes)):
        part = sig[g * kg:(g + 1) * kg]
        h = 0
        for v in part:
            h = (h * 31 + v) & 0x7FFFFFFF
        out.append(h)
    return out


@udtf("minhash", per_row=True, cols=("clusterid", "item"))
def minhash(item, features, options=None):
    """Emit (clusterid, item) for every minhash group of the item's features."""
    nh, kg = 5, 2
    if options:
        toks = str(options).split()
        if "-n" in toks:
            nh = int(toks[toks.index("-n") + 1])
        if "-k" in toks:
            kg = int(toks[toks.index("-k") + 1])
    for c in minhashes(features, False, nh, kg):
        yield (c, item)


@udf("bbit_minhash")
def bbit_minhash(features, num_hashes: int = 128, b: int = 1):
    """b-bit minwise hashing: the lowest ``b`` bits of each of ``num_hashes`` minhashes packed
    into a hex string."""
    sig = _minhash_values(features, int(num_hashes), 1)
    bits = 0
    for i, v in enumerate(sig):
        bits |= (v & ((1 << int(b)) - 1)) << (i * int(b))
    return format(bits, "x")


# ------------------------------------------------------------------ top-k
@udtf("each_top_k", per_row=False)
def each_top_k(k, group, score, *cols):
    """Top-|k| rows by ``score`` within each consecutive ``group`` (k < 0: bottom-k).
    Output columns: (rank, key(=score), cols...)."""
    import pandas as pd
    kk = int(k[0] if isinstance(k, (list, tuple)) else k)
    rev = kk > 0
    kk = abs(kk)
    rows = []
    n = len(group)
    order = {}
    for i in range(n):
        order.setdefault(group[i], []).append(i)
    for g, idxs in order.items():
        idxs = sorted(idxs, key=lambda i: score[i], reverse=rev)[:kk]
        for r, i in enumerate(idxs, start=1):
            rows.append((r, score[i]) + tuple(c[i] for c in cols))
    return pd.DataFrame(rows, columns=["rank", "key"] + [f"c{i}" for i in range(len(cols))])


def topk_similar(X: torch.Tensor, Y: torch.Tensor | None = None, k: int = 10):
    """Batched cosine top-k on the device: (scores, indices) of the k most similar rows of Y
    for every row of X (self-matches excluded when Y is None)."""
    Xn = torch.nn.functional.normalize(X.float(), dim=1)
    Yn = Xn if Y is None else torch.nn.functional.normalize(Y.float(), dim=1)
    if k <= 64 and Xn.shape[1] <= 256:
        # fused MFMA similarity + running top-k (ops/topk_mips.py): no N x N matrix in HBM
        from ..ops.topk_mips import mips_topk

        ix, sc = mips_topk(Xn, Yn, min(k, Yn.shape[0]), exclude_self_offset=0 if Y is None else None)
        return sc, ix
    dt = torch.bfloat16 if X.is_cuda else torch.float32
    S = (Xn.to(dt) @ Yn.to(dt).T).float()
    if Y is None:
        S.fill_diagonal_(-float("inf"))
    return torch.topk(S, min(k, S.shape[1]), dim=1)
