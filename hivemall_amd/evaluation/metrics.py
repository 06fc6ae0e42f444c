"""Evaluation UDAFs (upstream core/src/main/java/hivemall/evaluation/
{AUCUDAF,LogarithmicLossUDAF,MeanAbsoluteErrorUDAF,MeanSquaredErrorUDAF,RootMeanSquaredErrorUDAF,
R2UDAF,F1ScoreUDAF,FMeasureUDAF,PrecisionUDAF,RecallUDAF,HitRateUDAF,MRRUDAF,MAPUDAF,NDCGUDAF,
BinaryResponsesMeasures,GradedResponsesMeasures}.java).

Every metric accepts numpy arrays, Python lists or torch tensors; on ``cuda`` tensors the
reductions (and the AUC sort) run on the GPU.  ``*_partial`` / ``*_merge`` give the UDAF
partial-aggregate form used to combine ranks (the distributed ``merge`` step is an RCCL
all-reduce of the partial tensors, see parallel.mix.ModelMixer.all_reduce_sum).
"""
from __future__ import annotations

import math
from typing import Iterable, Sequence

import numpy as np
import torch

from ..registry import udaf
from ..utils.options import Options, UDFArgumentException, opt


def _t(x, dtype=torch.float64) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(dtype)
    return torch.as_tensor(np.asarray(x, dtype=np.float64), dtype=dtype)


# ------------------------------------------------------------------ binary classification
@udaf("auc")
def auc(scores, labels=None, *rest):
    """AUC.  Two forms (like upstream AUCUDAF):
    * ``auc(score double, label int)``  — binary classification ROC AUC (ties averaged);
    * ``auc(array rankItems, array groundTruth [, int recommendSize])`` — ranking AUC per row,
      averaged over the group."""
    if labels is not None and len(scores) and isinstance(_first(scores), (list, tuple, np.ndarray)):
        k = rest[0] if rest else None
        return _mean([ranking_auc(r, g, _first(k) if isinstance(k, (list, tuple)) else k)
                      for r, g in zip(scores, labels)])
    s = _t(scores)
    y = _t(labels)
    ok = ~torch.isnan(s) & ~torch.isnan(y)
    s, y = s[ok], (y[ok] > 0).to(torch.float64)
    n_pos = float(y.sum().item())
    n_neg = float(y.numel() - n_pos)
    if n_pos == 0 or n_neg == 0:
        return float("nan")
    # rank-sum (Mann-Whitney U) with average ranks for ties
    order = torch.argsort(s)
    ss = s[order]
    yy = y[order]
    n = ss.numel()
    ranks = torch.arange(1, n + 1, dtype=torch.float64, device=s.device)
    uniq, inv, counts = torch.unique_consecutive(ss, return_inverse=True, return_counts=True)
    ends = torch.cumsum(counts, 0).to(torch.float64)
    starts = ends - counts.to(torch.float64) + 1
    avg = (starts + ends) / 2
    ranks = avg[inv]
    rank_pos = float((ranks * yy).sum().item())
    return (rank_pos - n_pos * (n_pos + 1) / 2) / (n_pos * n_neg)


def _first(x):
    for v in x:
        if v is not None:
            return v
    return None


def _mean(vals):
    vals = [v for v in vals if v is not None and not (isinstance(v, float) and math.isnan(v))]
    return float(np.mean(vals)) if vals else float("nan")


def ranking_auc(rank_items: Sequence, truth: Sequence, recommend_size: int | None = None) -> float:
    """Ranking AUC of one recommendation list (BinaryResponsesMeasures.AUC)."""
    rank = list(rank_items)[: recommend_size or None]
    gt = set(truth)
    n_pos = sum(1 for r in rank if r in gt)
    n_neg = len(rank) - n_pos
    if n_pos == 0:
        return 0.0
    if n_neg == 0:
        return 1.0
    correct = 0
    neg_seen = 0
    for r in rank:
        if r in gt:
            correct += n_neg - neg_seen
        else:
            neg_seen += 1
    return correct / (n_pos * n_neg)


@udaf("logloss")
def logloss(probs, labels):
    """Logarithmic loss of predicted probabilities against 0/1 labels (eps-clipped)."""
    p = _t(probs).clamp(1e-15, 1 - 1e-15)
    y = (_t(labels) > 0).to(torch.float64)
    return float((-(y * torch.log(p) + (1 - y) * torch.log1p(-p))).mean().item())


def logloss_partial(probs, labels) -> torch.Tensor:
    p = _t(probs).clamp(1e-15, 1 - 1e-15)
    y = (_t(labels) > 0).to(torch.float64)
    return torch.stack([(-(y * torch.log(p) + (1 - y) * torch.log1p(-p))).sum(),
                        torch.tensor(float(p.numel()), dtype=torch.float64, device=p.device)])


def logloss_merge(partial: torch.Tensor) -> float:
    return float((partial[0] / partial[1]).item())


# ------------------------------------------------------------------ regression
@udaf("mae")
def mae(predicted, actual):
    return float((_t(predicted) - _t(actual)).abs().mean().item())


@udaf("mse")
def mse(predicted, actual):
    return float(((_t(predicted) - _t(actual)) ** 2).mean().item())


@udaf("rmse")
def rmse(predicted, actual):
    return math.sqrt(mse(predicted, actual))


@udaf("r2")
def r2(predicted, actual):
    """Coefficient of determination 1 - SS_res / SS_tot."""
    p, a = _t(predicted), _t(actual)
    ss_res = float(((a - p) ** 2).sum().item())
    ss_tot = float(((a - a.mean()) ** 2).sum().item())
    return 1.0 - ss_res / ss_tot if ss_tot > 0 else float("nan")


def regression_partial(predicted, actual) -> torch.Tensor:
    """[n, Σ|e|, Σe², Σa, Σa²] — mergeable by addition (mae/mse/rmse/r2)."""
    p, a = _t(predicted), _t(actual)
    e = a - p
    return torch.stack([torch.tensor(float(p.numel()), dtype=torch.float64, device=p.device),
                        e.abs().sum(), (e * e).sum(), a.sum(), (a * a).sum()])


def regression_merge(part: torch.Tensor) -> dict:
    n, sae, sse, sa, saa = [float(x) for x in part.tolist()]
    ss_tot = saa - sa * sa / n
    return {"mae": sae / n, "mse": sse / n, "rmse": math.sqrt(sse / n),
            "r2": 1 - sse / ss_tot if ss_tot > 0 else float("nan")}


# ------------------------------------------------------------------ set-based classification
def _as_set(x):
    if x is None:
        return set()
    if isinstance(x, (list, tuple, np.ndarray, set)):
        return set(np.asarray(list(x)).tolist())
    return {x}


@udaf("f1score")
def f1score(actual, predicted):
    """Micro-averaged F1 over rows of (actual labels, predicted labels) arrays."""
    tp = fp = fn = 0
    for a, p in zip(actual, predicted):
        A, P = _as_set(a), _as_set(p)
        tp += len(A & P)
        fp += len(P - A)
        fn += len(A - P)
    return 2 * tp / (2 * tp + fp + fn) if (tp + fp + fn) else 0.0


_FMEASURE_OPTS = Options([opt("beta", None, 1.0, float, "beta"),
                          opt("average", None, "micro", str, "micro | macro | binary")], "fmeasure")


@udaf("fmeasure")
def fmeasure(predicted, actual, options=None):
    """F-beta measure; ``-average micro|macro|binary`` (binary: 0/1 or boolean labels)."""
    o = options[0] if isinstance(options, (list, tuple)) else options
    cl = _FMEASURE_OPTS.parse(o)
    beta2 = cl["beta"] ** 2
    avg = cl["average"]
    if avg == "binary":
        p = np.asarray([bool(v) and v != 0 for v in predicted])
        a = np.asarray([bool(v) and v != 0 for v in actual])
        tp = float((p & a).sum())
        fp = float((p & ~a).sum())
        fn = float((~p & a).sum())
        d = (1 + beta2) * tp + beta2 * fn + fp
        return (1 + beta2) * tp / d if d else 0.0
    if avg == "micro":
        tp = fp = fn = 0
        for pr, ac in zip(predicted, actual):
            P, A = _as_set(pr), _as_set(ac)
            tp += len(A & P)
            fp += len(P - A)
            fn += len(A - P)
        d = (1 + beta2) * tp + beta2 * fn + fp
        return (1 + beta2) * tp / d if d else 0.0
    if avg == "macro":
        labels = set()
        pairs = [(_as_set(pr), _as_set(ac)) for pr, ac in zip(predicted, actual)]
        for P, A in pairs:
            labels |= P | A
        scores = []
        for lab in labels:
            tp = sum(1 for P, A in pairs if lab in P and lab in A)
            fp = sum(1 for P, A in pairs if lab in P and lab not in A)
            fn = sum(1 for P, A in pairs if lab not in P and lab in A)
            d = (1 + beta2) * tp + beta2 * fn + fp
            scores.append((1 + beta2) * tp / d if d else 0.0)
        return float(np.mean(scores)) if scores else 0.0
    raise UDFArgumentException(f"fmeasure: unknown -average {avg}")


# ------------------------------------------------------------------ ranking measures
def _k(rest):
    if not rest:
        return None
    k = rest[0]
    if isinstance(k, (list, tuple, np.ndarray)):
        k = _first(k)
    return None if k is None else int(k)


def precision_at_one(rank, truth, k=None) -> float:
    rank = list(rank)[: k or None]
    if not rank:
        return 0.0
    gt = _as_set(truth)
    return sum(1 for r in rank if r in gt) / len(rank)


def recall_at_one(rank, truth, k=None) -> float:
    rank = list(rank)[: k or None]
    gt = _as_set(truth)
    if not gt:
        return 0.0
    return sum(1 for r in rank if r in gt) / len(gt)


def hitrate_one(rank, truth, k=None) -> float:
    rank = list(rank)[: k or None]
    gt = _as_set(truth)
    return 1.0 if any(r in gt for r in rank) else 0.0


def mrr_one(rank, truth, k=None) -> float:
    gt = _as_set(truth)
    for i, r in enumerate(list(rank)[: k or None]):
        if r in gt:
            return 1.0 / (i + 1)
    return 0.0


def average_precision_one(rank, truth, k=None) -> float:
    gt = _as_set(truth)
    if not gt:
        return 0.0
    hits = 0
    s = 0.0
    for i, r in enumerate(list(rank)[: k or None]):
        if r in gt:
            hits += 1
            s += hits / (i + 1)
    return s / min(len(gt), k) if k else s / len(gt)


def ndcg_one(rank, truth, k=None) -> float:
    """Binary relevance when ``truth`` is a list of items; graded when it is a dict
    item -> relevance or a list of (item, relevance) pairs."""
    rank = list(rank)[: k or None]
    if isinstance(truth, dict):
        rel = {kk: float(v) for kk, v in truth.items()}
    elif truth is not None and len(truth) and isinstance(_first(truth), (tuple, list)):
        rel = {t[0]: float(t[1]) for t in truth}
    else:
        rel = {t: 1.0 for t in _as_set(truth)}
    dcg = sum((2 ** rel.get(r, 0.0) - 1) / math.log2(i + 2) for i, r in enumerate(rank))
    ideal = sorted(rel.values(), reverse=True)[: len(rank) if k else None]
    idcg = sum((2 ** g - 1) / math.log2(i + 2) for i, g in enumerate(ideal))
    return dcg / idcg if idcg > 0 else 0.0


def _rank_udaf(fn):
    def agg(rank_items, truth, *rest):
        k = _k(rest)
        return _mean([fn(r, g, k) for r, g in zip(rank_items, truth)])
    return agg


precision_at = udaf("precision_at", "precision")(_rank_udaf(precision_at_one))
recall_at = udaf("recall_at", "recall")(_rank_udaf(recall_at_one))
hitrate = udaf("hitrate")(_rank_udaf(hitrate_one))
mrr = udaf("mrr")(_rank_udaf(mrr_one))
average_precision = udaf("average_precision")(_rank_udaf(average_precision_one))
ndcg = udaf("ndcg")(_rank_udaf(ndcg_one))
