"""XGBoost-style second-order gradient boosting on the histogram tree engine.

Reference behaviour: upstream ``xgboost/src/main/java/hivemall/xgboost/**`` (SURVEY.md §2.1,
§2.3.6): ``train_xgboost`` (+ the older ``train_xgboost_classifier``, ``train_xgboost_regr``,
``train_multiclass_xgboost_classifier``) buffer the rows into a DMatrix and call libxgboost over
JNI; ``xgboost_predict`` / ``xgboost_predict_one`` / ``xgboost_predict_triple`` /
``xgboost_multiclass_predict`` score rows joined to the model table.

This engine does not load XGBoost.  The same objective is trained on the device by
:class:`~hivemall_amd.models.trees.HistTreeBuilder` with the ``xgb`` criterion: per-row
gradient/hessian statistics, gain ``T(G_L)^2/(H_L+λ) + T(G_R)^2/(H_R+λ) - T(G)^2/(H+λ)``
(T = L1 soft threshold by α), split only when the gain exceeds 2γ (XGBoost's γ is on half the
gain), children need hessian ≥ ``min_child_weight``, leaves ``-η·T(G)/(H+λ)``.  Histograms are
256-bin quantiles (``tree_method=hist``); with a mixer the per-level histograms are all-reduced
over RCCL (data-parallel boosting, identical trees on every rank).

Differences (docs/compat.md): the model string is this engine's JSON→Deflate→Base91 encoding,
not an XGBoost binary; absent sparse features are 0.0 (not "missing"); NaN values take the
right branch (no learned default direction).
"""
from __future__ import annotations

import json
import math
import zlib

import ctypes as C

import numpy as np
import pandas as pd
import torch

from .. import _native
from ..registry import udtf
from ..utils import base91
from ..utils.options import UDFArgumentException, opt
from .base import Learner
from .trees import (HistTreeBuilder, PendingTree, Tree, _encode_classes_dp, _to_dense, materialize_trees,
                    predict_forest, quantize)

XGB_OPTS = [
    opt("objective", None, "binary:logistic", str,
        "binary:logistic | reg:logistic | reg:squarederror (reg:linear) | multi:softprob | multi:softmax"),
    opt("num_round", "iters", 10, int, "Number of boosting rounds", aliases=("num_boost_round",)),
    opt("eta", "learning_rate", 0.3, float, "Shrinkage"),
    opt("max_depth", None, 6, int, "Maximum tree depth"),
    opt("min_child_weight", None, 1.0, float, "Minimum hessian sum in a child"),
    opt("gamma", "min_split_loss", 0.0, float, "Minimum loss reduction to split"),
    opt("lambda", "reg_lambda", 1.0, float, "L2 on leaf weights"),
    opt("alpha", "reg_alpha", 0.0, float, "L1 on leaf weights"),
    opt("subsample", None, 1.0, float, "Row subsampling per round"),
    opt("colsample_bytree", None, 1.0, float, "Feature subsampling per tree"),
    opt("colsample_bynode", None, 1.0, float, "Feature subsampling per split"),
    opt("num_class", None, None, int, "Number of classes (multi:*)"),
    opt("base_score", None, 0.5, float, "Initial prediction (probability for logistic objectives)"),
    opt("max_leaves", None, None, int, "Maximum leaves per tree"),
    opt("seed", None, 43, int, "Seed"),
    opt("num_bins", "max_bin", 256, int, "[engine] histogram bins (<= 256)"),
    opt("booster", None, "gbtree", str, "gbtree (only)"),
    opt("tree_method", None, "hist", str, "Accepted; always histogram"),
    opt("eval_metric", None, None, str, "Accepted"),
    opt("silent", None, None, str, "Accepted"),
]

_OBJ_ALIASES = {"reg:linear": "reg:squarederror", "binary:logitraw": "binary:logistic"}


class XGBoostTrainer(Learner):
    SQL_DP = "shard"
    NAME = "train_xgboost"
    OPTIONS = XGB_OPTS
    DEFAULT_OBJECTIVE = None

    def __init__(self, options=None, device=None, **kw):
        super().__init__(options, device, **kw)
        obj = self.cl["objective"]
        if self.DEFAULT_OBJECTIVE and (options is None or "-objective" not in str(options)):
            obj = self.DEFAULT_OBJECTIVE
        self.objective = _OBJ_ALIASES.get(obj, obj)
        if self.objective not in ("binary:logistic", "reg:logistic", "reg:squarederror",
                                  "multi:softprob", "multi:softmax"):
            raise UDFArgumentException(f"{self.NAME}: unsupported objective {obj}")
        if self.cl["booster"] != "gbtree":
            raise UDFArgumentException(f"{self.NAME}: only -booster gbtree is supported")
        self.trees: list[list[Tree]] = []
        self.classes = None
        self.base_margin: list[float] = []
        self.K = 1

    # -- objective
    def _grad(self, F: torch.Tensor, Y: torch.Tensor):
        if self.objective in ("binary:logistic", "reg:logistic"):
            p = torch.sigmoid(F)
            return p - Y, (p * (1 - p)).clamp_min(1e-16)
        if self.objective == "reg:squarederror":
            return F - Y, torch.ones_like(F)
        p = torch.softmax(F, 1)
        return p - Y, (2.0 * p * (1 - p)).clamp_min(1e-16)

    def fit(self, features, labels):
        c = self.cl
        dev = self.device
        X = features if torch.is_tensor(features) else torch.from_numpy(_to_dense(features))
        X = X.float().to(dev)
        n, d = X.shape
        lab = labels if torch.is_tensor(labels) else torch.as_tensor(np.asarray(labels, dtype=np.float64))
        lab = lab.to(dev)
        if self.objective.startswith("multi:"):
            self.classes, yi = _encode_classes_dp(lab, self.mixer)
            yi = yi.to(dev)
            self.K = int(c["num_class"] or len(self.classes))
            if len(self.classes) > self.K:
                raise UDFArgumentException(f"{self.NAME}: more labels than -num_class")
            Y = torch.nn.functional.one_hot(yi, self.K).float()
            self.base_margin = [0.0] * self.K
        else:
            y = lab.float()
            if self.objective == "binary:logistic":
                y = (y > 0).float()          # accepts 0/1 and -1/+1
                self.classes = [0, 1]
            Y = y[:, None]
            bs = float(c["base_score"])
            if self.objective in ("binary:logistic", "reg:logistic"):
                bs = min(max(bs, 1e-6), 1 - 1e-6)
                self.base_margin = [math.log(bs / (1 - bs))]
            else:
                self.base_margin = [bs]
        # NaN = missing: the last bin is reserved for it and every split learns where missing
        # rows go (XGBoost's sparsity-aware default direction; tree JSON field "m")
        has_nan = bool(torch.isnan(X).any().item())
        if self.mixer is not None and self.mixer.world > 1:
            has_nan = self.mixer.all_reduce_scalar(float(has_nan), "max") > 0
        q = quantize(X, min(256, int(c["num_bins"])), seed=self.seed, mixer=self.mixer, missing=has_nan,
                     edges=self.kw.get("edges"))
        F = torch.tensor(self.base_margin, device=dev).repeat(n, 1)
        g = torch.Generator(device=dev).manual_seed(self.seed)
        gcpu = torch.Generator().manual_seed(self.seed)
        eta = float(c["eta"])
        m_sub = max(1, int(round(n * float(c["subsample"]))))
        ncol = max(1, int(round(d * float(c["colsample_bytree"]))))
        mtry = None
        if float(c["colsample_bynode"]) < 1.0:
            mtry = max(1, int(round(ncol * float(c["colsample_bynode"]))))
        self.importance = np.zeros(d)
        # binary logistic on the GPU: the round's (g, h) and |max| in one fused kernel
        fused = F.is_cuda and self.K == 1 and self.objective in ("binary:logistic", "reg:logistic")
        if fused:
            y1 = Y[:, 0].contiguous()
            stats_buf = torch.empty((n, 2), dtype=torch.float32, device=dev)
            smax = torch.zeros(2, dtype=torch.float32, device=dev)
            all_rows = torch.arange(n, dtype=torch.int32, device=dev)
        imp_dev = None
        for it in range(int(c["num_round"])):
            if fused:
                mask = None
                if m_sub < n:
                    sel = torch.randperm(n, generator=g, device=dev)[:m_sub]
                    mask = torch.zeros(n, dtype=torch.bool, device=dev)
                    mask[sel] = True
                smax.zero_()
                _native.check(_native.hip().hm_xgb_stats(
                    _native.ptr(F), _native.ptr(y1), _native.ptr(mask), C.c_int64(n), _native.ptr(stats_buf),
                    _native.ptr(smax), _native.stream_of(dev)), "hm_xgb_stats")
            else:
                Gr, Hs = self._grad(F, Y)
            if not fused and m_sub < n:
                sel = torch.randperm(n, generator=g, device=dev)[:m_sub]
                w = torch.zeros(n, device=dev)
                w[sel] = 1.0
                Gr, Hs = Gr * w[:, None], Hs * w[:, None]
            fmask = None
            if ncol < d:
                fmask = torch.zeros(d, dtype=torch.bool)
                fmask[torch.randperm(d, generator=gcpu)[:ncol]] = True
            round_trees = []
            for k in range(self.K):
                stats = stats_buf if fused else torch.stack([Gr[:, k], Hs[:, k]], 1).contiguous()
                b = HistTreeBuilder(q, "xgb", int(c["max_depth"]), 2 * float(c["min_child_weight"]),
                                    float(c["min_child_weight"]), mtry, c["max_leaves"],
                                    seed=self.seed * 7919 + it * self.K + k, mixer=self.mixer,
                                    lam=float(c["lambda"]), alpha=float(c["alpha"]),
                                    min_gain=2.0 * float(c["gamma"]), feature_mask=fmask)
                if fused:
                    tree = b.build(stats, smax=smax, act_rows=all_rows if mask is None else None,
                                   identity_rows=mask is None, defer=True)
                else:
                    tree = b.build(stats)
                if isinstance(tree, PendingTree):       # node arrays still on the device
                    tree.scale = eta
                else:
                    tree.value = [None if v is None else [eta * v[0]] for v in tree.value]
                if F.is_cuda:   # fused leaf update (trees.hip gbt_apply_kernel)
                    vals = b.node_values.float().contiguous()
                    _native.check(_native.hip().hm_gbt_apply(
                        _native.ptr(F), F.shape[1], k, _native.ptr(vals), vals.shape[1], _native.ptr(b.leaf_of_row),
                        C.c_int64(n), C.c_float(eta), int(b.leaf_of_row.dtype == torch.int16),
                        _native.stream_of(F.device)), "hm_gbt_apply")
                else:
                    F[:, k] += eta * b.node_values[b.leaf_of_row.long(), 0]
                if isinstance(tree, PendingTree):
                    imp_dev = b.imp_dev if imp_dev is None else imp_dev + b.imp_dev
                else:
                    self.importance += b.importance
                round_trees.append(tree)
            self.trees.append(round_trees)
        self.trees = materialize_trees(self.trees)
        if imp_dev is not None:
            self.importance += imp_dev.cpu().numpy()
        return self

    # -- inference
    def margin(self, features) -> torch.Tensor:
        X = features if torch.is_tensor(features) else torch.from_numpy(_to_dense(features))
        return _margin(self._model_dict(), X.float().to(self.device))

    def predict_proba(self, features) -> np.ndarray:
        return _transform(self.objective, self.margin(features)).cpu().numpy()

    def predict(self, features) -> np.ndarray:
        p = self.predict_proba(features)
        if self.objective.startswith("multi:"):
            return np.asarray(self.classes)[p.argmax(1)]
        if self.objective == "binary:logistic":
            return (p[:, 0] > 0.5).astype(np.int64)
        return p[:, 0]

    def _model_dict(self) -> dict:
        return {"v": 1, "objective": self.objective, "K": self.K, "base_margin": self.base_margin,
                "classes": self.classes,
                "trees": [[t.to_json() for t in rt] for rt in self.trees]}

    def model_table(self) -> pd.DataFrame:
        s = base91.encode(zlib.compress(json.dumps(self._model_dict(), separators=(",", ":")).encode()))
        return pd.DataFrame([(f"xgb-{0 if self._dp() else self.rank}-{self.seed}", s)], columns=["model_id", "model"])


class XGBoostClassifier(XGBoostTrainer):
    NAME = "train_xgboost_classifier"
    DEFAULT_OBJECTIVE = "binary:logistic"


class XGBoostRegressor(XGBoostTrainer):
    NAME = "train_xgboost_regr"
    DEFAULT_OBJECTIVE = "reg:squarederror"


class XGBoostMulticlass(XGBoostTrainer):
    NAME = "train_multiclass_xgboost_classifier"
    DEFAULT_OBJECTIVE = "multi:softprob"


# ------------------------------------------------------------------ model strings / scoring
_CACHE: dict = {}


def load_model(model: str) -> dict:
    key = hash(model)
    m = _CACHE.get(key)
    if m is None:
        m = json.loads(zlib.decompress(base91.decode(model)).decode())
        m["_trees"] = [[Tree.from_json(t) for t in rt] for rt in m["trees"]]
        if len(_CACHE) > 256:
            _CACHE.clear()
        _CACHE[key] = m
    return m


def _margin(m: dict, X: torch.Tensor) -> torch.Tensor:
    trees = m["_trees"] if "_trees" in m else [[Tree.from_json(t) for t in rt] for rt in m["trees"]]
    K = int(m["K"])
    F = torch.tensor(m["base_margin"], dtype=torch.float32, device=X.device).repeat(X.shape[0], 1)
    for k in range(K):
        ts = [rt[k] for rt in trees]
        if ts:
            F[:, k] += predict_forest(ts, X)[:, 0]
    return F


def _transform(objective: str, F: torch.Tensor) -> torch.Tensor:
    if objective in ("binary:logistic", "reg:logistic"):
        return torch.sigmoid(F)
    if objective.startswith("multi:"):
        return torch.softmax(F, 1)
    return F


def _batched(rowid, features, model_id, model, session=None):
    """Group the joined rows by model and score each group with one batched traversal."""
    dev = getattr(session, "device", None) or "cpu"
    groups: dict = {}
    for i, mid in enumerate(model_id):
        groups.setdefault((mid, model[i]), []).append(i)
    for (mid, ms), idxs in groups.items():
        m = load_model(ms)
        X = torch.from_numpy(_to_dense([features[i] for i in idxs])).to(dev)
        P = _transform(m["objective"], _margin(m, X)).cpu().numpy()
        yield m, [rowid[i] for i in idxs], P


def _udtf(name, cols, fn):
    fn.wants_session = True
    udtf(name, per_row=False, cols=cols)(fn)


def xgboost_predict(rowid, features, model_id, model, options=None, session=None):
    """(rowid, predicted array<double>): probabilities (classification) or values."""
    rows = []
    for m, rids, P in _batched(rowid, features, model_id, model, session):
        rows += [(r, P[j].tolist()) for j, r in enumerate(rids)]
    return pd.DataFrame(rows, columns=["rowid", "predicted"])


def xgboost_predict_one(rowid, features, model_id, model, options=None, session=None):
    """(rowid, predicted double): P(y=1) for binary objectives, the value for regression."""
    rows = []
    for m, rids, P in _batched(rowid, features, model_id, model, session):
        if P.shape[1] != 1:
            raise UDFArgumentException("xgboost_predict_one: use xgboost_predict_triple for multiclass")
        rows += [(r, float(P[j, 0])) for j, r in enumerate(rids)]
    return pd.DataFrame(rows, columns=["rowid", "predicted"])


def xgboost_predict_triple(rowid, features, model_id, model, options=None, session=None):
    """(rowid, label, probability): one row per class."""
    rows = []
    for m, rids, P in _batched(rowid, features, model_id, model, session):
        classes = m.get("classes") or list(range(P.shape[1]))
        if P.shape[1] == 1:
            P = np.concatenate([1 - P, P], 1)
        for j, r in enumerate(rids):
            rows += [(r, str(classes[k]), float(P[j, k])) for k in range(P.shape[1])]
    return pd.DataFrame(rows, columns=["rowid", "label", "probability"])


_udtf("xgboost_predict", ("rowid", "predicted"), xgboost_predict)
_udtf("xgboost_predict_one", ("rowid", "predicted"), xgboost_predict_one)
_udtf("xgboost_predict_triple", ("rowid", "label", "probability"), xgboost_predict_triple)
_udtf("xgboost_multiclass_predict", ("rowid", "label", "probability"), xgboost_predict_triple)


def register_sql(reg):
    reg("train_xgboost", lambda: XGBoostTrainer)
    reg("train_xgboost_classifier", lambda: XGBoostClassifier)
    reg("train_xgboost_regr", lambda: XGBoostRegressor)
    reg("train_multiclass_xgboost_classifier", lambda: XGBoostMulticlass)
