"""Random forests and gradient tree boosting on quantised histograms.

Reference behaviour: Hivemall's Smile-derived learners (upstream core/src/main/java/hivemall/
smile/classification/{RandomForestClassifierUDTF,GradientTreeBoostingClassifierUDTF,
DecisionTree}.java, smile/regression/{RandomForestRegressionUDTF,RegressionTree}.java,
smile/tools/{TreePredictUDF,RandomForestEnsembleUDAF,GuessAttributesUDF,TreeExportUDF}.java,
xgboost/**).

Algorithm change (documented in docs/compat.md): upstream grows trees with exact splits on
pre-sorted columns; here features are quantised to <= 256 bins and every tree level is one
LDS-privatised histogram kernel (csrc/kernels/trees.hip) + a vectorised split search on the
device.  Parity is accuracy / logloss parity, not tree identity.  The model string is our own
versioned encoding (JSON -> Deflate -> Base91): Java-serialised upstream models cannot be read.

Distributed: ``GradientTreeBoosting`` all-reduces the per-level histograms over RCCL when a
mixer is given (data parallel boosting); ``RandomForest`` splits its trees over the ranks.
"""
from __future__ import annotations

import ctypes as C
import gc
import json
import math
import os
import zlib
from dataclasses import dataclass, field

import numpy as np
import pandas as pd
import torch

from .. import _native
from ..registry import udaf, udf
from ..utils import base91
from ..utils.options import UDFArgumentException, flag, opt
from .base import Learner, log

MODEL_VERSION = 1
CAT_FLAG = 1 << 30   # nominal split flag in flattened node arrays (HM_TREE_CAT in trees.hip)
DLEFT_FLAG = 1 << 29  # missing values go left at this split (HM_TREE_DLEFT)
HIST_BLOCKS = 256    # histogram grid (blocks per feature group); benchmarks/hist_sweep.py, profiles/hist_sweep_r1.jsonl
HIST_WIDE = os.environ.get("HM_HIST_WIDE", "1") == "1"   # all-features single-pass histogram
ROUTE_FUSED = os.environ.get("HM_ROUTE_FUSED", "1") == "1"  # route + small-child count in one pass
ROUTE_COLS = os.environ.get("HM_ROUTE_COLS", "1") == "1"    # routing reads a feature-major bins copy
# heap trees: the last level's leaf statistics from the split search, not from histograms
LAST_FROM_SPLITS = os.environ.get("HM_TREE_LAST_FROM_SPLITS", "1") == "1"
ROUTE_GRID = int(os.environ.get("HM_ROUTE_GRID", "2048"))   # blocks of the fused route + count pass
GBT2 = os.environ.get("HM_GBT2", "1") == "1"    # GBT histograms of (r, w), Newton leaves summed per leaf
HEAP_TREES = os.environ.get("HM_TREE_HEAP", "1") == "1"   # fixed-shape levels, no per-level host read
HEAP_MAX_DEPTH = 10
HIST_WIDE_BLOCKS = int(os.environ.get("HM_HIST_WIDE_BLOCKS", "256"))


# ------------------------------------------------------------------ quantisation
def parse_attrs(spec, d: int) -> torch.Tensor | None:
    """``-attrs Q,C,Q`` (or ``QCQ``; Q = quantitative, C = categorical/nominal) -> bool [d] mask
    of the nominal columns, None when every column is quantitative (Smile's attribute types,
    SURVEY.md §2.3.6)."""
    if not spec:
        return None
    t = str(spec).replace(",", "").replace(" ", "").upper()
    if len(t) != d or any(c not in "QC" for c in t):
        raise UDFArgumentException(f"-attrs needs one of Q/C for each of the {d} columns: {spec!r}")
    m = torch.tensor([c == "C" for c in t])
    return m if bool(m.any()) else None


@dataclass
class Quantized:
    bins: torch.Tensor        # uint8 [n, dpad]
    edges: torch.Tensor       # f32 [d, B-1]
    d: int
    B: int
    cat: torch.Tensor | None = None   # bool [d]: nominal columns (bin = category index)
    missing: bool = False             # bin B-1 holds exactly the NaN values
    _bins_t: torch.Tensor | None = field(default=None, repr=False)

    @property
    def dpad(self) -> int:
        return self.bins.shape[1]

    def route_src(self):
        """(bins pointer, column stride) for the routing kernels: the feature-major copy
        [d, n] on a GPU (built once per matrix; a wave's rows then read one 64-B run per distinct
        split feature instead of their whole 32-B rows), else row-major (stride 0)."""
        if not (ROUTE_COLS and self.bins.is_cuda):
            return _native.ptr(self.bins), 0
        if self._bins_t is None:
            self._bins_t = self.bins[:, : self.d].t().contiguous()
        return _native.ptr(self._bins_t), self.bins.shape[0]


def quantize(X: torch.Tensor, num_bins: int = 256, sample: int = 200_000, seed: int = 0,
             edges: torch.Tensor | None = None, mixer=None,
             categorical: torch.Tensor | None = None, missing: bool = False) -> Quantized:
    """Per-feature quantile edges (from a row sample) and uint8 bins on X's device.

    With a mixer over several ranks every rank contributes an equal-size sample of its shard and
    the edges are computed from the all-gathered sample, so all ranks bin identically (required
    by the histogram all-reduce of data-parallel boosting).

    Nominal columns (``categorical`` mask) get their sorted distinct values as edges, so a
    category's bin is its index (exact, at most ``num_bins - 1`` categories; NaN takes the last
    bin)."""
    X = X.float().contiguous()
    n, d = X.shape
    B = int(num_bins)
    if edges is None:
        world = mixer.world if mixer is not None else 1
        g = torch.Generator(device="cpu").manual_seed(seed + 7919 * (mixer.ctx.rank if world > 1 else 0))
        if world > 1:
            m = max(1, sample // world)
            idx = torch.randint(0, n, (m,), generator=g).to(X.device)
            S = mixer.all_gather_cat(X[idx])
        else:
            idx = (torch.arange(n) if n <= sample else torch.randint(0, n, (sample,), generator=g)).to(X.device)
            S = X[idx]
        qs = torch.linspace(0, 1, (B if missing else B + 1), device=X.device)[1:-1]
        St = S.T.contiguous()
        E = (torch.nanquantile(St, qs, dim=1) if missing else torch.quantile(St, qs, dim=1)).T.contiguous()
        E = torch.nan_to_num(E, nan=float("inf"))
        if missing:                      # [d, B-2] edges + inf: finite values never reach bin B-1
            E = torch.cat([E, torch.full((d, 1), float("inf"), device=X.device)], 1)
        # strictly increasing edges (ties collapse to the same bin)
        if categorical is not None:
            for j in torch.nonzero(categorical).flatten().tolist():
                col = X[:, j]
                u = torch.unique(col[~torch.isnan(col)])
                if world > 1:      # every rank needs the union of the categories
                    pad = torch.full((1, B - 1), float("inf"), device=X.device)
                    pad[0, : min(B - 1, u.numel())] = u[: B - 1]
                    u = torch.unique(mixer.all_gather_cat(pad))
                    u = u[torch.isfinite(u)]
                if u.numel() > B - 1:
                    raise UDFArgumentException(
                        f"nominal column {j} has {u.numel()} distinct values (at most {B - 1})")
                row = torch.full((B - 1,), float("inf"), device=X.device)
                row[: u.numel()] = u
                E[j] = row
        edges = E.contiguous()
    dpad = (d + 15) // 16 * 16   # 16-byte rows: a feature group is one aligned load
    bins = torch.zeros((n, dpad), dtype=torch.uint8, device=X.device)
    p = _native.ptr
    args = (p(X), C.c_int64(n), d, dpad, p(edges), edges.shape[1], p(bins))
    if X.is_cuda:
        _native.check(_native.hip().hm_quantize(*args, _native.stream_of(X.device)), "hm_quantize")
    else:
        _native.host().hm_quantize_cpu(*args)
    cat = None if categorical is None else categorical.to(torch.bool).cpu()
    return Quantized(bins, edges, d, B, cat, bool(missing) and edges.shape[1] == B - 1)


# ------------------------------------------------------------------ trees
@dataclass
class Tree:
    feature: list = field(default_factory=list)     # -1 = leaf
    threshold: list = field(default_factory=list)   # go left when x <= threshold
    left: list = field(default_factory=list)
    right: list = field(default_factory=list)
    value: list = field(default_factory=list)       # list of floats per node (leaf output)
    n_out: int = 1
    cat: list = field(default_factory=list)         # 1 = nominal node: left when x == threshold
    dleft: list = field(default_factory=list)       # 1 = missing (NaN) goes left (learned default)

    def is_cat(self, k: int) -> bool:
        return bool(self.cat) and bool(self.cat[k])

    def goes_left(self, k: int, v) -> bool:
        """Smile's test: ``x <= t`` (ordinal) / ``x == t`` (nominal); missing/NaN goes right
        unless the split learned a default direction (XGBoost-style, ``dleft``)."""
        if v is None or (isinstance(v, float) and math.isnan(v)):
            return bool(self.dleft) and bool(self.dleft[k])
        return v == self.threshold[k] if self.is_cat(k) else v <= self.threshold[k]

    def to_json(self) -> dict:
        j = {"v": MODEL_VERSION, "f": self.feature,
             "t": [None if not math.isfinite(x) else x for x in self.threshold],
             "l": self.left, "r": self.right, "val": self.value, "o": self.n_out}
        if any(self.cat):
            j["c"] = self.cat
        if any(self.dleft):
            j["m"] = self.dleft
        return j

    @staticmethod
    def from_json(j: dict) -> "Tree":
        return Tree(j["f"], [math.inf if x is None else x for x in j["t"]], j["l"], j["r"], j["val"],
                    j["o"], list(j.get("c", [])), list(j.get("m", [])))

    def serialize(self) -> str:
        return base91.encode(zlib.compress(json.dumps(self.to_json(), separators=(",", ":")).encode()))

    @staticmethod
    def deserialize(s: str) -> "Tree":
        return Tree.from_json(json.loads(zlib.decompress(base91.decode(s)).decode()))

    def predict_one(self, x) -> list:
        k = 0
        while self.feature[k] >= 0:
            # missing / NaN goes right, as in Smile's `x <= t ? trueChild : falseChild`, unless
            # the split learned a default direction
            k = self.left[k] if self.goes_left(k, x[self.feature[k]]) else self.right[k]
        return self.value[k]

    def depth(self) -> int:
        def rec(k):
            return 0 if self.feature[k] < 0 else 1 + max(rec(self.left[k]), rec(self.right[k]))
        return rec(0)


def flatten(trees: list[Tree], device) -> dict:
    feat, thr, lft, rgt, voff, vals, roots = [], [], [], [], [], [], []
    base = 0
    for t in trees:
        roots.append(base)
        for k in range(len(t.feature)):
            fk = t.feature[k]
            if fk >= 0:
                fk |= (CAT_FLAG if t.is_cat(k) else 0) | (DLEFT_FLAG if (t.dleft and t.dleft[k]) else 0)
            feat.append(fk)
            thr.append(t.threshold[k] if math.isfinite(t.threshold[k]) else 3.4e38)
            lft.append(t.left[k] + base if t.feature[k] >= 0 else 0)
            rgt.append(t.right[k] + base if t.feature[k] >= 0 else 0)
            voff.append(len(vals))
            v = t.value[k] if t.value[k] is not None else [0.0] * t.n_out
            vals.extend(list(v) + [0.0] * (t.n_out - len(v)))
        base += len(t.feature)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=device)
    return dict(feature=i32(feat), threshold=torch.tensor(thr, dtype=torch.float32, device=device),
                left=i32(lft), right=i32(rgt), voff=i32(voff),
                values=torch.tensor(vals, dtype=torch.float32, device=device), roots=i32(roots),
                n_out=trees[0].n_out if trees else 1)


def predict_forest(trees: list[Tree], X: torch.Tensor, sum_trees: bool = True,
                   weights: list | None = None) -> torch.Tensor:
    """Batched traversal kernel: [n, n_out] (summed) or [n, T, n_out]."""
    X = X.float().contiguous()
    n, d = X.shape
    fl = flatten(trees, X.device)
    T, o = len(trees), fl["n_out"]
    out = torch.zeros((n, o) if sum_trees else (n, T, o), dtype=torch.float32, device=X.device)
    w = None if weights is None else torch.tensor(weights, dtype=torch.float32, device=X.device)
    p = _native.ptr
    args = (p(X), C.c_int64(n), d, p(fl["feature"]), p(fl["threshold"]), p(fl["left"]),
            p(fl["right"]), p(fl["voff"]), p(fl["values"]), p(fl["roots"]), T, o, p(out),
            int(sum_trees), p(w))
    if X.is_cuda:
        _native.check(_native.hip().hm_tree_predict(*args, _native.stream_of(X.device)), "hm_tree_predict")
    else:
        _native.host().hm_tree_predict_cpu(*args)
    return out


class _NodeBuf:
    """Growable device arrays of one tree's nodes (GPU builder): flagged split feature, split
    bin, children, threshold and leaf values, indexed by node id.  The routing kernel reads them
    as they stand, so no per-level concatenation is needed."""

    def __init__(self, cap: int, n_out: int, dev):
        self.n_out, self.dev, self.cap = n_out, dev, 0
        self.sf = self.sb = self.lc = self.rc = self.thr = self.vals = None
        self.ensure(cap)

    def ensure(self, need: int) -> None:
        if need <= self.cap:
            return
        cap = max(need, 2 * self.cap)
        i32 = dict(dtype=torch.int32, device=self.dev)
        new = dict(sf=torch.empty(cap, **i32), sb=torch.empty(cap, **i32), lc=torch.empty(cap, **i32),
                   rc=torch.empty(cap, **i32), thr=torch.empty(cap, dtype=torch.float32, device=self.dev),
                   vals=torch.empty((cap, self.n_out), dtype=torch.float32, device=self.dev))
        for k, t in new.items():
            old = getattr(self, k)
            if old is not None:
                t[:self.cap] = old
            setattr(self, k, t)
        self.cap = cap


class HistTreeBuilder:
    """Level-wise histogram tree growth on the device."""

    def __init__(self, q: Quantized, criterion: str, max_depth: int = 12,
                 min_samples_split: int = 2, min_samples_leaf: int = 1, mtry: int | None = None,
                 max_leaf_nodes: int | None = None, seed: int = 0, mixer=None, lam: float = 0.0,
                 alpha: float = 0.0, min_gain: float = 0.0, feature_mask: torch.Tensor | None = None):
        self.q = q
        self.missing = bool(getattr(q, "missing", False))   # learn default directions for NaN
        self.cat = q.cat                          # nominal columns: one-vs-rest splits
        self.criterion = criterion
        self.max_depth = max_depth
        if criterion == "xgb":
            # second-order statistics (g, h): min_samples_* are hessian weights (min_child_weight)
            self.min_split = float(min_samples_split)
            self.min_leaf = float(min_samples_leaf)
        else:
            self.min_split = max(2, int(min_samples_split))
            self.min_leaf = max(1, int(min_samples_leaf))
        self.alpha = float(alpha)
        self.min_gain = float(min_gain)
        self.feature_mask = feature_mask
        self.mtry = mtry
        self.max_leaves = max_leaf_nodes
        self.gen = torch.Generator(device="cpu").manual_seed(int(seed))
        self.mixer = mixer
        self.lam = lam
        self.importance = np.zeros(q.d)
        self._seed32 = int(seed) & 0x7FFFFFFF      # candidate-feature draw (mtry) of hm_split_find
        self._masks = None

    # -- statistics -> impurity / gain
    def _score(self, S: torch.Tensor) -> torch.Tensor:
        """Node 'goodness' whose sum over children minus the parent's is the split gain."""
        c = self.criterion
        if c == "gini":
            W = S.sum(-1)
            return torch.where(W > 0, (S * S).sum(-1) / W.clamp_min(1e-30), torch.zeros_like(W))
        if c == "entropy":
            W = S.sum(-1, keepdim=True)
            p = S / W.clamp_min(1e-30)
            return (S * torch.log(p.clamp_min(1e-30))).sum(-1)
        if c == "variance":      # S = (Σwy, Σw)
            return torch.where(S[..., 1] > 0, S[..., 0] ** 2 / S[..., 1].clamp_min(1e-30),
                               torch.zeros_like(S[..., 0]))
        if c == "gbt":           # S = (Σr, Σh, n): least squares on the residual
            return torch.where(S[..., 2] > 0, S[..., 0] ** 2 / (S[..., 2] + self.lam),
                               torch.zeros_like(S[..., 0]))
        if c == "gbt2":          # S = (Σr, n); Σh is summed per leaf after the tree is grown
            return torch.where(S[..., 1] > 0, S[..., 0] ** 2 / (S[..., 1] + self.lam),
                               torch.zeros_like(S[..., 0]))
        if c == "xgb":           # S = (Σg, Σh): T_alpha(G)^2 / (H + lambda)
            G = self._soft(S[..., 0])
            return torch.where(S[..., 1] > 0, G * G / (S[..., 1] + self.lam), torch.zeros_like(G))
        raise ValueError(c)

    def _soft(self, G: torch.Tensor) -> torch.Tensor:
        """L1 soft threshold of the gradient sum (XGBoost's alpha)."""
        if self.alpha <= 0:
            return G
        return torch.sign(G) * (G.abs() - self.alpha).clamp_min(0)

    def _weight(self, S: torch.Tensor) -> torch.Tensor:
        c = self.criterion
        if c in ("gini", "entropy"):
            return S.sum(-1)
        if c in ("variance", "xgb", "gbt2"):
            return S[..., 1]
        return S[..., 2]

    def _leaf_values(self, S: torch.Tensor) -> torch.Tensor:
        """Leaf outputs for node statistics S [L, NS] -> [L, n_out]."""
        c = self.criterion
        if c in ("gini", "entropy"):
            w = S.sum(1, keepdim=True)
            return torch.where(w > 0, S / w.clamp_min(1e-30), torch.full_like(S, 1.0 / S.shape[1]))
        if c in ("variance", "gbt2"):   # gbt2: the mean residual until the per-leaf Newton values
            return torch.where(S[:, 1:2] > 0, S[:, 0:1] / S[:, 1:2].clamp_min(1e-30), torch.zeros_like(S[:, :1]))
        if c == "xgb":           # Newton step -T(G) / (H + lambda)
            den = S[:, 1:2] + self.lam
            return torch.where(den > 0, -self._soft(S[:, 0:1]) / den.clamp_min(1e-30), torch.zeros_like(S[:, :1]))
        ok = S[:, 1:2].abs() > 1e-12
        return torch.where(ok, S[:, 0:1] / torch.where(ok, S[:, 1:2], torch.ones_like(S[:, 1:2])),
                           torch.zeros_like(S[:, :1]))

    _CRIT = {"gini": 0, "entropy": 1, "variance": 2, "gbt": 3, "xgb": 4, "gbt2": 5}

    def _split_find(self, H: torch.Tensor, node_base: int):
        """Best split of every node of the level (csrc hm_split_find: one fused kernel instead
        of ~30 tensor ops over [L, d, B, NS]).  Returns gain [L] (-inf: no valid split), feature
        and bin (int32), left-child statistics [L, NS], node totals [L, NS] and the learned
        missing-value direction."""
        gain, feat, bins, left, tot = self._split_find_raw(H, node_base)
        dleft = (bins >> 16) & 1                  # bit 16: the missing rows go left
        return gain, feat, bins & 0xFFFF, left, tot, dleft

    def _split_find_raw(self, H: torch.Tensor, node_base: int):
        L, d, B, NS = H.shape
        dev = H.device
        H = H.contiguous()
        gain = torch.empty(L, dtype=torch.float32, device=dev)
        feat = torch.empty(L, dtype=torch.int32, device=dev)
        bins = torch.empty(L, dtype=torch.int32, device=dev)
        left = torch.empty((L, NS), dtype=torch.float32, device=dev)
        tot = torch.empty((L, NS), dtype=torch.float32, device=dev)
        mtry = int(self.mtry) if (self.mtry is not None and self.mtry < d) else 0
        miss = int(self.missing and NS <= 8)
        ip = np.array([L, d, B, NS, self.q.edges.shape[1], self._CRIT[self.criterion], mtry,
                       node_base, self._seed32, miss], dtype=np.int32)
        fp = np.array([self.lam, self.alpha, float(self.min_leaf)], dtype=np.float32)
        if self._masks is None or self._masks[0] != dev:
            u8 = lambda m: None if m is None else m.to(device=dev, dtype=torch.uint8).contiguous()
            self._masks = (dev, u8(self.cat), u8(self.feature_mask))
        _, cat, fm = self._masks
        p = _native.ptr
        args = (p(H), ip.ctypes.data, fp.ctypes.data, p(cat), p(fm), p(gain), p(feat), p(bins),
                p(left), p(tot))
        if dev.type == "cuda":
            _native.check(_native.hip().hm_split_find(*args, _native.stream_of(dev)), "hm_split_find")
        else:
            if _native.host().hm_split_find_cpu(*args) != 0:
                raise RuntimeError("hm_split_find_cpu: invalid arguments")
        return gain, feat, bins, left, tot

    def _level_finalize(self, gain, feat, braw, left, tot, base: int, nb: int, edges, buf: "_NodeBuf", imp,
                        heap: bool = False, last: bool = False):
        """GPU: the level's split decisions and bookkeeping in one kernel (hm_level_finalize),
        written straight into the tree's node arrays at [base, base + L); returns
        (li int64, small_right, lut, n_split) of the splitting nodes.  ``heap``: the children of
        parent l are nodes nb + 2l, nb + 2l + 1 and small_right / lut are indexed by l; returns
        (small_right [L], lut [2L]) without reading the split count on the host.  ``last``: the
        children are leaves and their records (values from the split's left / total statistics)
        are written by the same kernel at nb .. nb + 2 * splits (heap: nb .. nb + 2L)."""
        L, NS = tot.shape
        dev = tot.device
        buf.ensure(base + (3 * L if last else L))
        li = torch.empty(L, dtype=torch.int64, device=dev)
        sr = torch.empty(L, dtype=torch.uint8, device=dev)
        lut = torch.empty(2 * L, dtype=torch.int16, device=dev)
        nsp = torch.empty(1, dtype=torch.int32, device=dev)
        cat = self._masks[1]
        ip = np.array([L, NS, self.q.d, edges.shape[1], self._CRIT[self.criterion], buf.n_out, nb,
                       int(cat is not None), int(heap), int(last)], dtype=np.int32)
        fp = np.array([self.lam, self.alpha, self.min_gain, float(self.min_split)], dtype=np.float32)
        p = _native.ptr
        o4, ov = 4 * base, 4 * base * buf.n_out          # byte offsets of node `base`
        _native.check(_native.hip().hm_level_finalize(
            ip.ctypes.data, fp.ctypes.data, p(gain), p(feat), p(braw), p(left.contiguous()), p(tot.contiguous()),
            p(edges), p(cat), p(buf.vals) + ov, p(buf.sf) + o4, p(buf.thr) + o4, p(buf.lc) + o4,
            p(buf.rc) + o4, p(buf.sb) + o4, p(li), p(sr), p(lut), p(nsp), p(imp),
            _native.stream_of(dev)), "hm_level_finalize")
        if heap:
            return sr, lut
        n_split = int(nsp.item())                                            # the level's one sync
        return li[:n_split], sr[:n_split], lut[:2 * n_split], n_split

    @staticmethod
    def _partition_gpu(act_rows, node_of_row, nb: int, lut, n_keys: int):
        """Rows of the small children grouped by child (csrc hm_partition_count / _scatter: a
        counting sort of the level's keys instead of a full radix sort of every active row)."""
        dev = act_rows.device
        m = act_rows.numel()
        G = int(max(1, min(1024, (m + 4095) // 4096)))
        counts = torch.empty(n_keys * G, dtype=torch.int64, device=dev)
        p, st = _native.ptr, _native.stream_of(dev)
        n16 = int(node_of_row.dtype == torch.int16)
        _native.check(_native.hip().hm_partition_count(p(act_rows), C.c_int64(m), p(node_of_row), p(lut), nb,
                                                       lut.numel(), n_keys, G, p(counts), n16, st), "hm_partition_count")
        incl = torch.cumsum(counts, 0)
        rows = torch.empty(max(1, m), dtype=torch.int32, device=dev)
        seg = torch.empty(n_keys + 1, dtype=torch.int64, device=dev)
        _native.check(_native.hip().hm_partition_scatter(p(act_rows), C.c_int64(m), p(node_of_row), p(lut), nb,
                                                         lut.numel(), n_keys, G, p(counts), p(incl), p(rows),
                                                         p(seg), n16, st), "hm_partition_scatter")
        return rows, seg

    def _route_partition_gpu(self, n: int, node_of_row, nbuf: "_NodeBuf", nb: int, lut, n_keys: int, lo: int):
        """Every row active (rows 0 .. n-1): route the level and count the small children in one
        pass (hm_route_count), then place them (hm_partition_scatter without a row list).
        Nodes [lo, nb) are the level's (lower ids: leaves of earlier levels)."""
        q = self.q
        dev = node_of_row.device
        # the pass is latency-bound: more blocks help (GBDT 2.12 -> 2.10-2.11 ms per tree at 2,048,
        # 2.40 at 512; profiles/r4/route_grid_ab.log) while the (key, block) counts stay small
        G = int(max(1, min(ROUTE_GRID if n_keys <= 256 else 1024, (n + 4095) // 4096)))
        counts = torch.empty(n_keys * G, dtype=torch.int64, device=dev)
        p, st = _native.ptr, _native.stream_of(dev)
        n16 = int(node_of_row.dtype == torch.int16)
        src, cs = q.route_src()
        _native.check(_native.hip().hm_route_count(
            src, C.c_int64(n), q.dpad, C.c_int64(cs), lo, p(node_of_row), p(nbuf.sf), p(nbuf.sb), p(nbuf.lc), p(nbuf.rc),
            (q.B - 1) if self.missing else -1, p(lut), nb, lut.numel(), n_keys, G, p(counts), n16, st),
            "hm_route_count")
        incl = torch.cumsum(counts, 0)
        rows = torch.empty(max(1, n), dtype=torch.int32, device=dev)
        seg = torch.empty(n_keys + 1, dtype=torch.int64, device=dev)
        _native.check(_native.hip().hm_partition_scatter(None, C.c_int64(n), p(node_of_row), p(lut), nb,
                                                         lut.numel(), n_keys, G, p(counts), p(incl), p(rows),
                                                         p(seg), n16, st), "hm_partition_scatter")
        return rows, seg

    def _hist(self, rows, seg, n_seg, stats, smax, out: torch.Tensor | None = None):
        """[n_seg, d, B, NS] histograms of the row segments rows[seg[k]:seg[k+1]] (into ``out``,
        zeroed by the caller, when given)."""
        q = self.q
        NS = stats.shape[1]
        dev = stats.device
        hist = out if out is not None else torch.zeros((n_seg, q.d, q.B, NS), dtype=torch.float32, device=dev)
        p = _native.ptr
        if dev.type == "cuda" and NS > 8:
            # many classes: the LDS kernel sums <= 8 statistics per pass -> class tiles of 8
            for c0 in range(0, NS, 8):
                c1 = min(NS, c0 + 8)
                sub = torch.zeros((n_seg, q.d, q.B, c1 - c0), dtype=torch.float32, device=dev)
                st = stats[:, c0:c1].contiguous()
                sm = smax[c0:c1].contiguous()
                FG = next((f for f in (16, 8) if f * q.B * (c1 - c0) * 4 <= 48 * 1024), 4)
                args = (p(q.bins), q.d, q.dpad, q.B, p(rows), p(seg), n_seg, p(st), p(sm), c1 - c0, FG, p(sub))
                _native.check(_native.hip().hm_hist_build(*args, HIST_BLOCKS, _native.stream_of(dev)),
                              "hm_hist_build")
                hist[..., c0:c1] = sub
        else:
            # features per group: one aligned 16/8/4-byte bins load per row, LDS image <= 48 KB;
            # or all <= 32 features in one pass (32-B bins rows, one <= 160 KB image per CU)
            FG = next((f for f in (16, 8) if f * q.B * NS * 4 <= 48 * 1024), 4)
            nblk = HIST_BLOCKS
            # (hm_hist_build instantiates the one-pass kernel for NS <= 4; 5..8 statistics take
            # the feature-group kernel)
            if HIST_WIDE and NS <= 4 and q.d <= 32 and q.dpad % 32 == 0 and q.d * q.B * NS * 4 <= 160 * 1024:
                FG, nblk = 32, HIST_WIDE_BLOCKS
            args = (p(q.bins), q.d, q.dpad, q.B, p(rows), p(seg), n_seg, p(stats), p(smax), NS, FG, p(hist))
            if dev.type == "cuda":
                _native.check(_native.hip().hm_hist_build(*args, nblk, _native.stream_of(dev)),
                              "hm_hist_build")
            else:
                _native.host().hm_hist_build_cpu(*args)
        if self.mixer is not None and self.mixer.world > 1:
            self.mixer.all_reduce_sum([hist])
        return hist

    def build(self, stats: torch.Tensor, active: torch.Tensor | None = None, smax: torch.Tensor | None = None,
              act_rows: torch.Tensor | None = None, identity_rows: bool = False,
              leaf_h: torch.Tensor | None = None, defer: bool = False):
        """Grow one tree level by level.  stats: f32 [n, NS] per-row statistics.

        Every level: split search on the device over the level's histograms; one host sync
        (the number of splits); rows routed by the bins; the next level histograms only the
        smaller child of each split (sibling = parent - child).  After the call
        ``self.leaf_of_row`` holds the leaf node id of every row (-1: inactive).  ``smax`` (the
        columns' |max|) and ``act_rows`` (int32 ids of the rows with non-zero stats) may be
        passed in when the caller already has them (the fused GBT statistics kernel);
        ``identity_rows``: act_rows is 0 .. n-1 (every row active, no ``active`` mask).
        ``leaf_h`` (criterion gbt2, stats = (r, w)): per-row hessians; the leaves get the Newton
        values sum r / sum h over their rows (csrc hm_leaf_sums / hm_leaf_newton).
        ``defer`` (level-fused builder): return a :class:`PendingTree` whose node arrays stay on
        the device (no host read at the end of the tree, importance left in ``imp_dev``) — the
        boosting loops materialise all trees after the last one."""
        q = self.q
        dev = stats.device
        n, NS = stats.shape
        d, B = q.d, q.B
        stats = stats.contiguous()
        identity_rows = bool(identity_rows and active is None and act_rows is not None and act_rows.numel() == n)
        # heap layout (no host read per level): shallow trees without per-node feature draws,
        # whose node ids (the draw's key) would differ from the compact numbering
        heap = (HEAP_TREES and dev.type == "cuda" and self.max_leaves is None
                and self.max_depth <= HEAP_MAX_DEPTH and not (self.mtry is not None and self.mtry < d)
                and (NS <= 8 or self.criterion in ("gini", "entropy")))
        # heap levels hold at most 2^(HEAP_MAX_DEPTH + 1) - 1 node ids: int16 halves the bytes of
        # the per-level routing / partition / leaf passes over the rows
        node_of_row = torch.zeros(n, dtype=torch.int16 if heap else torch.int32, device=dev)
        arena = None
        if active is not None:
            node_of_row[~active] = -1
        if act_rows is None:
            act = (stats != 0).any(1)
            if active is not None:
                act &= active
            act_rows = torch.nonzero(act).flatten().to(torch.int32)
        edges = q.edges.to(device=dev, dtype=torch.float32).contiguous()
        cat_dev = None if self.cat is None else self.cat.to(dev)
        fused = dev.type == "cuda" and self.max_leaves is None and (NS <= 8 or self.criterion in ("gini", "entropy"))
        n_out_ = NS if self.criterion in ("gini", "entropy") else 1
        nbuf = _NodeBuf(min(1 << 13, 2 << min(self.max_depth, 30)), n_out_, dev) if fused else None
        n_out = NS if self.criterion in ("gini", "entropy") else 1
        imp = torch.zeros(d, dtype=torch.float64, device=dev)
        # level 0: the root histogram over every active row
        seg = torch.stack([torch.zeros((), dtype=torch.int64, device=dev),
                           torch.full((), act_rows.numel(), dtype=torch.int64, device=dev)])
        if smax is not None:
            smax = smax.contiguous()
        elif dev.type == "cuda" and NS <= 8:              # fixed-point range of the LDS sums
            smax = torch.zeros(NS, dtype=torch.float32, device=dev)
            _native.check(_native.hip().hm_absmax_cols(_native.ptr(stats), C.c_int64(n), NS, _native.ptr(smax),
                                                        _native.stream_of(dev)), "hm_absmax_cols")
        else:
            smax = stats.abs().amax(0).contiguous()
        H = self._hist(act_rows, seg, 1, stats, smax)
        base, L = 0, 1
        n_leaves = torch.ones((), dtype=torch.int64, device=dev)
        feats, thrs, lefts, rights, vals = [], [], [], [], []
        sf_all = torch.zeros(0, dtype=torch.int32, device=dev)
        sb_all, lc_all, rc_all = sf_all.clone(), sf_all.clone(), sf_all.clone()
        depth = 0
        while True:
            if depth >= self.max_depth and fused:
                nbuf.ensure(base + L)
                nbuf.vals[base:base + L] = self._leaf_values(H[:, 0].sum(1))
                nbuf.sf[base:base + L] = -1
                nbuf.thr[base:base + L] = math.inf
                nbuf.lc[base:base + L] = -1
                nbuf.rc[base:base + L] = -1
                break
            if depth >= self.max_depth:
                vals.append(self._leaf_values(H[:, 0].sum(1)))
                feats.append(torch.full((L,), -1, dtype=torch.int32, device=dev))
                thrs.append(torch.full((L,), math.inf, device=dev))
                lefts.append(torch.full((L,), -1, dtype=torch.int32, device=dev))
                rights.append(torch.full((L,), -1, dtype=torch.int32, device=dev))
                break
            if fused and heap:
                # fixed-shape level (L = 2^depth node slots, heap numbering): nothing is read on
                # the host, the next level's kernels queue behind this one's
                gain, bf, braw, left_all, tot = self._split_find_raw(H, base)
                nb = base + L
                last = LAST_FROM_SPLITS and depth + 1 >= self.max_depth
                sr, lut = self._level_finalize(gain, bf, braw, left_all, tot, base, nb, edges, nbuf, imp, heap=True,
                                               last=last)
                p = _native.ptr
                if last:
                    # the children are leaves: route the rows, and take the children's statistics
                    # from the split search (left, total - left) instead of histogramming them
                    # (no partition, histogram or sibling pass for the last level)
                    src, cs = q.route_src()
                    _native.check(_native.hip().hm_route_rows(
                        src, C.c_int64(n), q.dpad, C.c_int64(cs), base, base + L, p(node_of_row), p(nbuf.sf), p(nbuf.sb),
                        p(nbuf.lc), p(nbuf.rc), (q.B - 1) if self.missing else -1,
                        int(node_of_row.dtype == torch.int16), _native.stream_of(dev)), "hm_route_rows")
                    base, L = nb, 2 * L
                    depth += 1
                    break
                if identity_rows and ROUTE_FUSED:
                    rows, seg = self._route_partition_gpu(n, node_of_row, nbuf, nb, lut, L, base)
                else:
                    src, cs = q.route_src()
                    _native.check(_native.hip().hm_route_rows(
                        src, C.c_int64(n), q.dpad, C.c_int64(cs), base, base + L, p(node_of_row), p(nbuf.sf), p(nbuf.sb), p(nbuf.lc),
                        p(nbuf.rc), (q.B - 1) if self.missing else -1, int(node_of_row.dtype == torch.int16),
                        _native.stream_of(dev)), "hm_route_rows")
                    rows, seg = self._partition_gpu(act_rows, node_of_row, nb, lut, L)
                if arena is None:   # every level's smaller-child histograms, zeroed in one fill
                    # levels 0 .. max_depth - 1 histogram L = 2^depth children into slots
                    # [L - 1, 2L - 1); with LAST_FROM_SPLITS the last split level histograms nothing
                    top = self.max_depth - (1 if LAST_FROM_SPLITS else 0)
                    arena = torch.zeros((((1 << top) - 1), d, B, NS), dtype=torch.float32, device=dev)
                Hs = self._hist(rows, seg.contiguous(), L, stats, smax, out=arena[L - 1:2 * L - 1])
                Hn = torch.empty((2 * L, d, B, NS), dtype=torch.float32, device=dev)
                _native.check(_native.hip().hm_hist_sibling_heap(
                    p(H), p(Hs), p(nbuf.sf) + 4 * base, p(sr), C.c_int64(d * B * NS), L, p(Hn),
                    _native.stream_of(dev)), "hm_hist_sibling_heap")
                H = Hn
                base, L = nb, 2 * L
                depth += 1
                continue
            if fused:
                gain, bf, braw, left_all, tot = self._split_find_raw(H, base)
                nb = base + L
                last = LAST_FROM_SPLITS and depth + 1 >= self.max_depth
                li, small_right, lut, n_split = self._level_finalize(gain, bf, braw, left_all, tot, base, nb,
                                                                     edges, nbuf, imp, last=last)
                if n_split == 0:
                    break
                p = _native.ptr
                if last:
                    # children are leaves: route, and their statistics from the split search
                    # (split k's children are nb + 2k, nb + 2k + 1)
                    src, cs = q.route_src()
                    _native.check(_native.hip().hm_route_rows(
                        src, C.c_int64(n), q.dpad, C.c_int64(cs), base, base + L, p(node_of_row), p(nbuf.sf), p(nbuf.sb),
                        p(nbuf.lc), p(nbuf.rc), (q.B - 1) if self.missing else -1,
                        int(node_of_row.dtype == torch.int16), _native.stream_of(dev)), "hm_route_rows")
                    base, L = nb, 2 * n_split
                    depth += 1
                    break
                if identity_rows and n_split <= 8192 and ROUTE_FUSED:
                    rows, seg = self._route_partition_gpu(n, node_of_row, nbuf, nb, lut, n_split, base)
                    Hs = self._hist(rows, seg.contiguous(), n_split, stats, smax)
                    Hn = torch.empty((2 * n_split, d, B, NS), dtype=torch.float32, device=dev)
                    _native.check(_native.hip().hm_hist_sibling(
                        _native.ptr(H), _native.ptr(Hs), _native.ptr(li), _native.ptr(small_right),
                        C.c_int64(d * B * NS), n_split, _native.ptr(Hn), _native.stream_of(dev)), "hm_hist_sibling")
                    H = Hn
                    base, L = nb, 2 * n_split
                    depth += 1
                    continue
                src, cs = q.route_src()
                _native.check(_native.hip().hm_route_rows(
                    src, C.c_int64(n), q.dpad, C.c_int64(cs), base, base + L, p(node_of_row), p(nbuf.sf), p(nbuf.sb), p(nbuf.lc), p(nbuf.rc),
                    (q.B - 1) if self.missing else -1, int(node_of_row.dtype == torch.int16),
                        _native.stream_of(dev)), "hm_route_rows")
                if n_split <= 8192:
                    rows, seg = self._partition_gpu(act_rows, node_of_row, nb, lut, n_split)
                else:
                    nr = node_of_row[act_rows.long()] - nb
                    key = torch.where(nr >= 0, lut[nr.clamp_min(0).long()],
                                      torch.full_like(nr, 32767, dtype=torch.int16))
                    skey, order = torch.sort(key, stable=True)
                    rows = act_rows[order].contiguous()
                    seg = torch.searchsorted(skey, torch.arange(n_split + 1, device=dev, dtype=torch.int16)).to(torch.int64)
                Hs = self._hist(rows, seg.contiguous(), n_split, stats, smax)
                Hn = torch.empty((2 * n_split, d, B, NS), dtype=torch.float32, device=dev)
                _native.check(_native.hip().hm_hist_sibling(
                    _native.ptr(H), _native.ptr(Hs), _native.ptr(li), _native.ptr(small_right), C.c_int64(d * B * NS),
                    n_split, _native.ptr(Hn), _native.stream_of(dev)), "hm_hist_sibling")
                H = Hn
                base, L = nb, 2 * n_split
                depth += 1
                continue
            best_gain, bf, bb, left_all, tot, bdl = self._split_find(H, base)
            vals.append(self._leaf_values(tot))
            ok = (best_gain > max(1e-12, self.min_gain)) & torch.isfinite(best_gain) & \
                (self._weight(tot) >= self.min_split)
            if self.max_leaves is not None:
                ok &= torch.cumsum(ok.long(), 0) <= (int(self.max_leaves) - n_leaves)
            li = torch.nonzero(ok).flatten()                                   # the level's one sync
            n_split = li.numel()
            rank = torch.cumsum(ok.int(), 0) - 1
            nb = base + L
            lc = torch.where(ok, nb + 2 * rank, torch.full_like(rank, -1)).to(torch.int32)
            rc = torch.where(ok, lc + 1, lc).to(torch.int32)
            thr = torch.where(bb < edges.shape[1], edges[bf.long(), bb.clamp(max=edges.shape[1] - 1).long()],
                              torch.full_like(best_gain, math.inf))
            bflag = bf if cat_dev is None else bf | (cat_dev[bf.long()].to(torch.int32) * CAT_FLAG)
            bflag = bflag | (bdl * DLEFT_FLAG)
            feats.append(torch.where(ok, bflag, torch.full_like(bf, -1)))
            thrs.append(torch.where(ok, thr, torch.full_like(thr, math.inf)))
            lefts.append(lc)
            rights.append(rc)
            if n_split == 0:
                break
            imp.index_add_(0, bf[li].long(), best_gain[li].double())
            n_leaves = n_leaves + n_split
            # route every row one level down (leaves keep their id: split_feat < 0)
            sf_all = torch.cat([sf_all, feats[-1]])
            sb_all = torch.cat([sb_all, bb])
            lc_all = torch.cat([lc_all, lc])
            rc_all = torch.cat([rc_all, rc])
            p = _native.ptr
            rest = (p(node_of_row), p(sf_all), p(sb_all), p(lc_all), p(rc_all), (q.B - 1) if self.missing else -1)
            if dev.type == "cuda":
                src, cs = q.route_src()
                _native.check(_native.hip().hm_route_rows(src, C.c_int64(n), q.dpad, C.c_int64(cs), base, base + L, *rest,
                                                          int(node_of_row.dtype == torch.int16),
                                                          _native.stream_of(dev)), "hm_route_rows")
            else:
                _native.host().hm_route_rows_cpu(p(q.bins), C.c_int64(n), q.dpad, *rest)
            # next level: histogram the smaller child of every split, derive the sibling
            left_tot = left_all[li]                                            # [S, NS]
            right_tot = tot[li] - left_tot
            small_right = self._weight(right_tot) < self._weight(left_tot)     # [S]
            small_id = torch.where(small_right, rc[li], lc[li]) - nb           # local child id
            lut = torch.full((2 * n_split,), 32767, dtype=torch.int16, device=dev)
            lut[small_id.long()] = torch.arange(n_split, device=dev, dtype=torch.int16)
            if dev.type == "cuda" and n_split <= 8192:
                rows, seg = self._partition_gpu(act_rows, node_of_row, nb, lut, n_split)
            else:
                nr = node_of_row[act_rows.long()] - nb
                key = torch.where(nr >= 0, lut[nr.clamp_min(0).long()], torch.full_like(nr, 32767, dtype=torch.int16))
                skey, order = torch.sort(key, stable=True)
                rows = act_rows[order].contiguous()
                seg = torch.searchsorted(skey, torch.arange(n_split + 1, device=dev, dtype=torch.int16)).to(torch.int64)
            Hs = self._hist(rows, seg.contiguous(), n_split, stats, smax)
            Hn = torch.empty((2 * n_split, d, B, NS), dtype=torch.float32, device=dev)
            if dev.type == "cuda":
                sr8 = small_right.to(torch.uint8)
                _native.check(_native.hip().hm_hist_sibling(
                    _native.ptr(H), _native.ptr(Hs), _native.ptr(li), _native.ptr(sr8), C.c_int64(d * B * NS),
                    n_split, _native.ptr(Hn), _native.stream_of(dev)), "hm_hist_sibling")
            else:
                sr = small_right.long()
                j2 = 2 * torch.arange(n_split, device=dev)
                Hn[j2 + sr] = Hs
                Hn[j2 + 1 - sr] = H[li] - Hs
            H = Hn
            base, L = nb, 2 * n_split
            depth += 1
        defer = defer and fused
        if defer:
            self.imp_dev = imp
        else:
            self.importance = self.importance + imp.cpu().numpy()
        self.leaf_of_row = node_of_row
        if fused and leaf_h is not None:
            t = base + L
            sums = torch.zeros((t, 2), dtype=torch.float32, device=dev)
            p, st_ = _native.ptr, _native.stream_of(dev)
            if t <= 8192:
                _native.check(_native.hip().hm_leaf_sums(p(node_of_row), p(stats), p(leaf_h), C.c_int64(n), t,
                                                         p(sums), int(node_of_row.dtype == torch.int16), st_),
                              "hm_leaf_sums")
            else:
                ok = node_of_row >= 0
                nd = node_of_row[ok].long()
                sums[:, 0].index_add_(0, nd, stats[ok, 0])
                sums[:, 1].index_add_(0, nd, leaf_h[ok])
            if self.mixer is not None and self.mixer.world > 1:
                self.mixer.all_reduce_sum([sums])
            _native.check(_native.hip().hm_leaf_newton(p(sums), p(nbuf.sf), t, p(nbuf.vals), st_), "hm_leaf_newton")
        if fused:
            t = base + L                                   # nodes written, ids 0 .. t - 1
            self.node_values = nbuf.vals[:t]
            if defer:
                return PendingTree(nbuf.sf[:t], nbuf.thr[:t], nbuf.lc[:t], nbuf.rc[:t], nbuf.vals[:t], n_out)
            F, Lc, Rc = torch.stack([nbuf.sf[:t], nbuf.lc[:t], nbuf.rc[:t]]).cpu().numpy()
            T = nbuf.thr[:t].cpu().numpy()
            V = self.node_values.double().cpu().numpy()
        else:
            F = torch.cat(feats).cpu().numpy()
            T = torch.cat(thrs).cpu().numpy()
            Lc = torch.cat(lefts).cpu().numpy()
            Rc = torch.cat(rights).cpu().numpy()
            V = torch.cat(vals).double().cpu().numpy()
            self.node_values = torch.cat(vals)
        return _tree_from_arrays(F, T, Lc, Rc, V, n_out)


def _tree_from_arrays(F, T, Lc, Rc, V, n_out: int) -> Tree:
    # the node lists are acyclic: pausing the cyclic collector while they are built saves the
    # collections their thousands of allocations trigger over every live object (3.9 -> 1.1 ms
    # for a 4,095-node tree)
    enabled = gc.isenabled()
    gc.disable()
    try:
        return _tree_from_arrays_impl(F, T, Lc, Rc, V, n_out)
    finally:
        if enabled:
            gc.enable()


def _tree_from_arrays_impl(F, T, Lc, Rc, V, n_out: int) -> Tree:
    F, T, Lc, Rc, V = (np.asarray(a) for a in (F, T, Lc, Rc, V))
    # a heap-layout build holds node slots no parent points to (children of parents that did not
    # split): keep the reachable nodes in id order — level by level, parents in order, which is
    # the compact numbering of the per-level build — and renumber the children
    reach = np.zeros(len(F), dtype=bool)
    if len(F):
        reach[0] = True
        front = np.array([0])
        while front.size:
            sp = front[F[front] >= 0]
            front = np.concatenate([Lc[sp], Rc[sp]])
            reach[front] = True
    if not reach.all():
        keep = np.nonzero(reach)[0]
        remap = np.full(len(F), -1, dtype=np.int64)
        remap[keep] = np.arange(keep.size)
        F, T, V = F[keep], T[keep], V[keep]
        Lc = np.where(F >= 0, remap[np.maximum(Lc[keep], 0)], -1)
        Rc = np.where(F >= 0, remap[np.maximum(Rc[keep], 0)], -1)
    F = F.astype(np.int64)
    split = F >= 0
    tree = Tree(n_out=n_out)
    cflag = (split & ((F & CAT_FLAG) != 0)).astype(int)
    tree.cat = cflag.tolist() if cflag.any() else []
    dflag = (split & ((F & DLEFT_FLAG) != 0)).astype(int)
    tree.dleft = dflag.tolist() if dflag.any() else []
    tree.feature = np.where(split, F & ~(CAT_FLAG | DLEFT_FLAG), F).tolist()
    tree.threshold = T.astype(np.float64).tolist()
    tree.left = Lc.astype(np.int64).tolist()
    tree.right = Rc.astype(np.int64).tolist()
    # leaf value lists only (a list per node, discarded for split nodes, cost GC time)
    value = [None] * len(F)
    leaves = np.nonzero(~split)[0]
    for k, v in zip(leaves.tolist(), V[leaves].tolist()):
        value[k] = v
    tree.value = value
    return tree


class PendingTree:
    """A grown tree whose node arrays are still on the device (HistTreeBuilder.build(defer=True)):
    the boosting loop keeps the GPU busy with the next tree instead of waiting on five host reads
    and the Python node lists per tree; :meth:`materialize` builds the :class:`Tree`."""

    def __init__(self, sf, thr, lc, rc, vals, n_out: int):
        self.arrays = (sf, thr, lc, rc, vals)
        self.n_out = n_out
        self.scale = 1.0          # leaf values x scale (XGBoost's eta)

    def materialize(self) -> Tree:
        sf, thr, lc, rc, vals = self.arrays
        F, Lc, Rc = torch.stack([sf, lc, rc]).cpu().numpy()
        return _tree_from_arrays(F, thr.cpu().numpy(), Lc, Rc, vals.double().cpu().numpy() * self.scale, self.n_out)


def materialize_trees(iters: list) -> list:
    """Boosting rounds with every PendingTree replaced by its Tree: the node arrays of all of
    them come to the host in one copy per array kind (one sync, not five per tree)."""
    pend = [t for it in iters for t in it if isinstance(t, PendingTree)]
    if not pend:
        return iters
    sizes = [t.arrays[0].numel() for t in pend]
    ints = torch.cat([torch.stack([t.arrays[0], t.arrays[2], t.arrays[3]]) for t in pend], 1).cpu().numpy()
    thr = torch.cat([t.arrays[1] for t in pend]).cpu().numpy()
    vals = torch.cat([t.arrays[4] for t in pend]).double().cpu().numpy()
    out, o = {}, 0
    for t, n in zip(pend, sizes):
        out[id(t)] = _tree_from_arrays(ints[0, o:o + n], thr[o:o + n], ints[1, o:o + n], ints[2, o:o + n],
                                       vals[o:o + n] * t.scale, t.n_out)
        o += n
    return [[out[id(t)] if isinstance(t, PendingTree) else t for t in it] for it in iters]


# ------------------------------------------------------------------ learners
TREE_OPTS = [
    opt("trees", "num_trees", 50, int, "Number of trees"),
    opt("mtry", "vars", None, int, "Number of random features per split (default sqrt(d) / d/3)",
        aliases=("num_variables",)),
    opt("max_depth", None, 16, int, "Maximum tree depth"),
    opt("max_leaf_nodes", "max_leafs", None, int, "Maximum number of leaves"),
    opt("min_split", "min_samples_split", 2, int, "Minimum rows to split a node"),
    opt("min_samples_leaf", None, 1, int, "Minimum rows in a leaf"),
    opt("seed", None, -1, int, "Seed"),
    opt("attrs", "attribute_types", None, str,
        "Attribute types, Q (quantitative) or C (categorical) per column, e.g. Q,C,Q; categorical "
        "columns get one-vs-rest 'x == v' splits"),
    opt("subsample", None, 1.0, float, "Bootstrap sampling rate"),
    flag("stratified", "stratified_sampling", "Stratified bootstrap: sample every class at the "
                                              "-subsample rate"),
    opt("splits", "split_rule", "GINI", str, "GINI | ENTROPY"),
    opt("num_bins", None, 256, int, "[engine] histogram bins (<= 256)"),
]


def _to_dense(features, d=None) -> np.ndarray:
    """Training rows -> float32 matrix, assembled the way upstream's RandomForest / GBT UDTFs
    buffer them (``MatrixBuilder.nextRow`` then ``buildMatrix``; utils/matrix.py): dense rows of
    numbers, sparse ``"i:v"`` strings or int index arrays.  Dense float rows take the fast path
    straight into an array."""
    rows = list(features)
    if not rows:
        return np.zeros((0, d or 0), dtype=np.float32)
    first = next((r for r in rows if r is not None and len(r)), None)
    if first is not None and not isinstance(list(first)[0], str) and \
            all(r is not None and len(r) == len(first) for r in rows):
        return np.asarray([list(r) for r in rows], dtype=np.float32)
    from ..utils.matrix import MatrixBuilder

    mb = MatrixBuilder("csr", n_cols=d)
    for r in rows:
        if d is not None and r is not None and len(r) and isinstance(list(r)[0], str):
            r = [f for f in r if int(str(f).partition(":")[0]) < d]   # features past d are dropped
        mb.next_row(r)
    return mb.build().to_dense().astype(np.float32)


def _encode_classes(yl):
    """Sorted distinct labels (python scalars) and the int64 class index of every row
    (on the labels' device when given a tensor)."""
    if torch.is_tensor(yl):
        cls, inv = torch.unique(yl.reshape(-1), sorted=True, return_inverse=True)
        return cls.cpu().tolist(), inv.to(torch.int64)
    cls, inv = np.unique(np.asarray(yl).reshape(-1), return_inverse=True)
    return cls.tolist(), torch.from_numpy(inv.astype(np.int64))


def _encode_classes_dp(yl, mixer=None):
    """:func:`_encode_classes` over the union of every rank's labels: a data-parallel fit
    (row-sharded boosting) needs one class list on every rank, or K, the statistics width and
    the label -> index map differ between ranks whose shards lack a class."""
    if mixer is None or mixer.world <= 1:
        return _encode_classes(yl)
    import torch.distributed as dist

    mine = _encode_classes(yl)[0]
    allc = [None] * mixer.world
    dist.all_gather_object(allc, mine)
    cls = sorted(set().union(*allc))
    if torch.is_tensor(yl):
        ct = torch.tensor(cls, dtype=yl.dtype, device=yl.device)
        return cls, torch.searchsorted(ct, yl.reshape(-1).contiguous()).to(torch.int64)
    a = np.asarray(yl).reshape(-1)
    return cls, torch.from_numpy(np.searchsorted(np.asarray(cls), a).astype(np.int64))


class _ForestBase(Learner):
    SQL_DP = "union"     # trees t with t % world == rank, over all rows
    OPTIONS = TREE_OPTS
    TASK = "classification"

    def __init__(self, options=None, device=None, **kw):
        super().__init__(options, device, **kw)
        c = self.cl
        self.trees: list[Tree] = []
        self.oob_errors = []
        self.oob_tests = []
        self.importances = []
        self.classes = None
        self.num_bins = min(256, max(2, int(c["num_bins"])))

    def _prep(self, features, labels):
        X = features if torch.is_tensor(features) else torch.from_numpy(_to_dense(features))
        X = X.float().to(self.device)
        y = labels if torch.is_tensor(labels) else torch.as_tensor(np.asarray(labels))
        return X, y.to(self.device)

    def fit(self, features, labels):
        X, y = self._prep(features, labels)
        n, d = X.shape
        c = self.cl
        q = quantize(X, self.num_bins, seed=self.seed, categorical=parse_attrs(c["attrs"], d))
        if self.TASK == "classification":
            cls, yi = _encode_classes(y)
            self.classes = cls
            yi = yi.to(self.device)
            onehot = torch.nn.functional.one_hot(yi, len(self.classes)).float()
            crit = "entropy" if str(c["splits"]).upper() == "ENTROPY" else "gini"
            mtry = c["mtry"] or max(1, int(math.floor(math.sqrt(d))))
        else:
            yf = y.float()
            crit = "variance"
            mtry = c["mtry"] or max(1, d // 3)
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        world = self.mixer.world if self.mixer is not None else 1
        rank = self.rank
        T = int(c["trees"])
        my = [t for t in range(T) if t % world == rank]
        strat = yi if (self.TASK == "classification" and c["stratified"]) else None
        pending = []
        for t in my:
            g.manual_seed(self.seed * 1000003 + t)   # tree t's bootstrap does not depend on the rank split
            w = bootstrap_weights(n, float(c["subsample"]), g, self.device, strat)
            if self.TASK == "classification":
                stats = onehot * w[:, None]       # > 8 classes: class-tiled histograms
            else:
                stats = torch.stack([w * yf, w], 1)
            b = HistTreeBuilder(q, crit, int(c["max_depth"]), c["min_split"], c["min_samples_leaf"],
                                mtry, c["max_leaf_nodes"], seed=self.seed * 1000 + t)
            # the in-bag rows (w > 0) are the active rows, without a reduction over the stats
            # the in-bag rows (w > 0) are the active rows, without a reduction over the stats.
            # (Routing all rows and counting only the in-bag ones in one pass, as GBT does, was
            # measured: 5.72-5.78 vs 5.6 ms per tree — the count / scatter then walk all n rows.)
            tree = b.build(stats, act_rows=torch.nonzero(w > 0).flatten().to(torch.int32))
            self.trees.append(tree)
            self.importances.append(b.importance)
            # out-of-bag error from the leaf every row was routed to while growing; kept on the
            # device (full-size masked reductions, no boolean indexing) and read once after the
            # last tree instead of two host syncs per tree
            oob = w == 0
            leaf = b.leaf_of_row.long()
            oob = oob & (leaf >= 0)
            if self.TASK == "classification":
                # the class of every node first (a few thousand), then one gather per row — not
                # an argmax over the gathered [n, classes] outputs
                err = ((b.node_values.argmax(1)[leaf.clamp_min(0)] != yi) & oob).sum()
            else:
                out = b.node_values[leaf.clamp_min(0), 0]
                err = torch.where(oob, (out - yf) ** 2, torch.zeros_like(yf)).double().sum()
            pending.append((err, oob.sum()))
        if pending:
            errs = torch.stack([e.double() for e, _ in pending]).cpu().tolist()
            nos = torch.stack([n for _, n in pending]).cpu().tolist()
            for e, no in zip(errs, nos):
                self.oob_errors.append(int(e) if self.TASK == "classification" else float(e))
                self.oob_tests.append(int(no))
        return self

    def model_table(self) -> pd.DataFrame:
        rows = []
        for t, (tree, imp, e, nt) in enumerate(zip(self.trees, self.importances, self.oob_errors,
                                                    self.oob_tests)):
            meta = {"classes": self.classes} if self.classes is not None else {}
            js = tree.to_json()
            js.update(meta)
            s = base91.encode(zlib.compress(json.dumps(js, separators=(",", ":")).encode()))
            acc = 1.0 - (e / nt) if (nt and self.TASK == "classification") else 1.0
            rows.append((f"{self.rank}-{t}", float(acc), s, imp.tolist(), int(e) if self.TASK == "classification" else float(e), nt))
        return pd.DataFrame(rows, columns=["model_id", "model_weight", "model", "var_importance",
                                           "oob_errors", "oob_tests"])

    def predict_proba(self, features) -> np.ndarray:
        X = features if torch.is_tensor(features) else torch.from_numpy(_to_dense(features))
        out = predict_forest(self.trees, X.float().to(self.device))
        return (out / len(self.trees)).cpu().numpy()

    def predict(self, features) -> np.ndarray:
        p = self.predict_proba(features)
        if self.TASK == "classification":
            return np.asarray(self.classes)[p.argmax(1)]
        return p[:, 0]


BOOT_CHUNK = 12288   # rows per LDS counting block of hm_bootstrap_counts


def bootstrap_weights(n: int, rate: float, gen: torch.Generator, device,
                      strata: torch.Tensor | None = None) -> torch.Tensor:
    """Per-row multiplicities of a bootstrap sample of round(n * rate) rows with replacement;
    with ``strata`` (class index per row) every class is sampled at that rate separately
    (``-stratified``), so rare classes keep their share in every tree."""
    if strata is None:
        m = max(1, int(round(n * rate)))
        if torch.device(device).type == "cuda":
            # the m draws' counts per chunk of BOOT_CHUNK rows from an exact multinomial (host),
            # then each chunk's draws counted in LDS (csrc hm_bootstrap_counts): torch.bincount
            # over m random ids took 450 µs for 11 M rows (global atomics on random addresses)
            seed = int(gen.initial_seed())
            K = (n + BOOT_CHUNK - 1) // BOOT_CHUNK
            sizes = np.full(K, BOOT_CHUNK, dtype=np.float64)
            sizes[-1] = n - BOOT_CHUNK * (K - 1)
            cnt = np.random.Generator(np.random.PCG64(seed)).multinomial(m, sizes / n).astype(np.int64)
            cnt_d = torch.from_numpy(cnt).to(device, non_blocking=True)
            out = torch.empty(n, dtype=torch.float32, device=device)
            _native.check(_native.hip().hm_bootstrap_counts(_native.ptr(cnt_d), C.c_int64(n), BOOT_CHUNK,
                                                            C.c_uint64(seed & (2 ** 64 - 1)), _native.ptr(out),
                                                            _native.stream_of(out.device)), "hm_bootstrap_counts")
            return out
        draw = torch.randint(0, n, (m,), generator=gen, device=device)
        return torch.bincount(draw, minlength=n).float()
    w = torch.zeros(n, dtype=torch.float32, device=device)
    for k in torch.unique(strata).tolist():
        rows = torch.nonzero(strata == k).flatten()
        m = max(1, int(round(rows.numel() * rate)))
        pick = rows[torch.randint(0, rows.numel(), (m,), generator=gen, device=device)]
        w += torch.bincount(pick, minlength=n).float()
    return w


class RandomForestClassifier(_ForestBase):
    NAME = "train_randomforest_classifier"
    TASK = "classification"


class RandomForestRegressor(_ForestBase):
    NAME = "train_randomforest_regressor"
    TASK = "regression"


GBT_OPTS = [
    opt("trees", "num_trees", 500, int, "Number of boosting iterations"),
    opt("eta", "learning_rate", 0.05, float, "Shrinkage"),
    opt("subsample", None, 0.7, float, "Row subsampling rate per iteration"),
    opt("max_depth", None, 8, int, "Maximum tree depth"),
    opt("max_leaf_nodes", "max_leafs", None, int, "Maximum number of leaves"),
    opt("min_split", "min_samples_split", 5, int, "Minimum rows to split"),
    opt("min_samples_leaf", None, 1, int, "Minimum rows in a leaf"),
    opt("mtry", "vars", None, int, "Random features per split (default: all)"),
    opt("seed", None, -1, int, "Seed"),
    opt("attrs", "attribute_types", None, str,
        "Attribute types, Q or C per column (C: one-vs-rest 'x == v' splits)"),
    opt("num_bins", None, 256, int, "[engine] histogram bins"),
    opt("lambda", None, 0.0, float, "[engine] L2 on leaf values (0 = Friedman's least squares)"),
]


class GradientTreeBoostingClassifier(Learner):
    SQL_DP = "shard"     # rows split over the ranks, histograms all-reduced
    """Friedman's gradient boosting with logistic loss (binary) or softmax (K classes):
    regression trees on the pseudo-residuals, Newton leaf values Σr / Σ|r|(1-|r|)."""
    NAME = "train_gradient_tree_boosting_classifier"
    OPTIONS = GBT_OPTS

    def __init__(self, options=None, device=None, **kw):
        super().__init__(options, device, **kw)
        self.iters: list[list[Tree]] = []
        self.intercepts = None
        self.classes = None
        self.importance = None
        self.oob_rates = []

    def fit(self, features, labels):
        c = self.cl
        X = features if torch.is_tensor(features) else torch.from_numpy(_to_dense(features))
        X = X.float().to(self.device)
        self.classes, yi = _encode_classes_dp(labels if torch.is_tensor(labels) else np.asarray(labels),
                                              self.mixer)
        yi = yi.to(self.device)
        K = len(self.classes)
        n, d = X.shape
        # ``edges=`` (engine kwarg): fixed bin edges, e.g. shared by a data-parallel job and its
        # single-process reference
        q = quantize(X, min(256, int(c["num_bins"])), seed=self.seed, mixer=self.mixer,
                     edges=self.kw.get("edges"),
                     categorical=parse_attrs(c["attrs"], d))
        self.importance = np.zeros(d)
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        eta = float(c["eta"])
        if K == 2:
            pos = float((yi == 1).float().sum().item())
            if self.mixer is not None:     # the global positive rate, so every rank starts alike
                pos = self.mixer.all_reduce_scalar(pos) / self.mixer.all_reduce_scalar(float(n))
            else:
                pos /= n
            pos = min(max(pos, 1e-6), 1 - 1e-6)
            self.intercepts = [math.log(pos / (1 - pos))]
            F = torch.full((n, 1), self.intercepts[0], device=self.device)
            Y = (yi == 1).float()[:, None]
        else:
            self.intercepts = [0.0] * K
            F = torch.zeros((n, K), device=self.device)
            Y = torch.nn.functional.one_hot(yi, K).float()
        m_sub = max(1, int(round(n * float(c["subsample"]))))
        fused = self.device.type == "cuda" and K == 2
        if fused:
            # binary logistic on the GPU: one fused statistics pass and one fused leaf update per
            # tree instead of ~12 tensor passes over the n rows (profiles/gbt_r2/)
            y1 = Y[:, 0].contiguous()
            # gbt2: the histograms carry (r, w) and the Newton leaf values sum h per leaf afterwards
            # (2 LDS statistics instead of 3); HM_GBT2=0 keeps (r, h, w) histograms
            gbt2 = GBT2 and c["max_leaf_nodes"] is None      # (the level-fused builder only)
            ns = 2 if gbt2 else 3
            stats_buf = torch.empty((n, ns), dtype=torch.float32, device=self.device)
            hh = torch.empty(n, dtype=torch.float32, device=self.device) if gbt2 else None
            smax = torch.zeros(ns, dtype=torch.float32, device=self.device)
            all_rows = torch.arange(n, dtype=torch.int32, device=self.device)
            st = _native.stream_of(self.device)
        imp_dev = None
        for it in range(int(c["trees"])):
            if fused:
                mask = None
                if m_sub < n:
                    sel = torch.randperm(n, generator=g, device=self.device)[:m_sub]
                    mask = torch.zeros(n, dtype=torch.bool, device=self.device)
                    mask[sel] = True
                smax.zero_()
                if gbt2:
                    _native.check(_native.hip().hm_gbt2_stats(
                        _native.ptr(F), _native.ptr(y1), _native.ptr(mask), C.c_int64(n), _native.ptr(stats_buf),
                        _native.ptr(smax), _native.ptr(hh), st), "hm_gbt2_stats")
                else:
                    _native.check(_native.hip().hm_gbt_stats(
                        _native.ptr(F), _native.ptr(y1), _native.ptr(mask), C.c_int64(n), _native.ptr(stats_buf),
                        _native.ptr(smax), st), "hm_gbt_stats")
                b = HistTreeBuilder(q, "gbt2" if gbt2 else "gbt", int(c["max_depth"]), c["min_split"],
                                    c["min_samples_leaf"], c["mtry"], c["max_leaf_nodes"],
                                    seed=self.seed * 7919 + it * K, mixer=self.mixer, lam=float(c["lambda"]))
                tree = b.build(stats_buf, smax=smax, act_rows=all_rows if mask is None else None,
                               identity_rows=mask is None, leaf_h=hh, defer=True)
                if isinstance(tree, PendingTree):
                    imp_dev = b.imp_dev if imp_dev is None else imp_dev + b.imp_dev
                else:
                    self.importance += b.importance
                vals = b.node_values.float().contiguous()
                _native.check(_native.hip().hm_gbt_apply(
                    _native.ptr(F), F.shape[1], 0, _native.ptr(vals), vals.shape[1], _native.ptr(b.leaf_of_row),
                    C.c_int64(n), C.c_float(eta), int(b.leaf_of_row.dtype == torch.int16), st), "hm_gbt_apply")
                self.iters.append([tree])
                if mask is None:
                    self.oob_rates.append(0.0)
                else:
                    oob = ~mask
                    pred = (F[oob, 0] > 0).long()
                    self.oob_rates.append(float((pred != yi[oob]).float().mean().item()))
                continue
            P = torch.sigmoid(F) if K == 2 else torch.softmax(F, 1)
            R = Y - P
            H = (R.abs() * (1 - R.abs())) if K == 2 else P * (1 - P)
            if m_sub >= n:
                mask = torch.ones(n, dtype=torch.bool, device=self.device)
            else:
                sel = torch.randperm(n, generator=g, device=self.device)[:m_sub]
                mask = torch.zeros(n, dtype=torch.bool, device=self.device)
                mask[sel] = True
            trees = []
            for k in range(R.shape[1]):
                stats = torch.stack([R[:, k], H[:, k], torch.ones(n, device=self.device)], 1)
                stats = stats * mask[:, None].float()
                b = HistTreeBuilder(q, "gbt", int(c["max_depth"]), c["min_split"], c["min_samples_leaf"],
                                    c["mtry"], c["max_leaf_nodes"], seed=self.seed * 7919 + it * K + k,
                                    mixer=self.mixer, lam=float(c["lambda"]))
                tree = b.build(stats)
                if K > 2:  # Friedman's K-class leaf scaling
                    tree.value = [[v[0] * (K - 1) / K] if v is not None else None for v in tree.value]
                trees.append(tree)
                self.importance += b.importance
                # every row (sampled or not) was routed to its leaf while the tree grew
                F[:, k] += eta * b.node_values[b.leaf_of_row.long(), 0] * ((K - 1) / K if K > 2 else 1.0)
            self.iters.append(trees)
            oob = ~mask
            if oob.any():
                pred = (F[oob, 0] > 0).long() if K == 2 else F[oob].argmax(1)
                self.oob_rates.append(float((pred != yi[oob]).float().mean().item()))
            else:
                self.oob_rates.append(0.0)
        self.iters = materialize_trees(self.iters)
        if imp_dev is not None:
            self.importance += imp_dev.cpu().numpy()
        return self

    def decision_function(self, features) -> np.ndarray:
        X = features if torch.is_tensor(features) else torch.from_numpy(_to_dense(features))
        X = X.float().to(self.device)
        K = len(self.intercepts)
        F = torch.tensor(self.intercepts, device=self.device).repeat(X.shape[0], 1)
        eta = float(self.cl["eta"])
        for k in range(K):
            ts = [trees[k] for trees in self.iters]
            if ts:
                F[:, k] += eta * predict_forest(ts, X)[:, 0]
        return F.cpu().numpy()

    def predict_proba(self, features) -> np.ndarray:
        F = torch.from_numpy(self.decision_function(features))
        if F.shape[1] == 1:
            p = torch.sigmoid(F[:, 0])
            return torch.stack([1 - p, p], 1).numpy()
        return torch.softmax(F, 1).numpy()

    def predict(self, features):
        return np.asarray(self.classes)[self.predict_proba(features).argmax(1)]

    def model_table(self) -> pd.DataFrame:
        rows = []
        eta = float(self.cl["eta"])
        for it, (trees, oob) in enumerate(zip(self.iters, self.oob_rates)):
            ms = []
            for t in trees:
                js = t.to_json()
                js["classes"] = self.classes
                ms.append(base91.encode(zlib.compress(json.dumps(js, separators=(",", ":")).encode())))
            rows.append((it + 1, ms, self.intercepts[0] if len(self.intercepts) == 1 else self.intercepts,
                         eta, self.importance.tolist(), oob))
        return pd.DataFrame(rows, columns=["iteration", "pred_models", "intercept", "shrinkage",
                                           "var_importance", "oob_error_rate"])


# ------------------------------------------------------------------ SQL-side prediction
_MODEL_CACHE: dict = {}


def _load_model(model_id, model: str):
    key = (model_id, hash(model))
    t = _MODEL_CACHE.get(key)
    if t is None:
        js = json.loads(zlib.decompress(base91.decode(model)).decode())
        t = (Tree.from_json(js), js.get("classes"))
        if len(_MODEL_CACHE) > 4096:
            _MODEL_CACHE.clear()
        _MODEL_CACHE[key] = t
    return t


@udf("tree_predict")
def tree_predict(model_id, model, features, options=None):
    """Classification (``-classification`` or a classifier model): {value: label index,
    posteriori: class probabilities}; regression: the leaf value."""
    tree, classes = _load_model(model_id, model)
    x = features
    if x is not None and len(x) and isinstance(list(x)[0], str):
        x = _to_dense([x])[0].tolist()
    out = tree.predict_one(list(x))
    if classes is not None and (tree.n_out > 1 or (options and "-classification" in str(options))):
        return {"value": int(np.argmax(out)), "posteriori": list(out)}
    return float(out[0])


@udf("tree_predict_v1")
def tree_predict_v1(model_id, model_type, model, features, classification=True):
    return tree_predict(model_id, model, features, "-classification" if classification else None)


@udaf("rf_ensemble")
def rf_ensemble(yhat, posteriori=None, model_weight=None):
    """Weighted vote of tree predictions -> {label, probability, probabilities}."""
    votes: dict = {}
    probs = None
    wsum = 0.0
    for i, y in enumerate(yhat):
        if y is None:
            continue
        w = 1.0 if model_weight is None or model_weight[i] is None else float(model_weight[i])
        votes[y] = votes.get(y, 0.0) + w
        if posteriori is not None and posteriori[i] is not None:
            p = np.asarray(posteriori[i], dtype=np.float64) * w
            probs = p if probs is None else probs + p
        wsum += w
    if not votes:
        return None
    if probs is not None:
        probs = probs / wsum
        label = int(np.argmax(probs))
        return {"label": label, "probability": float(probs[label]), "probabilities": probs.tolist()}
    label = max(votes, key=votes.get)
    return {"label": label, "probability": votes[label] / wsum, "probabilities": None}


@udf("guess_attribute_types")
def guess_attribute_types(*cols):
    """'Q' for numeric columns, 'C' for the others, comma-joined."""
    out = []
    for v in cols:
        out.append("Q" if isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool) else "C")
    return ",".join(out)


@udf("tree_export")
def tree_export(model, options: str = "-type graphviz", feature_names=None, class_names=None):
    """Export a tree as Graphviz dot (``-type graphviz``) or a JavaScript function (``-type js``)."""
    tree, classes = _load_model("export", model)
    fname = (lambda f: feature_names[f]) if feature_names else (lambda f: f"x[{f}]")
    if "js" in str(options):
        def rec(k, ind):
            if tree.feature[k] < 0:
                v = tree.value[k]
                return f"{ind}return {int(np.argmax(v)) if len(v) > 1 else v[0]};\n"
            op = "==" if tree.is_cat(k) else "<="
            return (f"{ind}if ({fname(tree.feature[k])} {op} {tree.threshold[k]}) {{\n" +
                    rec(tree.left[k], ind + "  ") + f"{ind}}} else {{\n" + rec(tree.right[k], ind + "  ") +
                    f"{ind}}}\n")
        return "function predict(x) {\n" + rec(0, "  ") + "}"
    lines = ["digraph Tree {", " node [shape=box];"]
    for k in range(len(tree.feature)):
        if tree.feature[k] < 0:
            v = tree.value[k]
            lab = (class_names[int(np.argmax(v))] if class_names else int(np.argmax(v))) if len(v) > 1 else v[0]
            lines.append(f' {k} [label="{lab}"];')
        else:
            op = "==" if tree.is_cat(k) else "<="
            lines.append(f' {k} [label="{fname(tree.feature[k])} {op} {tree.threshold[k]:.6g}"];')
            lines.append(f" {k} -> {tree.left[k]} [label=\"yes\"];")
            lines.append(f" {k} -> {tree.right[k]} [label=\"no\"];")
    lines.append("}")
    return "\n".join(lines)


@udf("decision_path")
def decision_path(model_id, model, features, options=None):
    """The sequence of split tests taken by one row."""
    tree, _ = _load_model(model_id, model)
    x = features
    if x is not None and len(x) and isinstance(list(x)[0], str):
        x = _to_dense([x])[0].tolist()
    path = []
    k = 0
    while tree.feature[k] >= 0:
        f, t = tree.feature[k], tree.threshold[k]
        go_left = tree.goes_left(k, x[f])
        if tree.is_cat(k):
            path.append(f"{f} {'==' if go_left else '!='} {t:.6g}")
        else:
            path.append(f"{f} {'<=' if go_left else '>'} {t:.6g}")
        k = tree.left[k] if go_left else tree.right[k]
    path.append(f"value={tree.value[k]}")
    return path


def register_sql(reg):
    reg("train_randomforest_classifier", lambda: RandomForestClassifier)
    reg("train_randomforest_regressor", lambda: RandomForestRegressor)
    reg("train_randomforest_regr", lambda: RandomForestRegressor)
    reg("train_gradient_tree_boosting_classifier", lambda: GradientTreeBoostingClassifier)


_P = _native.c_p
_I64 = _native.c_i64
_native.register_hip("hm_hist_build", [_P, C.c_int, C.c_int, C.c_int, _P, _P, C.c_int, _P, _P, C.c_int,
                                       C.c_int, _P, C.c_int, _P])
_native.register_host("hm_hist_build_cpu", [_P, C.c_int, C.c_int, C.c_int, _P, _P, C.c_int, _P, _P, C.c_int,
                                            C.c_int, _P])
_native.register_hip("hm_tree_predict", [_P, _I64, C.c_int] + [_P] * 7 + [C.c_int, C.c_int, _P, C.c_int,
                                                                          _P, _P])
_native.register_host("hm_tree_predict_cpu", [_P, _I64, C.c_int] + [_P] * 7 + [C.c_int, C.c_int, _P,
                                                                               C.c_int, _P])
_native.register_hip("hm_quantize", [_P, _I64, C.c_int, C.c_int, _P, C.c_int, _P, _P])
_native.register_host("hm_quantize_cpu", [_P, _I64, C.c_int, C.c_int, _P, C.c_int, _P])
_native.register_hip("hm_absmax_cols", [_P, _I64, C.c_int, _P, _P])
_native.register_hip("hm_route_rows", [_P, _I64, C.c_int, _I64, C.c_int, C.c_int] + [_P] * 5 + [C.c_int, C.c_int, _P])
_native.register_host("hm_route_rows_cpu", [_P, _I64, C.c_int] + [_P] * 5 + [C.c_int])
_native.register_hip("hm_split_find", [_P] * 10 + [_P])
_native.register_host("hm_split_find_cpu", [_P] * 10)
_native.register_hip("hm_partition_count", [_P, _I64, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P, C.c_int, _P])
_native.register_hip("hm_partition_scatter", [_P, _I64, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P,
                                              _P, _P, C.c_int, _P])
_native.register_hip("hm_gbt2_stats", [_P, _P, _P, _I64, _P, _P, _P, _P])
_native.register_hip("hm_leaf_sums", [_P, _P, _P, _I64, C.c_int, _P, C.c_int, _P])
_native.register_hip("hm_leaf_newton", [_P, _P, C.c_int, _P, _P])
_native.register_hip("hm_bootstrap_counts", [_P, _I64, C.c_int, C.c_uint64, _P, _P])
_native.register_hip("hm_hist_sibling_heap", [_P, _P, _P, _P, _I64, C.c_int, _P, _P])
_native.register_hip("hm_route_count", [_P, _I64, C.c_int, _I64, C.c_int, _P, _P, _P, _P, _P, C.c_int, _P, C.c_int, C.c_int,
                                        C.c_int, C.c_int, _P, C.c_int, _P])
_native.register_hip("hm_hist_sibling", [_P, _P, _P, _P, _I64, C.c_int, _P, _P])
_native.register_hip("hm_gbt_stats", [_P, _P, _P, _I64, _P, _P, _P])
_native.register_hip("hm_xgb_stats", [_P, _P, _P, _I64, _P, _P, _P])
_native.register_hip("hm_level_finalize", [_P] * 21)
_native.register_hip("hm_gbt_apply", [_P, C.c_int, C.c_int, _P, C.c_int, _P, _I64, C.c_float, C.c_int, _P])
