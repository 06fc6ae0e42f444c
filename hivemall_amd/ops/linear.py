"""Online linear family ops: gfx950 kernel (``csrc/kernels/linear.hip``) on ``cuda`` tensors,
OpenMP C++ engine (``csrc/host/linear_cpu.cpp``) on CPU tensors.  Both execute the rules of
``csrc/kernels/linear_rules.h``.

State layout (``LinearState``):
  S        f32 [R, L, dims, 4]   per (replica, label, feature): {w, s1, s2, s3}
  touched  u8  [R, dims]         feature seen by the replica (mix + model-table export)
  RS       f32 [R, 8]            per-replica scalars (step t, online variance, Eve, ...)
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import _native

ALGOS = {
    "perceptron": 0, "pa": 1, "pa1": 2, "pa2": 3, "cw": 4, "arow": 5, "arowh": 6, "scw": 7,
    "scw2": 8, "adagrad_rda": 9, "logress": 10, "pa1_regr": 11, "pa2_regr": 12, "pa1a_regr": 13,
    "pa2a_regr": 14, "arow_regr": 15, "arowe_regr": 16, "arowe2_regr": 17, "adagrad_regr": 18,
    "adadelta_regr": 19, "general": 20,
}
COVAR_ALGOS = {"cw", "arow", "arowh", "scw", "scw2", "arow_regr", "arowe_regr", "arowe2_regr"}

LOSSES = {
    "hinge": 0, "hingeloss": 0,
    "log": 1, "logloss": 1, "logistic": 1, "logisticloss": 1,
    "squaredhinge": 2, "squared_hinge": 2, "squaredhingeloss": 2,
    "modifiedhuber": 3, "modified_huber": 3, "modifiedhuberloss": 3,
    "squared": 4, "squaredloss": 4, "squared_loss": 4,
    "quantile": 5, "quantileloss": 5,
    "epsilon_insensitive": 6, "epsiloninsensitive": 6, "epsiloninsensitiveloss": 6,
    "squared_epsilon_insensitive": 7, "squaredepsiloninsensitive": 7,
    "squaredepsiloninsensitiveloss": 7,
    "huber": 8, "huberloss": 8,
}
CLASSIFICATION_LOSSES = {0, 1, 2, 3}
OPTIMIZERS = {
    "sgd": 0, "momentum": 1, "nesterov": 2, "adagrad": 3, "rmsprop": 4, "rmspropgraves": 5,
    "rmsprop_graves": 5, "adadelta": 6, "adam": 7, "nadam": 8, "eve": 9, "adam_hd": 10,
    "adamhd": 10,
}
REGS = {"no": 0, "none": 0, "l1": 1, "l2": 2, "elasticnet": 3, "elastic_net": 3, "rda": 4}
ETAS = {"fixed": 0, "simple": 1, "inverse": 2, "inv": 2}


class LinParams(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("algo", "loss", "opt", "reg", "eta", "amsgrad", "n_labels")] + [
        (n, C.c_float) for n in ("eta0", "power_t", "total_steps", "lambda_", "l1_ratio", "c", "r",
                                 "phi", "epsilon", "alpha", "beta1", "beta2", "eps", "rho", "decay",
                                 "beta_hd", "scale", "quantile_tau", "huber_c", "init_covar")]


@dataclass
class LinearState:
    S: torch.Tensor
    touched: torch.Tensor
    RS: torch.Tensor
    covar: bool
    gacc: torch.Tensor | None = None
    tlist: torch.Tensor | None = None
    meta: dict = field(default_factory=dict)

    @property
    def R(self) -> int:
        return self.S.shape[0]

    @property
    def L(self) -> int:
        return self.S.shape[1]

    @property
    def dims(self) -> int:
        return self.S.shape[2]

    @property
    def device(self):
        return self.S.device


def new_state(R: int, L: int, dims: int, device, covar: bool, init_covar: float = 1.0,
              mini_batch: int = 1) -> LinearState:
    S = torch.zeros((R, L, dims, 4), dtype=torch.float32, device=device)
    if covar:
        S[..., 1] = init_covar
    st = LinearState(S, torch.zeros((R, dims), dtype=torch.uint8, device=device),
                     torch.zeros((R, 8), dtype=torch.float32, device=device), covar)
    if mini_batch > 1 and S.is_cuda:
        st.gacc = torch.zeros((R, dims, 2), dtype=torch.float32, device=device)
        cap = max(64 * 8, min(dims, 1 << 22))
        st.tlist = torch.zeros((R, cap), dtype=torch.int32, device=device)
        st.meta["touched_cap"] = cap
    return st


def _ip(st: LinearState, mini_batch: int) -> np.ndarray:
    return np.array([st.R, st.dims, st.L, mini_batch, st.meta.get("touched_cap", 0)], dtype=np.int32)


def train_pass(st: LinearState, P: LinParams, indptr: torch.Tensor, idx: torch.Tensor,
               val: torch.Tensor | None, y: torch.Tensor, order: torch.Tensor | None = None,
               mini_batch: int = 1) -> torch.Tensor:
    """One pass over the rows (each replica over its shard).  Returns per-replica loss sums."""
    n = indptr.numel() - 1
    dev = st.device
    for t in (indptr, idx, val, y, order):
        if t is not None:
            assert t.device == dev and t.is_contiguous(), "tensor device/layout mismatch"
    assert indptr.dtype == torch.int64 and idx.dtype == torch.int32 and y.dtype == torch.float32
    assert y.numel() >= n
    if val is not None:
        assert val.dtype == torch.float32 and val.numel() == idx.numel()
    if order is not None:
        assert order.dtype == torch.int32 and order.numel() == n
    loss = torch.zeros(st.R, dtype=torch.float64, device=dev)
    ip = _ip(st, mini_batch)
    p = _native.ptr
    args = [C.addressof(P), ip.ctypes.data, C.c_int64(n), p(indptr), p(idx), p(val), p(y), p(order),
            p(st.S), p(st.touched), p(st.RS), p(loss)]
    if dev.type == "cuda":
        if mini_batch > 1 and st.gacc is None:
            st.gacc = torch.zeros((st.R, st.dims, 2), dtype=torch.float32, device=dev)
            cap = max(64 * 8, min(st.dims, 1 << 22))
            st.tlist = torch.zeros((st.R, cap), dtype=torch.int32, device=dev)
            st.meta["touched_cap"] = cap
            ip = _ip(st, mini_batch)
            args[1] = ip.ctypes.data
        rc = _native.hip().hm_linear_train(*args, p(st.gacc), p(st.tlist), _native.stream_of(dev))
        _native.check(rc, "hm_linear_train")
    else:
        rc = _native.host().hm_linear_train_cpu(*args)
        if rc != 0:
            raise RuntimeError(f"hm_linear_train_cpu failed: {rc}")
    return loss


# Rows in flight = waves.  The Hogwild quality knob: a hot feature of a Zipf stream is read and
# rewritten by every concurrent row that holds it, so the fraction of its updates that survive
# falls with concurrency.  Measured on 2M Criteo-shaped rows at 2^24 dims, one AdaGrad epoch
# (sequential CPU engine: held-out logloss 0.4789; profiles/linear_shared_r2o_nt.log):
#   8192 waves 0.623-0.670 @ 65-230 M rows/s, 2048: 0.513-0.553 @ 108-183 M, 512: 0.4985 @ 47-56 M
SHARED_WAVES = 512


def shared_waves(n_rows: int, cap: int = SHARED_WAVES) -> int:
    """Waves of a shared-table pass: enough rows per wave to amortise its scalars, at most
    ``cap`` rows in flight."""
    return int(max(1, min(cap, n_rows // 8)))


def new_shared_state(dims: int, device, n_rows: int, waves: int | None = None, replicas: int = 1,
                     reload: bool = True, nt: bool = True) -> LinearState:
    """Shared-table Hogwild state (csrc/kernels/linear.hip linear_shared_kernel): ``replicas``
    tables S [R, 1, dims, 4] each shared by the waves of one XCD (R = 1 or a multiple of 8),
    touched [R, dims], per-wave scalars RS [W, 8]."""
    W = int(waves) if waves else shared_waves(n_rows)
    R = int(replicas)
    if R != 1 and (R % 8 or (W + 3) // 4 < R):
        raise ValueError(f"shared engine: replicas must be 1 or a multiple of 8 with >= 4 * R waves "
                         f"(R={R}, W={W})")
    st = LinearState(torch.zeros((R, 1, dims, 4), dtype=torch.float32, device=device),
                     torch.zeros((R, dims), dtype=torch.uint8, device=device),
                     torch.zeros((W, 8), dtype=torch.float32, device=device), False)
    st.meta["shared"] = True
    st.meta["reload"] = bool(int(os.environ.get("HM_LINEAR_RELOAD", int(reload))))
    st.meta["nt"] = bool(nt)
    return st


HOT_MAX = 4096          # <= csrc/kernels/linear.hip HM_HOT_MAX; 48 KB of LDS accumulators
# hot-feature flush schedule (csrc/kernels/linear.hip HOT): rows per wave per chunk, rows an
# accumulator must hold to be applied before the periodic flush, chunks between periodic flushes
# (profiles/linear_hot_r3/: 2 M Criteo-shaped rows, 2^24 dims, AdaGrad-RDA logistic)
HOT_CHUNK, HOT_MIN_ROWS, HOT_EVERY = 32, 32, 8


def hot_rule(P: LinParams) -> bool:
    """Rules whose hot features can be pre-aggregated: the general learner's AdaGrad with no / L2
    regularisation and AdaGrad-RDA, whose step is normalised by the accumulated squared
    gradient, so a block's summed gradient takes a bounded step.  Plain SGD applies the sum at
    full rate and diverges (measured: held-out logloss 273 at eta0 0.05); applying the block's
    mean gradient through the other rules' updates diverges for momentum and the Adam family
    (profiles/r4/linear_rules_mean_step.jsonl).  ``HM_LINEAR_HOT=0`` disables the
    pre-aggregation."""
    if os.environ.get("HM_LINEAR_HOT", "1") == "0":
        return False
    return (P.algo == ALGOS["general"] and P.opt == OPTIMIZERS["adagrad"]
            and P.reg in (REGS["no"], REGS["l2"], REGS["rda"]) and P.n_labels == 1)


def hot_owner_rule(P: LinParams) -> bool:
    """The general learner's other rules (csrc/kernels/linear.hip hot_owner_rule): their hot
    features are applied by one owner thread each, as n sequential steps of the chunk's mean
    gradient (hot_nstep), on a single table.  ``HM_LINEAR_HOT_OWNER=0`` leaves them Hogwild."""
    if os.environ.get("HM_LINEAR_HOT", "1") == "0" or os.environ.get("HM_LINEAR_HOT_OWNER", "1") == "0":
        return False
    # AdaGrad with L1 / elastic-net regularisation only: its n-step update is normalised by the
    # accumulated squared gradient, so a chunk's thousands of steps stay bounded.  The closed
    # forms of the unnormalised or exponentially-averaged rules take those steps without the
    # sequential learner's feedback and diverge (held-out logloss +0.5 .. +278 for SGD, momentum,
    # RMSprop, AdaDelta and the Adam family at 512 rows in flight,
    # profiles/r4/linear_rules_owner_all_rules.jsonl)
    return (P.algo == ALGOS["general"] and P.opt == OPTIMIZERS["adagrad"]
            and P.reg in (REGS["l1"], REGS["elasticnet"]) and P.n_labels == 1)


# Rows in flight of the shared-table engine per rule (``-shared_waves 0``), from the held-out
# logloss vs the sequential CPU engine at -dims 2^24 (1 M Criteo-shaped rows, every rule at a
# step size where the sequential learner converges; benchmarks/linear_rules_parity.py,
# profiles/r4/linear_rules_*.jsonl, docs/compat.md "Shared-table engine: per-rule parity"):
#  * AdaGrad with no / L2 regularisation and AdaGrad-RDA (hot features pre-aggregated as sums):
#    -6e-4 .. -1.1e-3 at 512 and 1,024 rows in flight -> 1,024 (~98 M rows/s);
#  * AdaGrad-L1 / elastic net (hot features in owner mode): +1.8e-3 .. +1.9e-3 at 512 -> 512
#    (~94 M rows/s);
#  * SGD, momentum, Nesterov, RMSprop(-Graves), AdaDelta (+3.4e-3 .. +8e-3 at 512) and the Adam
#    family: +2.5e-3 .. +1e-2 at 16 ..
#    1,024 rows in flight (plain Hogwild; their closed-form hot-feature updates diverge), and
#    within 1.3e-3 at <= 8 (linear_rules_fewwaves.jsonl) -> routed to 8 rows in flight
#    (~1.7 M rows/s, 3x the CPU engine).  -shared_waves 512 buys ~55x the rate at that gap.
SEQ_WAVES = 8


# Near-sequential engine (linear_seq_kernel, ``-engine seq``; round 6): W consecutive rows in
# flight, all on ONE XCD.  Held-out logloss minus the sequential CPU engine's after one epoch of
# 1 M Criteo-shaped rows at -dims 2^24, seeds 5 / 11 / 23 (profiles/r6/linear_seq_*.jsonl):
#   on one XCD, 512 rows: SGD / momentum / Nesterov / RMSprop(-Graves) / AdaDelta -1.8e-3 ..
#     +1.5e-3 (one AdaDelta run -3.3e-3, i.e. better than sequential) at 120-130 M rows/s;
#     Adam +0.7e-3 .. +2.7e-3 at 84 M; at 256 rows Adam -0.3e-3 .. +1.4e-3 at 53 M;
#   the same rows dealt over all 8 XCDs: +3e-3 .. +6e-3 at any W from 8 to 128 — the per-XCD
#     L2s are not coherent, so an XCD keeps reading its own copy of a hot feature's line;
#   AdaGrad (+0.5e-2 .. +2e-2) stays on the shared engine's hot-feature sums.
#   RMSprop-Graves at 512 rows measured -0.56e-3 on the sweep but +3.05e-3 once in the GPU test
#     suite (profiles/r6/val3/pytest_gpu.log): it runs at 256 (-0.68e-3 at 78 M rows/s).
SEQ_ENGINE_WAVES = 512
_SEQ_WAVES_BY_OPT = {"adam": 256, "nadam": 256, "adam_hd": 256, "rmspropgraves": 256, "eve": 128}
# HM_LINEAR_SEQ=0: the rules of seq_rule stay on the shared engine at SEQ_WAVES rows in flight
_SEQ_AUTO = os.environ.get("HM_LINEAR_SEQ", "1") != "0"


def seq_rule(P: LinParams) -> bool:
    """Rules routed to the near-sequential engine by ``-engine auto``: the general learner's
    rules that neither pre-aggregate (hot_rule) nor own (hot_owner_rule) their hot features,
    i.e. every optimizer but AdaGrad."""
    return (_SEQ_AUTO and P.algo == ALGOS["general"] and P.n_labels == 1 and not hot_rule(P)
            and not hot_owner_rule(P) and P.opt != OPTIMIZERS["adagrad"])


def seq_waves(P: LinParams) -> int:
    """Default rows in flight of the near-sequential engine for the rule (table above)."""
    for name, w in _SEQ_WAVES_BY_OPT.items():
        if P.opt == OPTIMIZERS[name]:
            return w
    return SEQ_ENGINE_WAVES


def rule_waves(P: LinParams) -> int:
    """Default rows in flight of the shared-table engine for the rule (see above)."""
    if hot_rule(P):
        return 1024
    general = P.algo == ALGOS["general"]
    if hot_owner_rule(P):
        return 512
    if general:
        return SEQ_WAVES
    return SHARED_WAVES


def hot_features(st: LinearState, P: LinParams, idx: torch.Tensor, n_rows: int):
    """The features the shared-table kernel pre-aggregates per block instead of updating them
    Hogwild (csrc/kernels/linear.hip, HOT): the at most ``HOT_MAX`` most frequent features of
    the pass that more than one in-flight row is expected to hit (count >= n_rows / W), for the
    rules of ``hot_rule``.  Returns (hot_slot i32 [dims], hot_feat i32 [H]) or None.
    Cached per index tensor (epochs reuse it).  ``HM_LINEAR_HOT=0`` disables."""
    if not (hot_rule(P) or (hot_owner_rule(P) and st.R == 1)):
        return None
    # keyed on the tensor object itself (weakly) and its version counter: a later pass whose
    # index tensor happens to land at a freed address must not reuse this pass's hot set
    key = (idx.numel(), st.dims, n_rows, idx._version)
    hit = st.meta.get("hot")
    if hit is not None and hit[0]() is idx and hit[1] == key:
        return hit[2]
    W = st.RS.shape[0]
    # counts from a strided sample of the indices (a prime stride: coprime with any row width
    # it does not divide, so every field is sampled): the hot set only needs the frequent features, and a full bincount of
    # a large pass costs as much as a training epoch
    want = idx.numel() // (1 << 22)
    stride = next((q for q in (1, 17, 31, 61, 127, 251, 509, 1021) if q >= want), 2039)
    ids = idx[::stride].long()
    ids = ids[(ids >= 0) & (ids < st.dims)]
    cnt = torch.bincount(ids, minlength=st.dims)
    vals, feats = torch.topk(cnt, min(HOT_MAX, st.dims))
    feats = feats[vals * stride >= max(2, n_rows // max(1, W))].to(torch.int32)
    res = None
    if feats.numel():
        slot = torch.full((st.dims,), -1, dtype=torch.int32, device=idx.device)
        slot[feats.long()] = torch.arange(feats.numel(), dtype=torch.int32, device=idx.device)
        res = (slot, feats.contiguous())
    st.meta["hot"] = (weakref.ref(idx), key, res)
    return res


def train_pass_shared(st: LinearState, P: LinParams, indptr: torch.Tensor, idx: torch.Tensor,
                      val: torch.Tensor | None, y: torch.Tensor, t0: int,
                      order: torch.Tensor | None = None) -> torch.Tensor:
    """One Hogwild pass of the shared tables over the rows; step of row q = t0 + q + 1.  Returns
    per-wave loss sums."""
    n = indptr.numel() - 1
    dev = st.device
    assert dev.type == "cuda", "the shared-table engine is a device engine"
    assert indptr.dtype == torch.int64 and idx.dtype == torch.int32 and y.dtype == torch.float32
    assert y.numel() >= n and (val is None or val.numel() == idx.numel())
    for t in (indptr, idx, val, y, order):
        if t is not None:
            assert t.device == dev and t.is_contiguous(), "tensor device/layout mismatch"
    W = st.RS.shape[0]
    loss = torch.zeros(W, dtype=torch.float64, device=dev)
    p = _native.ptr
    hot = hot_features(st, P, idx, n) if W > 1 else None
    hs, hf, H = (hot[0], hot[1], hot[1].numel()) if hot is not None else (None, None, 0)
    hacc = None
    if H and not hot_rule(P):                 # owner mode: zeroed [H] accumulators (re-zeroed by the pass)
        hacc = st.meta.get("hacc")
        if hacc is None or hacc.shape[0] < H:
            hacc = st.meta["hacc"] = torch.zeros((max(H, HOT_MAX), 4), dtype=torch.float32, device=dev)
    # rows per wave per chunk: HOT_CHUNK, or fewer so that a short pass still has >= 32 chunk
    # ends at which the hot features' sums are applied
    ch = int(os.environ.get("HM_LINEAR_HOT_CH", max(1, min(HOT_CHUNK, n // max(1, W * 32)))))
    hmin = int(os.environ.get("HM_LINEAR_HOT_MIN", min(HOT_MIN_ROWS, 4 * ch)))
    # a feature below min_rows per block per chunk is applied every `hevery` chunks: at most
    # HOT_EVERY, and at least 16 times over the pass — a short pass (200 K rows at 1,024 rows in
    # flight is 7 chunks) would otherwise hold most hot features' sums until its last chunk,
    # one huge step at the end (held-out logloss 0.61-0.67 vs the sequential 0.479-0.487)
    nchunks = -(-n // max(1, W * ch))
    hevery = int(os.environ.get("HM_LINEAR_HOT_EVERY", max(1, min(HOT_EVERY, nchunks // 16))))
    rc = _native.hip().hm_linear_train_shared(C.addressof(P), C.c_int64(n), st.dims, C.c_int64(int(t0)), W,
                                              st.R, int(st.meta.get("reload", False)),
                                              int(st.meta.get("nt", True)),
                                              p(indptr), p(idx), p(val), p(y), p(order), p(st.S),
                                              p(st.touched), p(st.RS), p(loss), p(hs), p(hf), H, ch, hmin, hevery,
                                              p(hacc),
                                              _native.stream_of(dev))
    _native.check(rc, "hm_linear_train_shared")
    return loss


def new_seq_state(dims: int, device, waves: int, spread: int = 8) -> LinearState:
    """Near-sequential engine state (csrc/kernels/linear.hip linear_seq_kernel): one table
    S [1, 1, dims, 4], touched [1, dims], per-wave scalars RS [W, 8]; ``spread`` 8 keeps the W
    waves on one XCD (1: dealt over all of them)."""
    st = LinearState(torch.zeros((1, 1, dims, 4), dtype=torch.float32, device=device),
                     torch.zeros((1, dims), dtype=torch.uint8, device=device),
                     torch.zeros((int(waves), 8), dtype=torch.float32, device=device), False)
    st.meta.update(seq=True, spread=int(spread), nt=True)
    return st


def train_pass_seq(st: LinearState, P: LinParams, indptr: torch.Tensor, idx: torch.Tensor,
                   val: torch.Tensor | None, y: torch.Tensor, t0: int,
                   order: torch.Tensor | None = None) -> torch.Tensor:
    """One pass of the near-sequential engine (row q on wave q % W, step t0 + q + 1).  Returns
    per-wave loss sums."""
    n = indptr.numel() - 1
    dev = st.device
    assert dev.type == "cuda" and st.meta.get("seq"), "near-sequential engine state on a GPU"
    assert indptr.dtype == torch.int64 and idx.dtype == torch.int32 and y.dtype == torch.float32
    assert y.numel() >= n and (val is None or val.numel() == idx.numel())
    for t in (indptr, idx, val, y, order):
        if t is not None:
            assert t.device == dev and t.is_contiguous(), "tensor device/layout mismatch"
    W = st.RS.shape[0]
    loss = torch.zeros(W, dtype=torch.float64, device=dev)
    p = _native.ptr
    rc = _native.hip().hm_linear_train_seq(C.addressof(P), C.c_int64(n), st.dims, C.c_int64(int(t0)), W,
                                           int(st.meta.get("spread", 8)), int(st.meta.get("nt", True)),
                                           p(indptr), p(idx), p(val), p(y), p(order), p(st.S),
                                           p(st.touched), p(st.RS), p(loss), _native.stream_of(dev))
    _native.check(rc, "hm_linear_train_seq")
    return loss


def new_minibatch_state(dims: int, device, max_rows_per_batch: int, max_nnz: int) -> LinearState:
    """Mini-batch engine state (csrc/kernels/linear.hip hm_linear_train_minibatch): one table
    S [1, 1, dims, 4] plus the batch buffers (gradient sums, touched marks, the batch's feature
    list and two list counters), all zeroed."""
    st = LinearState(torch.zeros((1, 1, dims, 4), dtype=torch.float32, device=device),
                     torch.zeros((1, dims), dtype=torch.uint8, device=device),
                     torch.zeros((1, 8), dtype=torch.float32, device=device), False)
    cap = int(min(dims, max(1, max_rows_per_batch) * max(1, max_nnz)))
    st.meta.update(minibatch=True, ga=torch.zeros(dims, dtype=torch.float32, device=device),
                   mark=torch.zeros(dims, dtype=torch.int32, device=device),
                   list=torch.zeros(cap, dtype=torch.int32, device=device),
                   cnt=torch.zeros(2, dtype=torch.int32, device=device))
    return st


def minibatch_rule(P: LinParams) -> bool:
    """Rules of the mini-batch engine: the general learner, one label, any optimizer but Eve
    (whose per-row loss feedback is a sequential chain, not a batch rule)."""
    return P.algo == ALGOS["general"] and P.n_labels == 1 and P.opt != OPTIMIZERS["eve"]


def train_pass_minibatch(st: LinearState, P: LinParams, indptr: torch.Tensor, idx: torch.Tensor,
                         val: torch.Tensor | None, y: torch.Tensor, t0: int, M: int,
                         order: torch.Tensor | None = None) -> torch.Tensor:
    """One pass of the mini-batch engine (batches of M rows in order; row q's step t0 + q + 1).
    Returns the pass's loss sum (device, [1])."""
    n = indptr.numel() - 1
    dev = st.device
    assert dev.type == "cuda" and st.meta.get("minibatch"), "mini-batch engine state on a GPU"
    assert indptr.dtype == torch.int64 and idx.dtype == torch.int32 and y.dtype == torch.float32
    for t in (indptr, idx, val, y, order):
        if t is not None:
            assert t.device == dev and t.is_contiguous(), "tensor device/layout mismatch"
    # the batch buffers are zeroed scratch (every batch leaves them zeroed): a state restored from
    # a checkpoint (io/checkpoint.py keeps only JSON scalars of state.meta) gets fresh ones
    for k, shape, dt in (("ga", (st.dims,), torch.float32), ("mark", (st.dims,), torch.int32),
                         ("cnt", (2,), torch.int32), ("list", (1,), torch.int32)):
        if not isinstance(st.meta.get(k), torch.Tensor) or st.meta[k].device != dev:
            st.meta[k] = torch.zeros(shape, dtype=dt, device=dev)
    if n > 0:
        nnz = int((indptr[1:] - indptr[:-1]).max().item())
        need = min(st.dims, M * max(1, nnz))
        if st.meta["list"].numel() < need:
            st.meta["list"] = torch.zeros(need, dtype=torch.int32, device=dev)
    loss = torch.zeros(1, dtype=torch.float64, device=dev)
    p = _native.ptr
    rc = _native.hip().hm_linear_train_minibatch(C.addressof(P), C.c_int64(n), st.dims, C.c_int64(int(t0)), int(M),
                                                 p(indptr), p(idx), p(val), p(y), p(order), p(st.S),
                                                 p(st.touched), p(st.meta["ga"]), p(st.meta["mark"]),
                                                 p(st.meta["list"]), p(st.meta["cnt"]), p(loss),
                                                 _native.stream_of(dev))
    _native.check(rc, "hm_linear_train_minibatch")
    return loss


def mix_reduce(st: LinearState, kld: bool):
    """Compact per-element sums (num, den, cnt) over the touching replicas."""
    R, L, dims = st.R, st.L, st.dims
    dev = st.device
    if dev.type == "cuda":
        num = torch.empty(L * dims, dtype=torch.float32, device=dev)
        den = torch.empty_like(num)
        cnt = torch.empty_like(num)
        rc = _native.hip().hm_linear_mix_reduce(_native.ptr(st.S), _native.ptr(st.touched), R, dims,
                                                L, int(kld), _native.ptr(num), _native.ptr(den),
                                                _native.ptr(cnt), _native.stream_of(dev))
        _native.check(rc, "hm_linear_mix_reduce")
        return num, den, cnt
    t = st.touched.to(torch.float32).view(R, 1, dims)          # [R,1,dims]
    w = st.S[..., 0]
    if kld:
        inv = 1.0 / st.S[..., 1].clamp_min(1e-12)
        num = (w * inv * t).sum(0)
        den = (inv * t).sum(0)
    else:
        num = (w * t).sum(0)
        den = t.expand(R, L, dims).sum(0)
    cnt = t.expand(R, L, dims).sum(0)
    return num.reshape(-1).contiguous(), den.reshape(-1).contiguous(), cnt.reshape(-1).contiguous()


def mix_apply(st: LinearState, kld: bool, num, den, cnt):
    """Write the mixed weights (and covariance) into every replica; return compact (w, cov)."""
    R, L, dims = st.R, st.L, st.dims
    dev = st.device
    w_out = torch.empty(L * dims, dtype=torch.float32, device=dev)
    cov_out = torch.empty_like(w_out) if st.covar else None
    if dev.type == "cuda":
        rc = _native.hip().hm_linear_mix_apply(_native.ptr(st.S), R, dims, L, int(kld),
                                               _native.ptr(num), _native.ptr(den), _native.ptr(cnt),
                                               _native.ptr(w_out), _native.ptr(cov_out),
                                               _native.stream_of(dev))
        _native.check(rc, "hm_linear_mix_apply")
        return w_out.view(L, dims), (cov_out.view(L, dims) if cov_out is not None else None)
    num, den, cnt = (x.view(L, dims) for x in (num, den, cnt))
    hit = cnt > 0
    w = torch.where(hit, num / den.clamp_min(1e-30), st.S[0, ..., 0])
    st.S[..., 0] = torch.where(hit.unsqueeze(0), w.unsqueeze(0), st.S[..., 0])
    cov = None
    if st.covar:
        if kld:
            cv = torch.where(hit, cnt / den.clamp_min(1e-30), st.S[0, ..., 1])
            st.S[..., 1] = torch.where(hit.unsqueeze(0), cv.unsqueeze(0), st.S[..., 1])
            cov = cv
        else:
            cov = st.S[0, ..., 1].clone()
    return w.contiguous(), cov


def predict_scores(w: torch.Tensor, indptr: torch.Tensor, idx: torch.Tensor,
                   val: torch.Tensor | None, cov: torch.Tensor | None = None):
    """Scores [n, L] (and xᵀΣx variances when ``cov`` is given) for CSR rows."""
    L, dims = w.shape
    n = indptr.numel() - 1
    dev = w.device
    out = torch.empty((n, L), dtype=torch.float32, device=dev)
    var = torch.empty((n, L), dtype=torch.float32, device=dev) if cov is not None else None
    p = _native.ptr
    w = w.contiguous()
    cov = cov.contiguous() if cov is not None else None
    if dev.type == "cuda":
        rc = _native.hip().hm_linear_predict(p(w), dims, L, p(indptr), p(idx), p(val), C.c_int64(n),
                                             p(out), p(cov), p(var), _native.stream_of(dev))
        _native.check(rc, "hm_linear_predict")
    else:
        _native.host().hm_linear_predict_cpu(p(w), dims, L, p(indptr), p(idx), p(val), C.c_int64(n),
                                             p(out), p(cov), p(var))
    return out, var


_P = _native.c_p
_native.register_hip("hm_linear_train", [_P, _P, _native.c_i64] + [_P] * 11 + [_P])
_native.register_host("hm_linear_train_cpu", [_P, _P, _native.c_i64] + [_P] * 9)
_native.register_hip("hm_linear_train_shared", [_P, _native.c_i64, C.c_int, _native.c_i64, C.c_int, C.c_int,
                                              C.c_int, C.c_int] + [_P] * 9 + [_P, _P] + [C.c_int] * 4
                     + [_P, _P])
_native.register_hip("hm_linear_train_seq", [_P, _native.c_i64, C.c_int, _native.c_i64, C.c_int, C.c_int, C.c_int]
                     + [_P] * 9 + [_P])
_native.register_hip("hm_linear_train_minibatch", [_P, _native.c_i64, C.c_int, _native.c_i64, C.c_int]
                     + [_P] * 12 + [_P])
_native.register_hip("hm_linear_mix_reduce", [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P])
_native.register_hip("hm_linear_mix_apply", [_P, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P, _P])
_native.register_hip("hm_linear_predict", [_P, C.c_int, C.c_int, _P, _P, _P, _native.c_i64, _P, _P, _P, _P])
_native.register_host("hm_linear_predict_cpu", [_P, C.c_int, C.c_int, _P, _P, _P, _native.c_i64, _P, _P, _P])
