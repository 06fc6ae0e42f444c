"""Matrix factorization: ``train_mf_sgd``, ``train_mf_adagrad`` (biased MF), ``train_bprmf``
(BPR-MF, Rendle UAI'09) and the predictors ``mf_predict`` / ``bprmf_predict``.

Reference behaviour: Hivemall OnlineMatrixFactorizationUDTF, MatrixFactorizationSGDUDTF,
MatrixFactorizationAdaGradUDTF, BPRMatrixFactorizationUDTF, MFPredictionUDF,
BPRMFPredictionUDF, FactorizedModel (upstream core/src/main/java/hivemall/mf/; SURVEY.md
§2.3.5, K7/K8, O7).

MI355X design: P [n_users, kp] and Q [n_items, kp] fp32 tables in HBM; the kernels in
``csrc/kernels/mf.hip`` pack 64/next_pow2(k) ratings per wave64 and update Hogwild.  BPR can
sample its negatives on the device (user->items CSR + counter-based RNG), so an epoch is one
launch with no host round trip.  Bulk scoring (``recommend_topk``) is a bf16 GEMM on the
matrix cores (torch.matmul -> hipBLASLt) + ``torch.topk``.

Model tables (pinned, docs/compat.md O7):
  MF : (idx int, Pu array<float>, Qi array<float>, Bu float, Bi float, mu float)
  BPR: (idx int, Pu array<float>, Qi array<float>, Bi float)
one row per index that is a user and/or an item (NULL where it is not).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import pandas as pd
import torch

from .. import _native
from ..ops import topk_mips
from ..registry import udf
from ..utils.options import UDFArgumentException, flag, opt
from .base import MIX_OPTS, ConversionState, Learner, log
from ..utils.reduce import tmax

_ETAS = {"fixed": 0, "simple": 1, "inverse": 2, "inv": 2, "bolddriver": 0, "bold_driver": 0}
_BOLD = ("bolddriver", "bold_driver")


class BoldDriverEta:
    """``-eta bolddriver``: Hivemall's AdjustingEtaEstimator driven by the epoch loss
    (hivemall.common.EtaEstimator.AdjustingEtaEstimator).

    The rate is constant within an epoch; after each epoch whose loss is known against the
    previous one it is multiplied by 1.05 when the loss decreased and by 0.5 when it increased,
    capped at MAX_ETA = 1.0, and a non-finite product leaves it unchanged."""

    MAX_ETA = 1.0
    UP, DOWN = 1.05, 0.5

    def __init__(self, eta0: float):
        self.eta = float(eta0)
        self.prev_loss: float | None = None
        self.history = [self.eta]

    def epoch_end(self, loss: float) -> float:
        if self.prev_loss is not None:
            mult = self.DOWN if loss > self.prev_loss else self.UP
            new = self.eta * mult
            if np.isfinite(new):
                self.eta = min(self.MAX_ETA, new)
        self.prev_loss = float(loss)
        self.history.append(self.eta)
        return self.eta

MF_OPTS = [
    opt("factors", "factor", 10, int, "Number of latent factors", aliases=("k",)),
    opt("lambda", None, 0.03, float, "Regularization"),
    opt("mu", "mean_rating", 0.0, float, "Mean rating (initial)"),
    flag("update_mean", "update_mu", "Update the mean rating from the data"),
    opt("rankinit", None, "random", str, "Init: random | gaussian"),
    opt("maxval", "max_init_value", 1.0, float, "Max value for random init"),
    opt("min_init_stddev", None, 0.1, float, "Stddev for gaussian init"),
    opt("iters", "iterations", 1, int, "Iterations", aliases=("iter",)),
    opt("eta0", None, 0.1, float, "Initial learning rate"),
    opt("eta", None, "fixed", str, "Learning rate scheme: fixed, simple, inverse, bolddriver"),
    opt("power_t", None, 0.1, float, "Inverse scaling exponent"),
    opt("t", "total_steps", -1.0, float, "Total steps for -eta simple"),
    opt("eps", None, 1.0, float, "AdaGrad denominator constant"),
    opt("scale", None, 100.0, float, "Scaling factor",
        inert="factor accumulators are fp32 (no half-float scaling)"),
    flag("disable_bias", "no_bias", "Do not learn user/item biases"),
    opt("cv_rate", "convergence_rate", 0.005, float, "Convergence threshold"),
    flag("disable_cv", "disable_cvtest", "Disable convergence check"),
    opt("seed", None, -1, int, "Seed"),
    opt("grid", None, 0, int, "[engine] kernel grid override"),
] + MIX_OPTS

BPR_OPTS = [
    opt("factors", "factor", 10, int, "Number of latent factors", aliases=("k",)),
    opt("loss", "loss_function", "lnLogistic", str, "lnLogistic | logistic | sigmoid"),
    opt("iters", "iterations", 30, int, "Iterations", aliases=("iter",)),
    opt("reg", "lambda", 0.0001, float, "Default regularization"),
    opt("reg_u", None, None, float, "Regularization of user factors"),
    opt("reg_i", None, None, float, "Regularization of positive item factors"),
    opt("reg_j", None, None, float, "Regularization of negative item factors"),
    opt("reg_bias", None, 0.01, float, "Regularization of item biases"),
    opt("eta0", None, 0.005, float, "Initial learning rate"),
    opt("eta", None, "fixed", str, "Learning rate scheme: fixed, simple, inverse, bolddriver"),
    opt("power_t", None, 0.1, float, "Inverse scaling exponent"),
    opt("t", "total_steps", -1.0, float, "Total steps"),
    opt("init", None, "random", str, "Init: random | gaussian"),
    opt("maxval", "max_init_value", 1.0, float, "Max value for random init"),
    opt("min_init_stddev", None, 0.1, float, "Stddev for gaussian init"),
    flag("no_bias", "disable_bias", "Do not learn item biases"),
    opt("cv_rate", "convergence_rate", 0.005, float, "Convergence threshold"),
    flag("disable_cv", "disable_cvtest", "Disable convergence check"),
    opt("seed", None, -1, int, "Seed"),
    opt("samples_per_epoch", None, 0, int, "[engine] device-sampled triples per epoch (0 = #positives)"),
    opt("grid", None, 0, int, "[engine] kernel grid override"),
    flag("shard_model", None, "[engine] row-shard P, Q, Bi over the ranks (model parallel: each "
         "GPU holds 1/world of the tables; batches pull/push the rows they touch)"),
    opt("shard_batch", None, 1 << 20, int, "[engine] triples per pull/compute/push step with "
        "-shard_model"),
] + MIX_OPTS
_BPR_LOSS = {"lnlogistic": 0, "logistic": 1, "sigmoid": 2}


def _init_factors(n, k, kp, scheme, maxval, stddev, gen) -> torch.Tensor:
    T = torch.zeros(n, kp)
    if scheme == "gaussian":
        T[:, :k] = torch.randn(n, k, generator=gen) * stddev
    else:
        T[:, :k] = torch.rand(n, k, generator=gen) * (maxval / k)
    return T


def _dev(x, dtype, dev) -> torch.Tensor:
    """Host arrays or (device) tensors -> contiguous ``dtype`` tensor on ``dev``."""
    if torch.is_tensor(x):
        return x.to(dev, dtype).contiguous()
    return torch.as_tensor(np.asarray(x, dtype=torch.empty(0, dtype=dtype).numpy().dtype)).to(dev)


class _MFBase(Learner):
    SQL_DP = "shard"
    def mix(self) -> None:
        """Replica averaging of the factor tables over the ranks (SURVEY.md §2.6 BPR/MF row);
        AdaGrad accumulators stay local, as each upstream mapper keeps its own."""
        if self.state is None:
            return
        ts = [self.state[k] for k in ("P", "Q", "Bu", "Bi", "mu") if k in self.state]
        self.mix_tensors(ts, [self.seen_u, self.seen_i])

    def _eta0(self) -> float:
        """Learning rate of the current epoch: -eta0, or the bold driver's adjusted rate."""
        if str(self.cl["eta"]).lower() in _BOLD:
            if getattr(self, "bold", None) is None:
                self.bold = BoldDriverEta(float(self.cl["eta0"]))
            return self.bold.eta
        return float(self.cl["eta0"])

    def _epoch_end(self, loss: float) -> None:
        if getattr(self, "bold", None) is not None:
            self.bold.epoch_end(loss)

    def _epoch_mix(self, ep: int) -> None:
        mi = int(self.cl["mix_interval"])
        if mi > 0 and (ep + 1) % mi == 0:
            self.mix()

    def _factors(self):
        k = int(self.cl["factors"])
        if not 0 < k <= 64:
            raise UDFArgumentException(f"{self.NAME}: -factors must be in [1, 64]")
        return k

    def _ip(self, loss=0, max_tries=16):
        c = self.cl
        eta = str(c["eta"]).lower()
        if eta not in _ETAS:
            raise UDFArgumentException(f"{self.NAME}: unknown -eta {eta}")
        return np.array([self.k, self.kp, self.n_users, self.n_items, int(self.adagrad),
                         int(self.use_bias), 0, _ETAS[eta], loss, self.seed & 0x7FFFFFFF, max_tries,
                         self._grid(), int(os.environ.get("HM_MF_PLAIN_LOADS", "0") == "1"),
                         int(os.environ.get("HM_MF_ATOMIC", "1")), 0,
                         int(os.environ.get("HM_BPR_VARIANT", "0"))],
                        dtype=np.int32)

    # Hogwild concurrency cap: rows (users/items) per 256-thread block in flight.  Explicit MF
    # updates are atomic delta adds (HM_MF_ATOMIC=1, default): with them the held-out RMSE
    # curve equals the sequential engine's at every grid (fixture grid 1..36: 0.1438-0.1439;
    # ML-20M shape 0.3228 vs sequential 0.3217 after 12 epochs), while read-modify-write
    # stores lost concurrent updates of popular rows and never left the bias-only level
    # (profiles/mf_atomic_r2/).  So the grid is sized for throughput, as for BPR: 32 rows per
    # block (ML-20M: 852 blocks; 794 M ratings/s at 106 blocks, 847 M at 3,392).  With
    # HM_MF_ATOMIC=0 (A/B only) the old cap of 256 rows per block applies.
    ROWS_PER_BLOCK = 256
    ROWS_PER_BLOCK_ATOMIC = 32

    def _grid(self) -> int:
        """Hogwild concurrency cap: keep the number of ratings in flight well below the number
        of distinct rows they update (plain SGD diverges when many stale gradients of one
        popular item are summed).  ~1 block (4 waves) per ``ROWS_PER_BLOCK`` items/users,
        >= 1."""
        g = int(self.cl["grid"])
        if g > 0:
            return g
        rows = self.ROWS_PER_BLOCK
        if self.ROWS_PER_BLOCK_ATOMIC and os.environ.get("HM_MF_ATOMIC", "1") != "0":
            rows = self.ROWS_PER_BLOCK_ATOMIC
        return int(max(1, min(4096, min(self.n_users, self.n_items) // rows)))


class MatrixFactorization(_MFBase):
    """Biased MF with SGD (``train_mf_sgd``) or AdaGrad (``train_mf_adagrad``)."""
    NAME = "train_mf_sgd"
    OPTIONS = MF_OPTS
    ADAGRAD = False

    def __init__(self, options=None, device=None, **kw):
        super().__init__(options, device, **kw)
        self.k = self._factors()
        self.kp = self.k
        self.adagrad = self.ADAGRAD
        self.use_bias = not self.cl["disable_bias"]
        self.state = None
        self.t = 0
        self.cv = ConversionState(not self.cl["disable_cv"], self.cl["cv_rate"])

    def init_state(self, n_users, n_items):
        self.n_users, self.n_items = int(n_users), int(n_items)
        g = torch.Generator().manual_seed(self.seed)
        c = self.cl
        dev = self.device
        P = _init_factors(self.n_users, self.k, self.kp, c["rankinit"], c["maxval"], c["min_init_stddev"], g)
        Q = _init_factors(self.n_items, self.k, self.kp, c["rankinit"], c["maxval"], c["min_init_stddev"], g)
        st = dict(P=P.to(dev), Q=Q.to(dev), Bu=torch.zeros(self.n_users, device=dev),
                  Bi=torch.zeros(self.n_items, device=dev),
                  mu=torch.tensor([float(c["mu"])], device=dev))
        if self.adagrad:
            st.update(GP=torch.zeros_like(st["P"]), GQ=torch.zeros_like(st["Q"]),
                      GBu=torch.zeros_like(st["Bu"]), GBi=torch.zeros_like(st["Bi"]))
        self.state = st
        self.seen_u = torch.zeros(self.n_users, dtype=torch.bool, device=dev)
        self.seen_i = torch.zeros(self.n_items, dtype=torch.bool, device=dev)

    def _hp(self):
        c = self.cl
        lam = float(c["lambda"])
        return np.array([self._eta0(), c["power_t"], c["t"], lam, lam, lam, lam, c["eps"]], dtype=np.float32)

    # Atomic bias updates on the GPU go to line-padded copies (one 64-B line per user / item):
    # in the packed arrays the 16 most popular items share one line, and its same-line atomics
    # bounded the whole kernel (ML-20M shape: 372 M ratings/s with biases, 890 M without;
    # profiles/mf_atomic_r2/contention.log).  Copied in and out around each training launch.
    BIAS_PAD = 16

    def _padded_bias(self, names):
        pads = getattr(self, "_bias_pads", None)
        if pads is None:
            pads = self._bias_pads = {}
        out = []
        for nm in names:
            t = self.state[nm]
            b = pads.get(nm)
            if b is None or b.shape[0] != t.shape[0]:
                b = pads[nm] = torch.zeros(t.shape[0], self.BIAS_PAD, dtype=t.dtype, device=t.device)
            b[:, 0].copy_(t)
            out.append(b)
        return out

    def _step(self, u, i, r, train=True, pred=None, loss=None):
        st = self.state
        p = _native.ptr
        ip, hp = self._ip(), self._hp()
        n = u.numel()
        names = ["Bu", "Bi"] + (["GBu", "GBi"] if self.adagrad else [])
        pad = u.is_cuda and train and self.use_bias and int(ip[13]) != 0
        bias = dict(zip(names, self._padded_bias(names))) if pad else {nm: st.get(nm) for nm in names}
        if pad:
            ip[14] = self.BIAS_PAD
        args = [ip.ctypes.data, hp.ctypes.data, p(u), p(i), p(r), C.c_int64(n), C.c_int64(self.t),
                p(st["P"]), p(st["Q"]), p(bias["Bu"]), p(bias["Bi"]), p(st["mu"]), p(st.get("GP")),
                p(st.get("GQ")), p(bias.get("GBu")), p(bias.get("GBi")), int(train), p(pred), p(loss)]
        if u.is_cuda:
            _native.check(_native.hip().hm_mf_step(*args, _native.stream_of(u.device)), "hm_mf_step")
            if pad:
                for nm in names:
                    st[nm].copy_(bias[nm][:, 0])
        else:
            _native.host().hm_mf_step_cpu(*args)
        if train:
            self.t += n

    def fit(self, users, items, ratings) -> "MatrixFactorization":
        dev = self.device
        u, i, r = _dev(users, torch.int32, dev), _dev(items, torch.int32, dev), \
            _dev(ratings, torch.float32, dev)
        if self.state is None:
            # data-parallel replicas share one shape: the max ids over every rank's shard
            self.init_state(*self.agree_max(int(tmax(u)) + 1 if u.numel() else 1,
                                            int(tmax(i)) + 1 if i.numel() else 1))
            if self.cl["update_mean"]:
                mu = self.dp_sum(float(r.double().sum().item())) / max(
                    1.0, self.dp_sum(float(r.numel())))
                self.state["mu"].fill_(mu)
        self.seen_u[u.long()] = True
        self.seen_i[i.long()] = True
        loss = torch.empty(u.numel(), device=dev)
        for ep in self.epochs(int(self.cl["iters"]), data=(u, i, r)):
            self._step(u, i, r, loss=loss)
            self._epoch_mix(ep)
            el = self.dp_sum(float(loss.double().sum().item()))
            self._epoch_end(el)
            if self.epoch_converged(el, reduced=True, rows=u.numel()):
                log.info("%s converged at epoch %d", self.NAME, ep + 1)
                break
        self.mix()
        return self

    def predict(self, users, items) -> np.ndarray:
        dev = self.device
        u = torch.as_tensor(np.asarray(users, dtype=np.int32)).to(dev)
        i = torch.as_tensor(np.asarray(items, dtype=np.int32)).to(dev)
        out = torch.empty(u.numel(), device=dev)
        self._step(u, i, torch.zeros(u.numel(), device=dev), train=False, pred=out)
        return out.cpu().numpy()

    def recommend_topk(self, users=None, k: int = 10, exclude: tuple | None = None):
        """Top-k items by mf_predict (mu + b_u + b_i + p_u.q_i) per user, best first:
        (scores [U,k], items [U,k]).  ``exclude`` = (row positions into ``users``, items).
        Fused MFMA score + top-k on the GPU (``ops/topk_mips.py``); k <= 64.
        (Predictions are not clipped to -min/-max here: clipping would only create ties.)"""
        st = self.state
        dev = st["P"].device
        uu = (torch.arange(self.n_users, device=dev) if users is None
              else torch.as_tensor(users, device=dev).long())
        ex = None
        if exclude is not None:
            ex = topk_mips.exclusion_csr(exclude[0], exclude[1], uu.numel(), device=dev)
        ix, sc = topk_mips.mips_topk(st["P"][uu][:, : self.k], st["Q"][:, : self.k], k,
                                     item_bias=st["Bi"], row_bias=st["Bu"][uu] + st["mu"][0],
                                     exclude=ex)
        return sc, ix

    def model_table(self) -> pd.DataFrame:
        st = self.state
        n = max(self.n_users, self.n_items)
        su = self.seen_u.cpu().numpy()
        si = self.seen_i.cpu().numpy()
        P = st["P"][:, : self.k].cpu().numpy()
        Q = st["Q"][:, : self.k].cpu().numpy()
        Bu = st["Bu"].cpu().numpy()
        Bi = st["Bi"].cpu().numpy()
        mu = float(st["mu"][0].item())
        rows = []
        for idx in range(n):
            iu = idx < self.n_users and su[idx]
            ii = idx < self.n_items and si[idx]
            if not (iu or ii):
                continue
            rows.append((idx, P[idx] if iu else None, Q[idx] if ii else None,
                         float(Bu[idx]) if iu else None, float(Bi[idx]) if ii else None, mu))
        return pd.DataFrame(rows, columns=["idx", "Pu", "Qi", "Bu", "Bi", "mu"])


class MatrixFactorizationAdaGrad(MatrixFactorization):
    NAME = "train_mf_adagrad"
    ADAGRAD = True


class BPRMF(_MFBase):
    """BPR-MF.  Input triples (user, pos_item, neg_item) as produced by ``bpr_sampling``, or
    (``fit_implicit``) the positive pairs only, with negatives sampled on the device."""
    # BPR's sigmoid-bounded pairwise steps tolerate 8x the concurrency: ML-20M-shaped k=64
    # sweep on MI355X (profiles/bpr_grid_r1.log): grid 106 -> 852 blocks = 170M -> 966M
    # triples/s at sampled AUC 0.7103 -> 0.7101 (sequential CPU engine 0.7105).
    ROWS_PER_BLOCK = 32
    ROWS_PER_BLOCK_ATOMIC = None   # BPR updates are plain stores (AUC-neutral at every grid)
    NAME = "train_bprmf"
    OPTIONS = BPR_OPTS

    def __init__(self, options=None, device=None, **kw):
        super().__init__(options, device, **kw)
        c = self.cl
        self.k = self._factors()
        self.kp = self.k
        self.adagrad = False
        self.use_bias = not c["no_bias"]
        loss = str(c["loss"]).lower()
        if loss not in _BPR_LOSS:
            raise UDFArgumentException(f"train_bprmf: unknown -loss {c['loss']}")
        self.loss_id = _BPR_LOSS[loss]
        self.state = None
        self.t = 0
        self.cv = ConversionState(not c["disable_cv"], c["cv_rate"])
        self.grid = int(c["grid"])
        self.sharded = None        # {"P", "Q", "Bi"} ShardedTables with -shard_model

    def _grid(self) -> int:
        """The base rule (1 block per 32 items / users), rounded up to a power of two once it
        reaches the 256 CUs: ML-20M-shaped k = 64 (16-lane float4 kernel, two boxes): 852 blocks
        3.33-3.36 G triples/s, 1,024 3.66-3.67 G, 1,280 / 2,048 / 2,560 3.65-3.68 G, but 1,536 and
        1,704 3.29-3.35 G; sampled AUC 0.7096-0.7101 at every grid up to 3,408
        (profiles/r6/bpr_grid/)."""
        g = super()._grid()
        if int(self.cl["grid"]) > 0 or g < 256:
            return g
        return min(4096, 1 << (g - 1).bit_length())

    def init_state(self, n_users, n_items):
        self.n_users, self.n_items = int(n_users), int(n_items)
        g = torch.Generator().manual_seed(self.seed)
        c = self.cl
        dev = self.device
        if c["shard_model"]:
            from ..parallel.sharded import ShardedTable

            ctx = self.mixer.ctx if self.mixer is not None else None
            # the same initial values as the unsharded model (generated once, each rank keeps its rows)
            P0 = _init_factors(self.n_users, self.k, self.kp, c["init"], c["maxval"], c["min_init_stddev"], g)
            Q0 = _init_factors(self.n_items, self.k, self.kp, c["init"], c["maxval"], c["min_init_stddev"], g)
            self.sharded = dict(
                P=ShardedTable(self.n_users, self.kp, ctx, device=dev, init=lambda gid: P0[gid.cpu()]),
                Q=ShardedTable(self.n_items, self.kp, ctx, device=dev, init=lambda gid: Q0[gid.cpu()]),
                Bi=ShardedTable(self.n_items, 1, ctx, device=dev))
            self.state = None
            self.seen_u = torch.zeros(self.n_users, dtype=torch.bool, device=dev)
            self.seen_i = torch.zeros(self.n_items, dtype=torch.bool, device=dev)
            return
        self.state = dict(
            P=_init_factors(self.n_users, self.k, self.kp, c["init"], c["maxval"], c["min_init_stddev"], g).to(dev),
            Q=_init_factors(self.n_items, self.k, self.kp, c["init"], c["maxval"], c["min_init_stddev"], g).to(dev),
            Bi=torch.zeros(self.n_items, device=dev))
        self.seen_u = torch.zeros(self.n_users, dtype=torch.bool, device=dev)
        self.seen_i = torch.zeros(self.n_items, dtype=torch.bool, device=dev)

    def _hp(self):
        c = self.cl
        reg = float(c["reg"])
        ru = c["reg_u"] if c["reg_u"] is not None else reg
        ri = c["reg_i"] if c["reg_i"] is not None else reg
        rj = c["reg_j"] if c["reg_j"] is not None else reg
        return np.array([self._eta0(), c["power_t"], c["t"], ru, ri, rj, c["reg_bias"], 1.0], dtype=np.float32)

    def step(self, tu=None, ti=None, tj=None, n=None, csr=None) -> float:
        """One launch over explicit triples, or ``n`` device-sampled triples from ``csr``."""
        st = self.state
        p = _native.ptr
        ip, hp = self._ip(loss=self.loss_id), self._hp()
        dev = st["P"].device
        loss = torch.zeros(1, dtype=torch.float64, device=dev)
        if tu is not None:
            n = tu.numel()
            uptr = uit = pu = None
            npos = 0
        else:
            uptr, uit, pu = csr
            npos = uit.numel()
        args = [ip.ctypes.data, hp.ctypes.data, p(tu), p(ti), p(tj), C.c_int64(n), p(uptr), p(uit),
                p(pu), C.c_int64(npos), C.c_int64(self.t), p(st["P"]), p(st["Q"]), p(st["Bi"]), p(loss)]
        if dev.type == "cuda":
            bm = self._positive_bitmap(csr) if tu is None else None
            _native.check(_native.hip().hm_bpr_step(*args, p(bm), _native.stream_of(dev)), "hm_bpr_step")
        else:
            _native.host().hm_bpr_step_cpu(*args)
        self.t += n
        return float(loss.item())

    # the per-user positive-item bitmap of device sampling: one load per negative test instead
    # of a binary search (csrc/kernels/mf.hip bpr_pf_kernel); skipped above this many bytes
    BITMAP_MAX_BYTES = 8 << 30

    def _positive_bitmap(self, csr) -> torch.Tensor | None:
        """n_users x ceil(n_items / 32) int32 bitmap of ``csr``'s positives, built once per
        positive set (cached on the CSR tensors' identity)."""
        uptr, uit, pu = csr
        hit = getattr(self, "_bitmap", None)
        if hit is not None and hit[0]() is uit and hit[1] == uit._version:
            return hit[2]
        words = (self.n_items + 31) // 32
        if self.n_users * words * 4 > self.BITMAP_MAX_BYTES:
            return None
        import weakref

        bm = torch.zeros(self.n_users * words, dtype=torch.int32, device=uit.device)
        _native.check(_native.hip().hm_bpr_bitmap(pu.data_ptr(), uit.data_ptr(), C.c_int64(uit.numel()),
                                                  self.n_items, bm.data_ptr(), _native.stream_of(uit.device)),
                      "hm_bpr_bitmap")
        self._bitmap = (weakref.ref(uit), uit._version, bm)
        return bm

    def _step_sharded(self, tu, ti, tj) -> float:
        """-shard_model: pull the rows the triples touch from their owner ranks, run the same
        kernel on the compact tables, push the changes back (parallel/sharded.py)."""
        sh = self.sharded
        B = max(1, int(self.cl["shard_batch"]))
        n = tu.numel()
        steps = sh["P"].steps_agreed((n + B - 1) // B)
        total = 0.0
        full_u, full_i = self.n_users, self.n_items
        try:
            for s in range(steps):
                cu, ci, cj = tu[s * B:(s + 1) * B], ti[s * B:(s + 1) * B], tj[s * B:(s + 1) * B]
                U = torch.unique(cu.long())
                I = torch.unique(torch.cat([ci, cj]).long())
                P0, Q0, B0 = sh["P"].pull(U), sh["Q"].pull(I), sh["Bi"].pull(I)
                self.state = dict(P=P0.clone(), Q=Q0.clone(), Bi=B0[:, 0].clone().contiguous())
                if cu.numel():
                    self.n_users, self.n_items = max(1, U.numel()), max(1, I.numel())
                    lu = torch.searchsorted(U, cu.long()).to(torch.int32)
                    li = torch.searchsorted(I, ci.long()).to(torch.int32)
                    lj = torch.searchsorted(I, cj.long()).to(torch.int32)
                    total += self.step(lu.contiguous(), li.contiguous(), lj.contiguous())
                    self.n_users, self.n_items = full_u, full_i
                sh["P"].push_add(U, self.state["P"] - P0)
                sh["Q"].push_add(I, self.state["Q"] - Q0)
                sh["Bi"].push_add(I, (self.state["Bi"] - B0[:, 0])[:, None])
        finally:
            self.n_users, self.n_items = full_u, full_i
            self.state = None
        return total

    def full_state(self) -> dict:
        """The model tables (all-gathered on every rank with -shard_model)."""
        if self.sharded is None:
            return self.state
        return dict(P=self.sharded["P"].full(), Q=self.sharded["Q"].full(),
                    Bi=self.sharded["Bi"].full()[:, 0].contiguous())

    def fit(self, users, pos_items, neg_items) -> "BPRMF":
        dev = self.device
        tu = torch.as_tensor(np.asarray(users, dtype=np.int32)).to(dev)
        ti = torch.as_tensor(np.asarray(pos_items, dtype=np.int32)).to(dev)
        tj = torch.as_tensor(np.asarray(neg_items, dtype=np.int32)).to(dev)
        if self.state is None and self.sharded is None:
            nu = int(tmax(tu)) + 1 if tu.numel() else 1
            ni = int(max(tmax(ti), tmax(tj))) + 1 if ti.numel() else 1
            if self._dp():        # every rank sizes the (sharded or mixed) tables alike
                nu = int(self.mixer.all_reduce_scalar(float(nu), "max"))
                ni = int(self.mixer.all_reduce_scalar(float(ni), "max"))
            self.init_state(nu, ni)
        if self.sharded is not None:
            self.seen_u[tu.long()] = True
            self.seen_i[ti.long()] = True
            self.seen_i[tj.long()] = True
            self.no_checkpoint("-shard_model")
            for ep in range(int(self.cl["iters"])):
                el = self.dp_sum(self._step_sharded(tu, ti, tj))
                self._epoch_end(el)
                if self.epoch_converged(el, reduced=True, rows=tu.numel()):
                    break
            if self._dp():
                f = [self.seen_u.to(torch.float32), self.seen_i.to(torch.float32)]
                self.mixer.all_reduce_sum(f)
                self.seen_u, self.seen_i = f[0] > 0, f[1] > 0
            self.state = self.full_state()
            return self
        self.seen_u[tu.long()] = True
        self.seen_i[ti.long()] = True
        self.seen_i[tj.long()] = True
        for ep in self.epochs(int(self.cl["iters"]), data=(tu, ti, tj)):
            el = self.dp_sum(self.step(tu, ti, tj))
            self._epoch_end(el)
            self._epoch_mix(ep)
            if self.epoch_converged(el, reduced=True, rows=tu.numel()):
                break
        self.mix()
        return self

    @staticmethod
    def build_csr(users: torch.Tensor, items: torch.Tensor, n_users: int):
        """Positive pairs -> (user ptr int64, items sorted per user int32, user of each pair)."""
        key = users.long() * (1 << 32) + items.long()
        key = torch.unique(key)
        u = (key >> 32).to(torch.int32)
        it = (key & 0xFFFFFFFF).to(torch.int32)
        counts = torch.bincount(u.long(), minlength=n_users)
        ptr = torch.zeros(n_users + 1, dtype=torch.int64, device=users.device)
        ptr[1:] = torch.cumsum(counts, 0)
        return ptr.contiguous(), it.contiguous(), u.contiguous()

    def fit_implicit(self, users, items, n_users=None, n_items=None, epochs=None) -> "BPRMF":
        """Train from positive (user, item) pairs; negatives are sampled on the device."""
        if self.cl["shard_model"]:
            raise UDFArgumentException("train_bprmf: -shard_model trains on explicit (user, pos, neg) "
                                       "triples (bpr_sampling); device negative sampling needs the "
                                       "whole item table on every GPU")
        dev = self.device
        u = torch.as_tensor(np.asarray(users, dtype=np.int32)).to(dev) if not torch.is_tensor(users) else users.to(dev)
        i = torch.as_tensor(np.asarray(items, dtype=np.int32)).to(dev) if not torch.is_tensor(items) else items.to(dev)
        if self.state is None:
            self.init_state(*self.agree_max(n_users or int(tmax(u)) + 1, n_items or int(tmax(i)) + 1))
        csr = self.build_csr(u, i, self.n_users)
        self.seen_u[u.long()] = True
        self.seen_i.fill_(True)
        per = int(self.cl["samples_per_epoch"]) or csr[1].numel()
        for ep in self.epochs(int(epochs or self.cl["iters"]), data=(u, i)):
            el = self.dp_sum(self.step(n=per, csr=csr))
            self._epoch_end(el)
            self._epoch_mix(ep)
            if self.epoch_converged(el, reduced=True, rows=per):
                break
        self.mix()
        return self

    def scores(self, users=None) -> torch.Tensor:
        st = self.state
        U = st["P"] if users is None else st["P"][torch.as_tensor(users, device=st["P"].device).long()]
        dt = torch.bfloat16 if U.is_cuda else torch.float32
        return (U.to(dt) @ st["Q"].to(dt).T).float() + st["Bi"][None, :]

    def recommend_topk(self, users=None, k: int = 10, exclude: tuple | None = None):
        """Top-k items per user, best first: (scores [U,k], items [U,k]).

        ``exclude`` = (row positions into ``users``, items) pairs to skip (already-seen items).
        On the GPU this is the fused MFMA score + top-k kernel (``ops/topk_mips.py``): the
        user x item score matrix is never materialised.  k > 64 falls back to GEMM + topk."""
        st = self.state
        U = st["P"] if users is None else st["P"][torch.as_tensor(users, device=st["P"].device).long()]
        if k <= topk_mips.KMAX:
            ex = None
            if exclude is not None:
                ex = topk_mips.exclusion_csr(exclude[0], exclude[1], U.shape[0], device=U.device)
            ix, sc = topk_mips.mips_topk(U[:, : self.k], st["Q"][:, : self.k], k,
                                         item_bias=st["Bi"], exclude=ex)
            return sc, ix
        S = self.scores(users)
        if exclude is not None:
            eu, ei = exclude
            S[torch.as_tensor(eu, device=S.device).long(), torch.as_tensor(ei, device=S.device).long()] = -float("inf")
        return torch.topk(S, k, dim=1)

    def model_table(self) -> pd.DataFrame:
        st = self.state
        su, si = self.seen_u.cpu().numpy(), self.seen_i.cpu().numpy()
        P = st["P"][:, : self.k].cpu().numpy()
        Q = st["Q"][:, : self.k].cpu().numpy()
        Bi = st["Bi"].cpu().numpy()
        rows = []
        for idx in range(max(self.n_users, self.n_items)):
            iu = idx < self.n_users and su[idx]
            ii = idx < self.n_items and si[idx]
            if iu or ii:
                rows.append((idx, P[idx] if iu else None, Q[idx] if ii else None,
                             float(Bi[idx]) if ii else None))
        return pd.DataFrame(rows, columns=["idx", "Pu", "Qi", "Bi"])


def auc_implicit(model: BPRMF, test_users, test_items, train_csr=None, n_neg: int = 100, seed: int = 0) -> float:
    """Sampled AUC: P(score(u, i_test) > score(u, j)) over random negatives j."""
    dev = model.state["P"].device
    g = torch.Generator(device="cpu").manual_seed(seed)
    u = torch.as_tensor(np.asarray(test_users), dtype=torch.long)
    i = torch.as_tensor(np.asarray(test_items), dtype=torch.long)
    j = torch.randint(0, model.n_items, (u.numel(), n_neg), generator=g)
    P, Q, B = model.state["P"], model.state["Q"], model.state["Bi"]
    u, i, j = u.to(dev), i.to(dev), j.to(dev)
    si = (P[u] * Q[i]).sum(1) + B[i]
    sj = (P[u][:, None, :] * Q[j]).sum(2) + B[j]
    return float((si[:, None] > sj).float().mean().item())


@udf("mf_predict")
def mf_predict(Pu, Qi, Bu=None, Bi=None, mu=None):
    """μ + b_u + b_i + p_u·q_i (NULL factors -> 0)."""
    s = 0.0
    if Pu is not None and Qi is not None:
        s = float(np.dot(np.asarray(Pu, dtype=np.float64), np.asarray(Qi, dtype=np.float64)))
    for b in (Bu, Bi, mu):
        if b is not None and not (isinstance(b, float) and np.isnan(b)):
            s += float(b)
    return s


@udf("bprmf_predict")
def bprmf_predict(Pu, Qi, Bi=None):
    s = 0.0
    if Pu is not None and Qi is not None:
        s = float(np.dot(np.asarray(Pu, dtype=np.float64), np.asarray(Qi, dtype=np.float64)))
    if Bi is not None and not (isinstance(Bi, float) and np.isnan(Bi)):
        s += float(Bi)
    return s


def register_sql(reg):
    reg("train_mf_sgd", lambda: MatrixFactorization, n_data_args=3)
    reg("train_mf_adagrad", lambda: MatrixFactorizationAdaGrad, n_data_args=3)
    reg("train_bprmf", lambda: BPRMF, n_data_args=3)


_P = _native.c_p
_native.register_hip("hm_mf_step", [_P, _P, _P, _P, _P, _native.c_i64, _native.c_i64] + [_P] * 9 +
                     [C.c_int, _P, _P, _P])
_native.register_host("hm_mf_step_cpu", [_P, _P, _P, _P, _P, _native.c_i64, _native.c_i64] + [_P] * 9 +
                      [C.c_int, _P, _P])
_native.register_hip("hm_bpr_step", [_P, _P, _P, _P, _P, _native.c_i64, _P, _P, _P, _native.c_i64,
                                     _native.c_i64, _P, _P, _P, _P, _P, _P])
_native.register_hip("hm_bpr_bitmap", [_P, _P, _native.c_i64, C.c_int, _P, _P])
_native.register_host("hm_bpr_step_cpu", [_P, _P, _P, _P, _P, _native.c_i64, _P, _P, _P, _native.c_i64,
                                          _native.c_i64, _P, _P, _P, _P])
