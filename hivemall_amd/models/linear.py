"""Online linear learners: binary classifiers, regressors, the general (loss x optimizer)
learners and the multiclass family.

Reference behaviour (upstream
core/src/main/java/hivemall/{LearnerBaseUDTF,GeneralLearnerBaseUDTF}.java,
hivemall/classifier/*.java, hivemall/classifier/multiclass/*.java, hivemall/regression/*.java,
hivemall/optimizer/*.java).  Every SQL function is a subclass that only declares its option
spec and algorithm id; the update rules are in ``csrc/kernels/linear_rules.h``.

Execution model ("mapper-in-a-wave", see csrc/kernels/linear.hip): ``R`` replicas, each one
a sequential Hivemall learner over its shard of the rows; after every epoch the replicas are
mixed (average over the replicas that saw the feature, or argmin-KLD for the covariance
learners) and, when running distributed, the compact sums are all-reduced over RCCL.  With
``R = 1`` (the CPU default) this is exactly upstream's single-mapper semantics.

Model tables (docs/compat.md):
  binary / regression : (feature, weight)            [+ covar for CW/AROW/SCW families]
  multiclass          : (label, feature, weight)     [+ covar]
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from statistics import NormalDist

import numpy as np
import pandas as pd
import torch

from ..ops import linear as LO
from ..utils.features import CSR, FeatureEncoder
from ..utils.options import UDFArgumentException, flag, opt
from .base import CKPT_OPTS, ConversionState, Learner, log
from ..utils.reduce import tmax, tmin

# ------------------------------------------------------------------ option specs
_MIX_INERT = ("mixing is a collective between the job's ranks over RCCL (-mix_interval), "
              "there is no MixServer")
_SCALE_INERT = "AdaGrad accumulators are fp32 (no half-float scaling)"
LEARNER_BASE_OPTS = [
    flag("dense", "densemodel", "Use a dense model",
         inert="models are always dense tables on the device"),
    opt("dims", "feature_dimensions", -1, int, "Dimension of the model (default: max index + 1)"),
    flag("disable_halffloat", None, "Disable half-float weights",
         inert="linear models are fp32"),
    opt("mini_batch", "mini_batch_size", 1, int, "Mini-batch size (general learners)"),
    opt("mix", "mix_servers", None, str, "MixServer addresses", inert=_MIX_INERT),
    opt("mix_session", "mix_session_name", None, str, "MixServer session", inert=_MIX_INERT),
    opt("mix_threshold", None, 3, int, "MixServer update threshold", inert=_MIX_INERT),
    flag("mix_cancel", "enable_mix_canceling", "MixServer cancel", inert=_MIX_INERT),
    flag("ssl", None, "MixServer SSL", inert=_MIX_INERT),
    opt("loadmodel", None, None, str, "Warm start: path of a model table (TSV/CSV/parquet)"),
    opt("iters", "iterations", 1, int, "The maximum number of iterations (epochs)", aliases=("iter",)),
    opt("cv_rate", "convergence_rate", 0.005, float, "Threshold to determine convergence"),
    flag("disable_cv", "disable_cvtest", "Whether to disable convergence check"),
    opt("seed", None, -1, int, "Seed value"),
    opt("replicas", None, 0, int, "[engine] model replicas (0 = auto; CPU default 1)"),
    opt("engine", None, "auto", str,
        "[engine] GPU execution: replica (private model per wave, mixed), shared (one Hogwild "
        "table for the whole chip, large -dims), minibatch (general learner with -mini_batch > 1: "
        "the whole chip on each batch, exact mini-batch rule), seq (one table, -shared_waves "
        "consecutive rows in flight on one XCD, software-pipelined: the near-sequential engine), "
        "auto (minibatch for -mini_batch > 1, else shared when the replicas would exceed 2 GiB)"),
    opt("seq_spread", None, 8, int,
        "[engine] seq engine: 8 = every wave on one XCD (one coherent L2), 1 = waves dealt over "
        "all 8 XCDs"),
    opt("shared_replicas", None, 1, int,
        "[engine] shared engine: model tables (1, or a multiple of 8: one set per XCD), averaged "
        "after every pass"),
    opt("shared_waves", None, 0, int,
        "[engine] shared / seq engine: rows in flight (0 = auto per rule: ops/linear.py "
        "rule_waves for the shared engine — 1024 AdaGrad / AdaGrad-RDA, 512 AdaGrad-L1 / elastic "
        "net; seq_waves for the seq engine, which auto picks for the other general-learner "
        "rules — 512 SGD / momentum / RMSprop / AdaDelta, 256 Adam / NAdam / AdamHD, 128 Eve)"),
] + CKPT_OPTS

GENERAL_OPTS = [
    opt("loss", "loss_function", None, str, "Loss function"),
    opt("opt", "optimizer", "adagrad", str, "Optimizer"),
    opt("reg", "regularization", "rda", str, "Regularization: no, l1, l2, elasticnet, rda"),
    opt("eta", None, "inverse", str, "Learning rate scheme: fixed, simple, inverse/inv"),
    opt("eta0", None, 0.1, float, "Initial learning rate"),
    opt("t", "total_steps", -1.0, float, "Total of n_samples * epochs (for -eta simple)"),
    opt("power_t", None, 0.1, float, "Exponent for inverse scaling learning rate"),
    opt("lambda", None, 1e-4, float, "Regularization term"),
    opt("l1_ratio", None, 0.5, float, "Elastic-net mixing"),
    opt("alpha", None, 1.0, float, "Coefficient of learning rate (momentum/Adam family)"),
    opt("beta1", "momentum", 0.9, float, "Adam beta1 / momentum"),
    opt("beta2", None, 0.999, float, "Adam beta2"),
    opt("eps", None, 1e-6, float, "Denominator constant"),
    opt("decay", None, 0.95, float, "RMSprop decay"),
    opt("rho", None, 0.95, float, "AdaDelta decay"),
    opt("beta", None, 1e-6, float, "AdamHD hyper-gradient step"),
    opt("scale", None, 100.0, float, "Scaling factor", inert=_SCALE_INERT),
    flag("amsgrad", None, "AMSGrad variant of Adam"),
    flag("inspect_opts", None, "Show the resolved options and raise"),
    opt("quantile_tau", "tau", 0.5, float, "Quantile loss tau"),
    opt("huber_c", None, 1.0, float, "Huber loss threshold"),
    opt("epsilon", None, 0.1, float, "Epsilon of the epsilon-insensitive losses"),
]


@dataclass
class SparseRows:
    """Device-resident CSR rows (+ labels)."""
    indptr: torch.Tensor      # int64 [n+1]
    idx: torch.Tensor         # int32 [nnz]
    val: torch.Tensor | None  # f32 [nnz] (None = all ones)
    y: torch.Tensor | None    # f32 [n]

    @property
    def n(self) -> int:
        return self.indptr.numel() - 1

    def to(self, device) -> "SparseRows":
        f = lambda t: None if t is None else t.to(device).contiguous()
        return SparseRows(f(self.indptr), f(self.idx), f(self.val), f(self.y))

    @staticmethod
    def from_csr(csr: CSR, y=None, device="cpu") -> "SparseRows":
        v = np.asarray(csr.val, dtype=np.float32)
        val = None if csr.nnz and v.min() == 1.0 == v.max() else torch.from_numpy(v.copy())
        idx = np.asarray(csr.idx)
        if idx.size and (idx.min() < 0 or idx.max() >= 2 ** 31 - 1):
            idx = np.where((idx >= 0) & (idx < 2 ** 31 - 1), idx, -1)
        idx = idx.astype(np.int32)
        yy = None if y is None else torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32))
        return SparseRows(torch.from_numpy(csr.indptr.astype(np.int64)), torch.from_numpy(idx),
                          val, yy).to(device)


def encode_rows(rows, encoder: FeatureEncoder | None, train: bool) -> tuple[CSR, FeatureEncoder]:
    """Hivemall feature rows -> CSR.  Integer names are used as indices; otherwise names are
    dictionary-encoded (collision free, decoded again for the model table)."""
    if isinstance(rows, CSR):
        return rows, encoder or FeatureEncoder("int")
    if encoder is None:
        enc = FeatureEncoder("int")
        # string features that are integer literals keep the string type in the model table
        if _arrow(rows):
            enc.string_names = True
        else:
            first = next((r[0] for r in rows if r is not None and len(r)), None)
            enc.string_names = isinstance(first, str)
        try:
            return enc.encode(rows), enc
        except UDFArgumentException:
            enc = FeatureEncoder("dict")
            return enc.encode(rows, add_new=True), enc
    return encoder.encode(rows, add_new=train and encoder.mode == "dict"), encoder


def _arrow(x) -> bool:
    from ..io.ingest import is_arrow_like

    return is_arrow_like(x)


def _arrow_string_lists(x) -> bool:
    """An Arrow list<string> column (parsed from its buffers by FeatureEncoder.encode)."""
    from ..io.ingest import to_arrow_lists

    try:
        to_arrow_lists(x)
        return True
    except (TypeError, ValueError):
        return False


class OnlineLinearLearner(Learner):
    SQL_DP = "shard"
    ARROW_INPUT = True      # Arrow list<string> rows with integer names are parsed on the device
    DEVICE_FEATURES = True  # accepts io.ingest.DeviceFeatures (SQL feature_hashing on the GPU)
    NAME = "train_linear"
    ALGO = "general"
    TASK = "binary"           # binary | regression | multiclass
    OPTIONS = LEARNER_BASE_OPTS
    DEFAULT_LOSS = "hinge"

    def __init__(self, options: str | None = None, device=None, **kw):
        super().__init__(options, device, **kw)
        self.covar = self.ALGO in LO.COVAR_ALGOS
        self.P = self.make_params()
        self.encoder: FeatureEncoder | None = None
        self.state: LO.LinearState | None = None
        self.labels: list | None = None
        self.cv = ConversionState(not self.cl["disable_cv"], self.cl["cv_rate"])
        self._w = self._cov = None
        self.rows_seen = 0
        self._warm = None
        if self.cl["loadmodel"]:
            from ..io.model_table import read_table
            self._warm = read_table(self.cl["loadmodel"])
        if self.cl.has("inspect_opts") and self.cl["inspect_opts"]:
            raise UDFArgumentException(f"{self.NAME} options: {self.cl.as_dict()}")

    # ------------------------------------------------------------------ params
    def _opt(self, name, default=None):
        try:
            return self.cl[name]
        except KeyError:
            return default

    def make_params(self) -> LO.LinParams:
        P = LO.LinParams()
        P.algo = LO.ALGOS[self.ALGO]
        P.n_labels = 1
        P.eta0 = self._opt("eta0", 0.1) if self._opt("eta0") is not None else 0.1
        P.power_t = self._opt("power_t", 0.1) or 0.1
        P.total_steps = self._opt("t", -1.0) or -1.0
        P.lambda_ = self._opt("lambda", 1e-4) if self._opt("lambda") is not None else 1e-4
        P.l1_ratio = self._opt("l1_ratio", 0.5) or 0.5
        P.c = self._opt("c", 1.0) if self._opt("c") is not None else 1.0
        P.r = self._opt("r", 0.1) if self._opt("r") is not None else 0.1
        phi = self._opt("phi", None)
        eta_conf = self._opt("eta", None) if self.ALGO in ("cw", "scw", "scw2") else None
        if phi is None and eta_conf is not None:
            phi = NormalDist().inv_cdf(float(eta_conf))
        P.phi = 1.0 if phi is None else float(phi)
        P.epsilon = self._opt("epsilon", 0.1) if self._opt("epsilon") is not None else 0.1
        P.alpha = self._opt("alpha", 1.0) if self._opt("alpha") is not None else 1.0
        P.beta1 = self._opt("beta1", 0.9) or 0.9
        P.beta2 = self._opt("beta2", 0.999) or 0.999
        P.eps = self._opt("eps", 1e-6) if self._opt("eps") is not None else 1e-6
        P.rho = self._opt("rho", 0.95) or 0.95
        P.decay = self._opt("decay", 0.95) or 0.95
        P.beta_hd = self._opt("beta", 1e-6) or 1e-6
        P.scale = self._opt("scale", 100.0) or 100.0
        P.quantile_tau = self._opt("quantile_tau", 0.5) or 0.5
        P.huber_c = self._opt("huber_c", 1.0) or 1.0
        P.init_covar = 1.0
        P.eta = LO.ETAS["inverse"]
        if self.ALGO == "general":
            loss = (self._opt("loss") or self.DEFAULT_LOSS).lower().replace("-", "_")
            if loss not in LO.LOSSES:
                raise UDFArgumentException(f"{self.NAME}: unsupported loss function: {loss}")
            P.loss = LO.LOSSES[loss]
            is_cls = P.loss in LO.CLASSIFICATION_LOSSES
            if (self.TASK == "binary") != is_cls:
                raise UDFArgumentException(
                    f"{self.NAME}: loss '{loss}' is not a "
                    f"{'classification' if self.TASK == 'binary' else 'regression'} loss")
            o = self._opt("opt").lower()
            if o not in LO.OPTIMIZERS:
                raise UDFArgumentException(f"{self.NAME}: unsupported optimizer: {o}")
            P.opt = LO.OPTIMIZERS[o]
            r = self._opt("reg").lower()
            if r not in LO.REGS:
                raise UDFArgumentException(f"{self.NAME}: unsupported regularization: {r}")
            P.reg = LO.REGS[r]
            e = self._opt("eta").lower()
            if e not in LO.ETAS:
                raise UDFArgumentException(f"{self.NAME}: unsupported eta scheme: {e}")
            P.eta = LO.ETAS[e]
            P.amsgrad = int(bool(self._opt("amsgrad")))
        elif self.ALGO == "logress":
            P.eta = LO.ETAS["inverse"] if self._opt("eta") is None else LO.ETAS["fixed"]
            if self._opt("eta") is not None:
                P.eta0 = float(self._opt("eta"))
        elif self.ALGO in ("adagrad_rda", "adagrad_regr"):
            if self._opt("eta") is not None:
                P.eta0 = float(self._opt("eta"))
            if self.ALGO == "adagrad_regr" and self._opt("eps") is None:
                P.eps = 1.0
        return P

    # ------------------------------------------------------------------ data
    def _labels_to_float(self, labels) -> np.ndarray:
        a = np.asarray(labels)
        if self.TASK == "binary":
            return np.where(a.astype(np.float64) > 0, 1.0, -1.0).astype(np.float32)
        if self.TASK == "multiclass":
            if self.labels is None:
                uniq = sorted(set(a.tolist()), key=lambda v: (isinstance(v, str), v))
                self.labels = uniq
            lut = {v: i for i, v in enumerate(self.labels)}
            out = np.array([lut.get(v, -1) for v in a.tolist()], dtype=np.float32)
            return out
        return a.astype(np.float32)

    def _prepare_device(self, features, y) -> SparseRows | None:
        """Integer-named string features ("123:0.5") parsed on the GPU (io/ingest.py
        hm_feat_parse) — None when the rows are not strings or hold non-integer names (the
        host encoder then dictionary-encodes them)."""
        from ..io import ingest
        from .fm import _string_rows

        if not _string_rows(features):
            return None
        try:
            ip, idx, val, _ = ingest.csr_device(features, "int", device=self.device)
        except UDFArgumentException:
            return None
        if idx.numel() and (int(tmin(idx)) < 0 or int(tmax(idx)) >= 2 ** 31 - 1):
            return None
        self.encoder = FeatureEncoder("int")
        self.encoder.string_names = True
        yt = None if y is None else torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32)).to(self.device)
        vv = None if (val.numel() and bool((val == 1.0).all().item())) else val
        return SparseRows(ip, idx.to(torch.int32), vv, yt)

    def prepare(self, features, labels=None, train: bool = True) -> SparseRows:
        from ..io.ingest import DeviceFeatures

        if isinstance(features, DeviceFeatures):
            # hashed on the device by the SQL planner (sql/device_ftvec.py): integer ids, as the
            # int encoder reads the "h:value" strings of the host feature_hashing
            self.encoder = FeatureEncoder("int")
            self.encoder.string_names = True
            y = None if labels is None else self._labels_to_float(labels)
            yt = None if y is None else torch.from_numpy(np.ascontiguousarray(y, dtype=np.float32)).to(self.device)
            val = features.val
            vv = None if (val.numel() and bool((val == 1.0).all().item())) else val
            return SparseRows(features.indptr.to(self.device), features.idx.to(self.device, torch.int32),
                              None if vv is None else vv.to(self.device), yt)
        if (self.device.type == "cuda" and self._warm is None and not isinstance(features, CSR)
                and (self.encoder is None or (self.encoder.mode == "int" and
                                              getattr(self.encoder, "string_names", False)))):
            y = None if labels is None else self._labels_to_float(labels)
            rows = self._prepare_device(features, y)
            if rows is not None:
                return rows
        if not isinstance(features, (list, CSR)) and _arrow(features) and not _arrow_string_lists(features):
            features = features.to_pylist() if hasattr(features, "to_pylist") else features.tolist()
        if self.encoder is None and self._warm is not None and not isinstance(features, CSR):
            feats = self._warm["feature"].tolist()
            if any(isinstance(f, str) and not f.lstrip("-").isdigit() for f in feats):
                self.encoder = FeatureEncoder("dict")
                self.encoder.encode([[str(f) for f in feats]], add_new=True)
        csr, self.encoder = encode_rows(features, self.encoder, train)
        y = None if labels is None else self._labels_to_float(labels)
        return SparseRows.from_csr(csr, y, self.device)

    # ------------------------------------------------------------------ state
    def _auto_replicas(self, n_rows: int) -> int:
        r = int(self.cl["replicas"])
        if r > 0:
            return r
        if self.device.type != "cuda":
            return 1
        return int(max(1, min(1024, n_rows // 4096)))

    def _ensure_state(self, rows: SparseRows) -> None:
        if self.state is not None:
            return
        dims = int(self.cl["dims"])
        if dims <= 0:
            dims = int(tmax(rows.idx)) + 1 if rows.idx.numel() else 1
            if self.encoder is not None and self.encoder.mode == "dict":
                if self._dp():
                    raise UDFArgumentException(
                        f"{self.NAME}: data-parallel training needs integer feature indices or "
                        "-feature_hashing (a per-rank string dictionary gives every rank its own ids)")
                dims = max(dims, self.encoder.vocab_size())
            elif self._warm is not None:
                dims = max(dims, int(np.max(np.asarray(self._warm["feature"], dtype=np.int64))) + 1)
            if self._dp():   # every rank's replica must have the same shape
                dims = int(self.mixer.all_reduce_scalar(float(dims), "max"))
        L = len(self.labels) if self.TASK == "multiclass" else 1
        if self.TASK == "multiclass" and L < 2:
            raise UDFArgumentException(f"{self.NAME}: needs at least two distinct labels")
        self.P.n_labels = L
        R = self._auto_replicas(rows.n)
        mb = int(self.cl["mini_batch"]) if self.ALGO == "general" else 1
        if self._use_minibatch(L, mb):
            nnz = int((rows.indptr[1:] - rows.indptr[:-1]).max().item()) if rows.n else 1
            self.state = LO.new_minibatch_state(dims, self.device, mb, nnz)
            if self._warm is not None:
                self.load_model_table(self._warm)
            return
        if self._use_seq(L, mb):
            W = int(self.cl["shared_waves"]) or LO.seq_waves(self.P)
            if int(self.cl["seq_spread"]) not in (1, 8):
                raise UDFArgumentException(f"{self.NAME}: -seq_spread must be 1 or 8")
            self.state = LO.new_seq_state(dims, self.device, max(1, min(W, max(1, rows.n))),
                                          int(self.cl["seq_spread"]))
            if self._warm is not None:
                self.load_model_table(self._warm)
            return
        if self._use_shared(R, L, dims, mb):
            try:
                W = LO.shared_waves(rows.n, int(self.cl["shared_waves"]) or LO.rule_waves(self.P))
                if W <= 16 and rows.n > 64 * W:
                    log.warning("%s: the shared-table engine runs this rule with %d rows in flight "
                                "(~%d M rows/s on one MI355X); -engine seq keeps the rows in flight "
                                "on one XCD at 128-512 rows (ops/linear.py seq_waves)",
                                self.NAME, W, max(1, W // 4))
                # at a few rows in flight the read-modify-write window is no hazard: skip the
                # state re-read before the update (+5 % at 8 rows, same parity:
                # profiles/r4/linear_reload_ab_8rows.jsonl)
                self.state = LO.new_shared_state(
                    dims, self.device, rows.n, replicas=int(self.cl["shared_replicas"]), waves=W,
                    reload=W > 16)
            except ValueError as e:
                raise UDFArgumentException(f"{self.NAME}: {e}") from None
            if self._warm is not None:
                self.load_model_table(self._warm)
            return
        bytes_ = R * L * dims * 16
        if bytes_ > (32 << 30):
            R = max(1, (32 << 30) // (L * dims * 16))
        self.state = LO.new_state(R, L, dims, self.device, self.covar, self.P.init_covar, mb)
        if self._warm is not None:
            self.load_model_table(self._warm)

    def _use_minibatch(self, L: int, mb: int) -> bool:
        """Mini-batch engine (``-mini_batch M > 1`` of the general learner on a GPU, one table,
        the whole chip on each batch; ops/linear.py train_pass_minibatch): the default for
        -mini_batch > 1 unless -engine replica / -replicas ask for per-wave replicas."""
        eng = str(self.cl["engine"]).lower()
        if eng == "minibatch":
            if not (self.device.type == "cuda" and mb > 1 and L == 1 and LO.minibatch_rule(self.P)):
                raise UDFArgumentException(f"{self.NAME}: -engine minibatch needs a GPU, -mini_batch > 1, "
                                           "a binary/regression general learner and -opt other than eve")
            return True
        return (eng == "auto" and int(self.cl["replicas"]) <= 0 and self.device.type == "cuda"
                and mb > 1 and L == 1 and LO.minibatch_rule(self.P))

    def _use_seq(self, L: int, mb: int) -> bool:
        """Near-sequential engine (ops/linear.py train_pass_seq): ``-engine seq``, or auto for the
        general-learner rules whose parity needs few rows in flight (ops/linear.py seq_rule)."""
        eng = str(self.cl["engine"]).lower()
        ok = self.device.type == "cuda" and not self.covar and L == 1 and mb == 1
        if eng == "seq":
            if not ok:
                raise UDFArgumentException(f"{self.NAME}: -engine seq needs a GPU, a rule without "
                                           "covariance, a binary/regression task and -mini_batch 1")
            return True
        return (eng == "auto" and ok and int(self.cl["replicas"]) <= 0
                and int(self.cl["shared_replicas"]) == 1 and LO.seq_rule(self.P))

    def _use_shared(self, R: int, L: int, dims: int, mb: int) -> bool:
        """Shared-table Hogwild engine: device only, binary/regression rules
        without covariance, per-row updates.  auto picks it when R private replicas of
        ``dims x 16 B`` would exceed 2 GiB (e.g. Hivemall's default 2^24 hashed dims)."""
        eng = str(self.cl["engine"]).lower()
        if eng not in ("auto", "replica", "shared", "minibatch", "seq"):
            raise UDFArgumentException(f"{self.NAME}: -engine must be auto, replica, shared, seq or minibatch")
        ok = (self.device.type == "cuda" and not self.covar and L == 1 and mb == 1)
        if eng == "shared" and not ok:
            raise UDFArgumentException(f"{self.NAME}: -engine shared needs a GPU, a rule without "
                                       "covariance, a binary/regression task and -mini_batch 1")
        if eng == "replica" or not ok or int(self.cl["replicas"]) > 0:
            return eng == "shared"
        return eng == "shared" or R * dims * 16 > (2 << 30)

    # ------------------------------------------------------------------ training
    def fit(self, features=None, labels=None, rows: SparseRows | None = None) -> "OnlineLinearLearner":
        rows = rows if rows is not None else self.prepare(features, labels, train=True)
        if rows.y is None:
            raise UDFArgumentException(f"{self.NAME}: labels are required")
        self._ensure_state(rows)
        if rows.idx.numel() and int(tmax(rows.idx)) >= self.state.dims:
            log.warning("%s: feature index >= dims (%d) ignored", self.NAME, self.state.dims)
        mb = int(self.cl["mini_batch"]) if self.ALGO == "general" else 1
        iters = int(self.cl["iters"])
        shared = self.state.meta.get("shared", False)
        minibatch = self.state.meta.get("minibatch", False)
        seq = self.state.meta.get("seq", False)
        for ep in self.epochs(iters, data=(rows.indptr, rows.idx, rows.val, rows.y)):
            if seq:
                loss = LO.train_pass_seq(self.state, self.P, rows.indptr, rows.idx, rows.val, rows.y,
                                         self.rows_seen)
            elif minibatch:
                loss = LO.train_pass_minibatch(self.state, self.P, rows.indptr, rows.idx, rows.val, rows.y,
                                               self.rows_seen, mb)
            elif shared:
                loss = LO.train_pass_shared(self.state, self.P, rows.indptr, rows.idx, rows.val, rows.y,
                                            self.rows_seen)
            else:
                loss = LO.train_pass(self.state, self.P, rows.indptr, rows.idx, rows.val, rows.y,
                                     None, mb)
            self.rows_seen += rows.n
            self.mix()
            if self.epoch_converged(float(loss.sum().item()), rows=rows.n):
                log.info("%s converged at epoch %d", self.NAME, ep + 1)
                break
        return self

    def mix(self) -> None:
        """Mix replicas (and ranks): average, or argmin-KLD for covariance learners."""
        st = self.state
        kld = self.covar
        if st.R == 1 and not kld and st.device.type == "cpu" and not self._dp():
            # one replica, plain average: num / den = w * 1 / 1 = w exactly, so the mix is the
            # identity; skip its three passes over the (2^24-dim) table
            self._w, self._cov = st.S[0, ..., 0].clone(), None
            return
        num, den, cnt = LO.mix_reduce(st, kld)
        if self.mixer is not None and self.mixer.world > 1:
            self.mixer.all_reduce_sum([num, den, cnt])
        self._w, self._cov = LO.mix_apply(st, kld, num, den, cnt)

    # ------------------------------------------------------------------ model
    def weights(self) -> tuple[torch.Tensor, torch.Tensor | None]:
        if self._w is None:
            self.mix()
        return self._w, self._cov

    def touched_features(self, device: bool = False):
        """Ids of the features any replica (any rank) updated: numpy, or the device tensor."""
        t = self.state.touched.amax(0) if self.state.R > 1 else self.state.touched[0]
        if self._dp():   # one model table on every rank: features seen by any rank
            f = t.to(torch.float32)
            self.mixer.all_reduce_sum([f])
            t = f > 0
        ids = torch.nonzero(t).flatten()
        return ids if device else ids.cpu().numpy()

    def _feature_names(self, ids, arrow: bool = False):
        """Model-table feature names of ``ids`` (numpy, or a device tensor)."""
        if self.encoder is not None and getattr(self.encoder, "string_names", False) and arrow:
            # integer-named string features (a feature_hashing result): an Arrow string column,
            # formatted on the device when the ids live there (ops/touched.py int_strings:
            # 2.9 M names 126 ms through pyarrow's host cast, 1.2 s as Python str objects)
            from ..ops.touched import int_strings

            t = ids if torch.is_tensor(ids) else torch.from_numpy(np.asarray(ids, dtype=np.int64))
            return pd.arrays.ArrowExtensionArray(int_strings(t))
        if torch.is_tensor(ids):
            ids = ids.cpu().numpy()
        if self.encoder is not None and self.encoder.mode == "dict":
            return self.encoder.decode(ids)
        if self.encoder is not None and getattr(self.encoder, "string_names", False):
            return list(map(str, ids.tolist()))
        return ids.tolist()

    def model_table(self) -> pd.DataFrame:
        w, cov = self.weights()
        ids = self.touched_features(device=True)
        W = w[:, ids].cpu().numpy()
        names = self._feature_names(ids, arrow=self.TASK != "multiclass")
        C = cov[:, ids].cpu().numpy() if (cov is not None and self.covar) else None
        if self.TASK == "multiclass":
            L = len(self.labels)
            d = {"label": np.repeat(np.array(self.labels, dtype=object), len(ids)),
                 "feature": names * L, "weight": W.reshape(-1)}
            if C is not None:
                d["covar"] = C.reshape(-1)
            return pd.DataFrame(d)
        d = {"feature": names, "weight": W[0]}
        if C is not None:
            d["covar"] = C[0]
        return pd.DataFrame(d)

    def load_model_table(self, df: pd.DataFrame) -> None:
        """Warm start (``-loadmodel``): seed every replica with (feature, weight[, covar])."""
        st = self.state
        feats = df["feature"].tolist()
        if self.encoder is not None and self.encoder.mode == "dict":
            csr = self.encoder.encode([[str(f)] for f in feats], add_new=False)
            ids = csr.idx
        else:
            ids = np.asarray([int(f) for f in feats], dtype=np.int64)
        ok = (ids >= 0) & (ids < st.dims)
        ids_t = torch.from_numpy(ids[ok]).to(st.device)
        lab = torch.zeros_like(ids_t)
        if self.TASK == "multiclass" and "label" in df.columns:
            lut = {v: i for i, v in enumerate(self.labels or [])}
            lab = torch.tensor([lut.get(v, 0) for v in np.asarray(df["label"])[ok]], device=st.device)
        wv = torch.tensor(np.asarray(df["weight"], dtype=np.float32)[ok], device=st.device)
        st.S[:, lab, ids_t, 0] = wv
        if self.covar and "covar" in df.columns:
            st.S[:, lab, ids_t, 1] = torch.tensor(np.asarray(df["covar"], dtype=np.float32)[ok],
                                                  device=st.device)
        st.touched[:, ids_t] = 1

    # ------------------------------------------------------------------ inference
    def decision_function(self, features=None, rows: SparseRows | None = None) -> torch.Tensor:
        rows = rows if rows is not None else self.prepare(features, None, train=False)
        w, _ = self.weights()
        out, _ = LO.predict_scores(w, rows.indptr, rows.idx, rows.val)
        return out if self.TASK == "multiclass" else out[:, 0]

    def predict(self, features=None, rows: SparseRows | None = None) -> np.ndarray:
        s = self.decision_function(features, rows)
        if self.TASK == "multiclass":
            best = s.argmax(1).cpu().numpy()
            return np.array([self.labels[i] for i in best], dtype=object)
        if self.ALGO in ("logress", "adagrad_regr", "adadelta_regr") or (
                self.ALGO == "general" and self.P.loss == LO.LOSSES["log"]):
            return torch.sigmoid(s).cpu().numpy()
        return s.cpu().numpy()


# ---------------------------------------------------------------- concrete SQL functions
def _learner(name, algo, task, extra_opts=(), doc="", default_iters=1, default_loss="hinge"):
    opts = [o for o in LEARNER_BASE_OPTS if not (o.name == "iters" and default_iters != 1)]
    if default_iters != 1:
        opts.append(opt("iters", "iterations", default_iters, int,
                        "The maximum number of iterations (epochs)", aliases=("iter",)))
    names = {o.name for o in opts}
    for o in extra_opts:
        if o.name not in names:
            opts.append(o)
            names.add(o.name)
    cls = type(name.title().replace("_", ""), (OnlineLinearLearner,),
               {"NAME": name, "ALGO": algo, "TASK": task, "OPTIONS": opts, "__doc__": doc,
                "DEFAULT_LOSS": default_loss})
    return cls


_C = opt("c", "aggressiveness", 1.0, float, "Aggressiveness parameter C")
_R = opt("r", "regularization", 0.1, float, "Regularization parameter r")
_PHI = opt("phi", "confidence", None, float, "Confidence parameter phi")
_ETA_CONF = opt("eta", "hyper_c", None, float, "Confidence level eta (phi = probit(eta))")
_EPS_INS = opt("epsilon", None, 0.1, float, "Sensitivity to prediction mistakes")

TrainPerceptron = _learner("train_perceptron", "perceptron", "binary", doc="Rosenblatt perceptron")
TrainPA = _learner("train_pa", "pa", "binary", doc="Passive-Aggressive (Crammer et al. 2006)")
TrainPA1 = _learner("train_pa1", "pa1", "binary", [_C], doc="PA-I")
TrainPA2 = _learner("train_pa2", "pa2", "binary", [_C], doc="PA-II")
TrainCW = _learner("train_cw", "cw", "binary", [_PHI, _ETA_CONF], doc="Confidence-weighted (Dredze 2008)")
TrainAROW = _learner("train_arow", "arow", "binary", [_R], doc="AROW (Crammer 2009)")
TrainAROWh = _learner("train_arowh", "arowh", "binary", [_R, _C], doc="AROW with hinge threshold C")
TrainSCW = _learner("train_scw", "scw", "binary", [_PHI, _ETA_CONF, _C], doc="SCW-I (Wang 2012)")
TrainSCW2 = _learner("train_scw2", "scw2", "binary", [_PHI, _ETA_CONF, _C], doc="SCW-II")
TrainAdaGradRDA = _learner("train_adagrad_rda", "adagrad_rda", "binary", [
    opt("eta", "eta0", 0.1, float, "Learning rate"),
    opt("lambda", None, 1e-6, float, "Regularization (RDA L1)"),
    opt("scale", None, 100.0, float, "Scaling factor", inert=_SCALE_INERT)], doc="AdaGrad-RDA hinge")
TrainClassifier = _learner("train_classifier", "general", "binary", GENERAL_OPTS, default_iters=10,
                           default_loss="hinge", doc="GeneralClassifierUDTF")

_LOGRESS_OPTS = [opt("eta0", None, 0.1, float, "Initial learning rate"),
                 opt("t", "total_steps", -1.0, float, "Total steps"),
                 opt("power_t", None, 0.1, float, "Inverse scaling exponent"),
                 opt("eta", None, None, float, "Fixed learning rate")]
Logress = _learner("logress", "logress", "regression", _LOGRESS_OPTS, doc="SGD logistic regression")
TrainLogregr = _learner("train_logregr", "logress", "regression", _LOGRESS_OPTS)
TrainLogisticRegr = _learner("train_logistic_regr", "logress", "regression", _LOGRESS_OPTS)
TrainPA1Regr = _learner("train_pa1_regr", "pa1_regr", "regression", [_C, _EPS_INS])
TrainPA1aRegr = _learner("train_pa1a_regr", "pa1a_regr", "regression", [_C, _EPS_INS])
TrainPA2Regr = _learner("train_pa2_regr", "pa2_regr", "regression", [_C, _EPS_INS])
TrainPA2aRegr = _learner("train_pa2a_regr", "pa2a_regr", "regression", [_C, _EPS_INS])
TrainAROWRegr = _learner("train_arow_regr", "arow_regr", "regression", [_R])
TrainAROWeRegr = _learner("train_arowe_regr", "arowe_regr", "regression", [_R, _EPS_INS])
TrainAROWe2Regr = _learner("train_arowe2_regr", "arowe2_regr", "regression", [_R, _EPS_INS])
TrainAdaGradRegr = _learner("train_adagrad_regr", "adagrad_regr", "regression", [
    opt("eta", "eta0", 1.0, float, "Learning rate"), opt("eps", None, 1.0, float, "Denominator"),
    opt("scale", None, 100.0, float, "Scaling factor", inert=_SCALE_INERT)])
TrainAdaDeltaRegr = _learner("train_adadelta_regr", "adadelta_regr", "regression", [
    opt("rho", "decay", 0.95, float, "Decay"), opt("eps", None, 1e-6, float, "Denominator"),
    opt("scale", None, 100.0, float, "Scaling factor", inert=_SCALE_INERT)])
TrainRegressor = _learner("train_regressor", "general", "regression", GENERAL_OPTS, default_iters=10,
                          default_loss="squared", doc="GeneralRegressorUDTF")

TrainMulticlassPerceptron = _learner("train_multiclass_perceptron", "perceptron", "multiclass")
TrainMulticlassPA = _learner("train_multiclass_pa", "pa", "multiclass")
TrainMulticlassPA1 = _learner("train_multiclass_pa1", "pa1", "multiclass", [_C])
TrainMulticlassPA2 = _learner("train_multiclass_pa2", "pa2", "multiclass", [_C])
TrainMulticlassCW = _learner("train_multiclass_cw", "cw", "multiclass", [_PHI, _ETA_CONF])
TrainMulticlassAROW = _learner("train_multiclass_arow", "arow", "multiclass", [_R])
TrainMulticlassAROWh = _learner("train_multiclass_arowh", "arowh", "multiclass", [_R, _C])
TrainMulticlassSCW = _learner("train_multiclass_scw", "scw", "multiclass", [_PHI, _ETA_CONF, _C])
TrainMulticlassSCW2 = _learner("train_multiclass_scw2", "scw2", "multiclass", [_PHI, _ETA_CONF, _C])

LEARNERS = {c.NAME: c for c in [
    TrainPerceptron, TrainPA, TrainPA1, TrainPA2, TrainCW, TrainAROW, TrainAROWh, TrainSCW,
    TrainSCW2, TrainAdaGradRDA, TrainClassifier, Logress, TrainLogregr, TrainLogisticRegr,
    TrainPA1Regr, TrainPA1aRegr, TrainPA2Regr, TrainPA2aRegr, TrainAROWRegr, TrainAROWeRegr,
    TrainAROWe2Regr, TrainAdaGradRegr, TrainAdaDeltaRegr, TrainRegressor,
    TrainMulticlassPerceptron, TrainMulticlassPA, TrainMulticlassPA1, TrainMulticlassPA2,
    TrainMulticlassCW, TrainMulticlassAROW, TrainMulticlassAROWh, TrainMulticlassSCW,
    TrainMulticlassSCW2]}


def train(name: str, features, labels, options: str | None = None, device=None, **kw) -> pd.DataFrame:
    """Functional UDTF form of any linear learner: returns its model table."""
    cls = LEARNERS[name]
    return cls(options, device, **kw).fit(features, labels).model_table()
