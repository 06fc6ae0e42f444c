"""``train_fm`` — factorization machines (Rendle ICDM'10) and ``fm_predict``.

Reference behaviour: Hivemall FactorizationMachineUDTF / FMHyperParameters /
FactorizationMachineModel / FMPredictGenericUDAF (upstream core/src/main/java/hivemall/fm/;
SURVEY.md §2.3.4, K5, O5).

MI355X design: the model is a dense HBM table (w fp32 [dims], V bf16 [dims, KP] with
stochastic-rounded SGD updates, w0 fp32); rows are uploaded once as CSR and replayed per
epoch; one launch of ``hm_fm_step`` trains a batch (one wave64 per row, Hogwild across
waves).  ``-fp32`` keeps V in fp32.

Model table (pinned, docs/compat.md O5): ``(feature, W_i float, V_if array<float>)``; the
global bias w0 is the row ``feature = 0`` with ``V_if = NULL``.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from ..ops.fm import FMHyper, fm_step, hot_flags, new_state_tables
from ..ops.touched import mark_touched

# global-bias shards on the GPU (see ops/fm.py): one same-address atomic per row capped train_fm
# at ~40 M rows/s on MI355X whatever the grid (profiles/fm_grid_probe_r1.log)
W0_SHARDS = 64
W0_STRIDE = 32      # floats between shards: one 128-B line each
from ..utils.features import CSR, FeatureEncoder
from ..utils.options import UDFArgumentException, flag, opt
from .base import MIX_OPTS, ConversionState, Learner, log, parse_labels_binary
from .linear import SparseRows, _arrow_string_lists, encode_rows
from ..utils.reduce import tmax


def _is_arrow(x) -> bool:
    from ..io.ingest import is_arrow_like

    return is_arrow_like(x)


def _string_rows(rows) -> bool:
    """Rows of feature strings (Arrow list<string>, or Python lists whose first row holds str)."""
    if _is_arrow(rows):
        import pyarrow as pa

        t = rows.dtype.pyarrow_dtype if hasattr(rows, "dtype") and hasattr(rows.dtype, "pyarrow_dtype") \
            else rows.type
        return (pa.types.is_list(t) or pa.types.is_large_list(t)) and \
            (pa.types.is_string(t.value_type) or pa.types.is_large_string(t.value_type))
    first = next((r for r in rows if r is not None and len(r)), None)
    return first is not None and all(isinstance(v, str) for v in first)


FM_OPTS = [
    flag("classification", "c", "Act as classification"),
    opt("factors", "factor", 5, int, "The number of latent factors", aliases=("k",)),
    opt("iters", "iterations", 1, int, "Iterations", aliases=("iter",)),
    opt("eta0", None, 0.05, float, "Initial learning rate"),
    opt("eta", None, "inverse", str, "Learning rate scheme: fixed, simple, inverse"),
    opt("power_t", None, 0.1, float, "Inverse scaling exponent"),
    opt("t", "total_steps", -1.0, float, "Total steps for -eta simple"),
    opt("lambda0", "lambda_w0", 0.01, float, "L2 regularization of w0"),
    opt("lambda", "lambda_v", 0.01, float, "L2 regularization of V"),
    opt("lambda_w", "lambdaW", 0.01, float, "L2 regularization of w"),
    opt("sigma", None, 0.1, float, "Stddev of the gaussian V initialisation"),
    opt("init_v", None, "gaussian", str, "V initialisation: random | gaussian"),
    opt("maxval", "max_init_value", 1.0, float, "Range of the uniform V initialisation"),
    opt("min", "min_target", None, float, "Minimum target (regression clipping)"),
    opt("max", "max_target", None, float, "Maximum target (regression clipping)"),
    opt("seed", None, -1, int, "Seed"),
    opt("num_features", "p", -1, int, "Number of features (default: max index + 1)"),
    opt("feature_hashing", None, -1, int, "Hash features into 2^bits"),
    flag("int_feature", None, "Features are integers"),
    flag("adareg", "adaptive_regularization", "Adaptive regularization (Rendle WSDM'12)"),
    opt("va_ratio", "validation_ratio", 0.05, float, "Held-out ratio for -adareg"),
    opt("va_threshold", "validation_threshold", 1000, int, "Min rows before -adareg starts"),
    opt("cv_rate", "convergence_rate", 0.005, float, "Convergence threshold"),
    flag("disable_cv", "disable_cvtest", "Disable convergence check"),
    flag("fp32", None, "[engine] keep V in fp32 on the GPU (default bf16)"),
    opt("batch_size", None, 1 << 20, int, "[engine] rows per kernel launch"),
    opt("grid", None, 0, int, "[engine] kernel workgroups: the Hogwild rows in flight / 4 "
                              "(0 = auto: 256 on 6 of the 8 XCDs, inside the bf16 3e-3 parity "
                              "tolerance; 128 with HM_FM_XCDS=8; docs/compat.md)"),
    opt("engine", None, "rowwise", str, "[engine] rowwise (per-row Hogwild kernel) | minibatch "
        "(dense mini-batch GEMMs + AdaGrad; for low-dimensional dense rows, models/fm_dense.py)"),
    opt("mini_batch", None, 8192, int, "[engine] rows per step of -engine minibatch"),
    opt("dp_lr_power", None, 0.5, float,
        "[engine] data-parallel training with -mix_interval > 0 over N ranks: every rank's "
        "replica steps with eta0 * N^p (docs/compat.md, FM/BPR data-parallel quality)"),
] + MIX_OPTS
_ETAS = {"fixed": 0, "simple": 1, "inverse": 2, "inv": 2}


class FMTrainer(Learner):
    SQL_DP = "shard"
    ARROW_INPUT = True      # Arrow list<string> rows are parsed on the device (-feature_hashing)
    NAME = "train_fm"
    OPTIONS = FM_OPTS

    def __init__(self, options: str | None = None, device=None, **kw):
        super().__init__(options, device, **kw)
        c = self.cl
        self.k = int(c["factors"])
        if self.k <= 0 or self.k > 32:
            raise UDFArgumentException("train_fm: -factors must be in [1, 32]")
        self.kp = next(p for p in (4, 8, 16, 32) if p >= self.k)
        eta = c["eta"].lower()
        if eta not in _ETAS:
            raise UDFArgumentException(f"train_fm: unknown -eta scheme {eta}")
        self.h = FMHyper(eta0=c["eta0"], power_t=c["power_t"], total_steps=c["t"],
                         eta_kind=_ETAS[eta], lambda0=c["lambda0"], lambda_w=c["lambda_w"],
                         lambda_v=c["lambda"],
                         min_target=c["min"] if c["min"] is not None else -3.4e38,
                         max_target=c["max"] if c["max"] is not None else 3.4e38,
                         classification=bool(c["classification"]), seed=self.seed)
        # data-parallel step rule, only for replicas mixed during training (-mix_interval > 0):
        # per-epoch mixing of N SGD replicas at eta0 * N^0.5 measured +2.8e-3 / +4.4e-3 / +7.5e-3
        # held-out logloss at N = 2 / 4 / 8 vs one learner, against +5.5e-3 / +1.2e-2 / +1.9e-2
        # for the plain mean (benchmarks/dp_sim_mf_fm.py, profiles/r5/dp_sim_fm.jsonl); with the
        # default -mix_interval 0 (one average at the end: Hivemall's mappers) eta0 is unchanged
        self.dp_power = float(c["dp_lr_power"]) if (self._dp() and int(c["mix_interval"]) > 0) else 0.0
        if self.dp_power:
            self.h.eta0 = float(c["eta0"]) * float(self.mixer.world) ** self.dp_power
        self.encoder: FeatureEncoder | None = None
        if c["feature_hashing"] > 0:
            self.encoder = FeatureEncoder("hash", num_features=1 << int(c["feature_hashing"]))
        self.state: dict | None = None
        self.dims: int | None = int(c["num_features"]) if c["num_features"] > 0 else None
        if c["feature_hashing"] > 0:
            self.dims = (1 << int(c["feature_hashing"])) + 1
        self.cv = ConversionState(not c["disable_cv"], c["cv_rate"])
        self.t = 0
        self.grid = int(c["grid"])

    # ------------------------------------------------------------------ state
    def init_state(self, dims: int) -> dict:
        self.dims = int(dims)
        g = torch.Generator(device="cpu").manual_seed(self.seed)
        dev = self.device
        bf16 = dev.type == "cuda" and not self.cl["fp32"]
        V = torch.zeros((self.dims, self.kp), dtype=torch.float32)
        if self.cl["init_v"] == "random":
            V[:, : self.k] = (torch.rand(self.dims, self.k, generator=g) - 0.5) * (
                self.cl["maxval"] / math.sqrt(self.k))
        else:
            V[:, : self.k] = torch.randn(self.dims, self.k, generator=g) * self.cl["sigma"]
        if dev.type == "cuda":
            # w in the padding of each feature's V row (ops/fm.py new_state_tables)
            w, Vt = new_state_tables(self.dims, self.kp, torch.bfloat16 if bf16 else torch.float32, dev)
            Vt.copy_(V)
        else:
            w, Vt = torch.zeros(self.dims, dtype=torch.float32), V.contiguous()
        self.state = dict(w=w, V=Vt,
                          w0=torch.zeros(W0_SHARDS * W0_STRIDE if dev.type == "cuda" else 1,
                                         dtype=torch.float32, device=dev))
        self.touched = torch.zeros(self.dims, dtype=torch.bool, device=dev)
        return self.state

    def adopt_state(self, st: dict) -> dict:
        """Checkpoint load (io/checkpoint.py): the saved tensors copied into this device's layout
        (w inside the V records with HM_FM_W_RECORD=1)."""
        self.init_state(int(st["V"].shape[0]))
        for k, v in st.items():
            cur = self.state.get(k)
            if cur is not None and cur.shape == v.shape and cur.dtype == v.dtype:
                cur.copy_(v)
            else:
                self.state[k] = v
        return self.state

    # ------------------------------------------------------------------ data
    def prepare(self, features, labels=None, train: bool = True) -> SparseRows:
        """Feature rows -> device CSR.  With -feature_hashing on the GPU, string rows are parsed
        and mhash'd there (io/ingest.py, hm_feat_parse); otherwise by the host encoder."""
        y = None
        if labels is not None:
            y = parse_labels_binary(labels) if self.h.classification else \
                np.asarray(labels, dtype=np.float32).reshape(-1)
        if (self.device.type == "cuda" and self.encoder is not None and self.encoder.mode == "hash"
                and not isinstance(features, CSR) and _string_rows(features)):
            from ..io import ingest

            ip, idx, val, _ = ingest.csr_device(features, "hash", self.encoder.num_features,
                                                device=self.device, seed=self.encoder.seed)
            yt = None if y is None else torch.from_numpy(y).to(self.device)
            return SparseRows(ip, idx.to(torch.int32), val, yt)
        if not isinstance(features, (list, CSR)) and _is_arrow(features) and not _arrow_string_lists(features):
            features = features.to_pylist()
        csr, self.encoder = encode_rows(features, self.encoder, train)
        return SparseRows.from_csr(csr, y, self.device)

    def _ensure(self, rows: SparseRows):
        if self.state is None:
            dims = self.dims
            if dims is None:
                dims = int(tmax(rows.idx)) + 1 if rows.idx.numel() else 1
                if self.encoder is not None and self.encoder.mode == "dict":
                    if self._dp():
                        raise UDFArgumentException(
                            "train_fm: data-parallel training needs integer feature indices or "
                            "-feature_hashing (a per-rank string dictionary gives every rank its own ids)")
                    dims = max(dims, self.encoder.vocab_size())
            # data-parallel replicas share one shape (each rank's shard has its own max id)
            self.init_state(self.agree_max(dims)[0])

    # ------------------------------------------------------------------ training
    def train_rows(self, rows: SparseRows, loss_buf: torch.Tensor | None = None) -> None:
        self._ensure(rows)
        bs = int(self.cl["batch_size"])
        n = rows.n
        # hot features of this pass: their stores go out write-through (ops/fm.py HOT_FRAC)
        self._hot = hot_flags(self.state, rows.idx, n, buf=getattr(self, "_hot", None))
        for k in range(self.dp_batches(n, bs)):
            s = min(n, k * bs)
            e = min(n, s + bs)
            ip = rows.indptr[s:e + 1]   # CSR slice: the kernel reads absolute offsets
            lb = None if loss_buf is None else loss_buf[s:e]
            if e > s:
                fm_step(self.state, ip, rows.idx, rows.val, rows.y[s:e], self.h, self.k, train=True,
                        t0=self.t, loss=lb, grid=self.grid, hot=self._hot)
            self.t += e - s
            mi = int(self.cl["mix_interval"])
            if mi > 0 and self._dp():
                self._nbatches = getattr(self, "_nbatches", 0) + 1
                if self._nbatches % mi == 0:
                    self.mix()
        mark_touched(self.touched, rows.idx, self.dims)

    def mix(self) -> None:
        """Replica averaging over the ranks (w, V, w0; the SGD state has no optimizer slots)."""
        self.mix_tensors([self.state["w"], self.state["V"], self.state["w0"]], [self.touched])

    def fit(self, features=None, labels=None, rows: SparseRows | None = None) -> "FMTrainer":
        rows = rows if rows is not None else self.prepare(features, labels)
        if rows.y is None:
            raise UDFArgumentException("train_fm: labels are required")
        self._ensure(rows)
        if str(self.cl["engine"]).lower() == "minibatch":
            return self._fit_minibatch(rows)
        va = None
        if self.cl["adareg"] and rows.n > int(self.cl["va_threshold"]):
            # hold out the tail as the validation slice for adaptive regularization
            nva = max(1, int(rows.n * float(self.cl["va_ratio"])))
            va = _slice_rows(rows, rows.n - nva, rows.n)
            rows = _slice_rows(rows, 0, rows.n - nva)
        loss_buf = torch.empty(rows.n, dtype=torch.float32, device=self.device)
        for ep in self.epochs(int(self.cl["iters"]), data=(rows.indptr, rows.idx, rows.val, rows.y)):
            self.train_rows(rows, loss_buf)
            if va is not None:
                self._adapt_lambda(va)
            if self.epoch_converged(float(loss_buf.double().sum().item()), rows=rows.n):
                log.info("train_fm converged at epoch %d", ep + 1)
                break
        self.mix()
        return self

    def _fit_minibatch(self, rows: SparseRows) -> "FMTrainer":
        """-engine minibatch (models/fm_dense.py): rows densified to X [n, dims] fp32 in HBM,
        mini-batch AdaGrad steps replayed from HIP graphs; the result is written back into the
        usual state so prediction, model_table and mixing are unchanged."""
        from .fm_dense import DenseMinibatchFM, densify

        dims = self.dims
        if dims > 4096 or rows.n * dims > (1 << 31):
            raise UDFArgumentException(
                f"train_fm -engine minibatch: {rows.n} x {dims} dense rows do not fit the dense "
                "engine (dims <= 4096); use the default rowwise engine for sparse rows")
        if self.cl["adareg"]:
            log.warning("train_fm -engine minibatch: -adareg is not applied by this engine")
        X = densify(rows.indptr, rows.idx, rows.val, dims, self.device)
        y = rows.y.to(self.device, torch.float32)
        if self.h.classification:
            y = torch.where(y > 0, 1.0, -1.0)
        st = self.state
        eng = DenseMinibatchFM(dims, self.k, st["V"].float(), self.device, int(self.cl["mini_batch"]),
                               self.h.eta0, self.h.lambda0, self.h.lambda_w, self.h.lambda_v,
                               self.h.classification, self.h.min_target, self.h.max_target)
        self.no_checkpoint("-engine minibatch")
        for ep in range(int(self.cl["iters"])):
            if self.epoch_converged(eng.epoch(X, y), rows=X.shape[0]):
                log.info("train_fm converged at epoch %d", ep + 1)
                break
        self.t += rows.n * (ep + 1)
        st["w"].copy_(eng.w)
        st["V"][:, : self.k] = eng.V[:, : self.k].to(st["V"].dtype)
        st["w0"].zero_()
        st["w0"][0] = eng.w0[0]
        mark_touched(self.touched, rows.idx, self.dims)
        self.mix()
        return self

    def _adapt_lambda(self, va: SparseRows) -> None:
        """Adaptive regularization, epoch-level form of Rendle (WSDM'12): one gradient step
        on (lambda_w, lambda_v) of the validation loss w.r.t. the regularised update."""
        pred = self.predict_raw(rows=va)
        y = va.y
        if self.h.classification:
            d = -y / (1 + torch.exp(y * pred))
        else:
            d = pred - y
        w = self.state["w"]
        V = self.state["V"].float()
        grad_scale = float(d.abs().mean().item())
        eta = self.h.eta0
        # d loss / d lambda ≈ -2 eta * <grad_va, theta>; use the parameter norms as the proxy
        self.h.lambda_w = max(0.0, self.h.lambda_w - eta * grad_scale * 1e-3 *
                              float(w.pow(2).mean().item()))
        self.h.lambda_v = max(0.0, self.h.lambda_v - eta * grad_scale * 1e-3 *
                              float(V.pow(2).mean().item()))

    # ------------------------------------------------------------------ inference
    def predict_raw(self, features=None, rows: SparseRows | None = None) -> torch.Tensor:
        rows = rows if rows is not None else self.prepare(features, None, train=False)
        self._ensure(rows)
        out = torch.empty(rows.n, dtype=torch.float32, device=self.device)
        fm_step(self.state, rows.indptr, rows.idx, rows.val, None, self.h, self.k, train=False,
                pred=out)
        return out

    def predict(self, features=None, rows: SparseRows | None = None) -> np.ndarray:
        p = self.predict_raw(features, rows)
        if self.h.classification:
            p = torch.sigmoid(p)
        return p.cpu().numpy()

    # ------------------------------------------------------------------ model table
    def model_table(self) -> pd.DataFrame:
        ids = torch.nonzero(self.touched).flatten()
        W = self.state["w"][ids].cpu().numpy()
        V = self.state["V"][ids][:, : self.k].float().cpu().numpy()
        ids = ids.cpu().numpy()
        if self.encoder is not None and self.encoder.mode == "dict":
            names = self.encoder.decode(ids)
        else:
            as_str = self.encoder is not None and getattr(self.encoder, "string_names", False)
            names = [str(int(i)) if as_str else int(i) for i in ids]
        bias_name = "0" if names and isinstance(names[0], str) else 0
        return pd.DataFrame({
            "feature": [bias_name] + names,
            "W_i": np.concatenate([[float(self.state["w0"].double().sum().item())], W]).astype(np.float32),
            "V_if": [None] + [v for v in V]})


def _slice_rows(rows: SparseRows, s: int, e: int) -> SparseRows:
    a, b = int(rows.indptr[s].item()), int(rows.indptr[e].item())
    return SparseRows((rows.indptr[s:e + 1] - a).contiguous(), rows.idx[a:b].contiguous(),
                      None if rows.val is None else rows.val[a:b].contiguous(),
                      None if rows.y is None else rows.y[s:e].contiguous())


def train_fm(features, labels, options: str | None = None, device=None, **kw) -> pd.DataFrame:
    return FMTrainer(options, device, **kw).fit(features, labels).model_table()


def fm_predict_from_table(table: pd.DataFrame, rows) -> np.ndarray:
    """Score rows of features with an FM model table (the fm_predict UDAF after the join)."""
    w0 = 0.0
    W, V = {}, {}
    for f, wi, vi in zip(table["feature"], table["W_i"], table["V_if"]):
        if vi is None or (isinstance(vi, float) and np.isnan(vi)):
            w0 = float(wi)
            continue
        W[f] = float(wi)
        V[f] = np.asarray(vi, dtype=np.float64)
    k = len(next(iter(V.values()))) if V else 0
    out = np.empty(len(rows))
    from ..utils.features import parse_feature
    for r, feats in enumerate(rows):
        s = np.zeros(k)
        sq = np.zeros(k)
        lin = w0
        for ft in feats:
            if isinstance(ft, str):
                name, x = parse_feature(ft)
                key = int(name) if name.lstrip("-").isdigit() else name
            else:
                key, x = int(ft), 1.0
            if key in W:
                lin += W[key] * x
                s += V[key] * x
                sq += (V[key] * x) ** 2
        out[r] = lin + 0.5 * float((s * s - sq).sum())
    return out


from ..registry import udaf as _udaf  # noqa: E402


@_udaf("fm_predict")
def fm_predict(Wj, Vjf, Xj):
    """FMPredictGenericUDAF: Σ W_j·x_j + ½ Σ_f [(Σ_j V_jf x_j)² − Σ_j V_jf² x_j²] over the
    joined rows of one example (the bias row ``feature 0`` carries w0 with x = 1)."""
    lin = 0.0
    S = None
    sq = None
    for w, v, x in zip(Wj, Vjf, Xj):
        if x is None:
            continue
        x = float(x)
        if w is not None and not (isinstance(w, float) and math.isnan(w)):
            lin += float(w) * x
        if v is not None and not (isinstance(v, float)):
            vv = np.asarray(v, dtype=np.float64) * x
            S = vv.copy() if S is None else S + vv
            sq = vv * vv if sq is None else sq + vv * vv
    if S is None:
        return lin
    return lin + 0.5 * float((S * S - sq).sum())
