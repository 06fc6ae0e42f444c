"""``train_ffm`` — field-aware factorization machines (Juan et al., RecSys'16).

Reference behaviour: Hivemall FieldAwareFactorizationMachineUDTF / FFMStringFeatureMapModel
(core/src/main/java/hivemall/fm/FieldAwareFactorizationMachineUDTF.java,
hivemall/fm/FFMHyperParameters).

MI355X design:
* the model is a dense HBM-resident table V/G [num_features, num_fields, Kp] (fp32) plus
  FTRL state for the linear term — 2^20 features x 39 fields x k=4 is 0.65 GB per table,
  trivially resident in 288 GB;
* training rows are uploaded once as padded-ELL tensors and replayed per epoch (replaces
  the NioStatefulSegment spill file);
* each batch is ONE launch of the fused kernel ``hm_ffm_step`` (gather -> pair dots ->
  logistic loss -> AdaGrad(V) + FTRL(w) Hogwild update);
* data parallelism: with a mixer (``parallel.mix.ModelMixer``) the replicas are averaged
  over RCCL every ``-mix_interval`` batches and at the end (the MixServer / GROUP BY avg
  replacement).

Model table (pinned, docs/compat.md O4): ``(model_id string, i int, Wi float, Vi array<float>)``
keyed as in :mod:`models.ffm_keys`: ``i = -1`` bias, ``i = feature`` linear weight,
``i = NF + feature*F + field`` the latent vector V[feature, field].
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from ..ops import ffm as _ffm_ops
from ..ops.ffm import (FFMHyper, ffm_step, is_packed, lin_record_views, linear_mix_tensors,
                       new_state_tables)

# GPU block layouts: w / wz / wn as the 16-B record after each feature's slots (ops/ffm.py
# lin_record_views); HM_FFM_LIN_SEPARATE=1 keeps three separate arrays (A/B only)
LIN_IN_BLOCK = os.environ.get("HM_FFM_LIN_SEPARATE", "0") != "1"
from ..ops.touched import mark_touched
from ..utils.features import CSR, parse_ffm_rows
from ..utils.options import opt, flag, UDFArgumentException
from .base import COMMON_ITER_OPTS, ConversionState, Learner, log, parse_labels_binary
from ..utils.reduce import tmax


@dataclass
class FFMBatch:
    idx: torch.Tensor               # int32 [B, F]
    fld: torch.Tensor | None        # int32 [B, F] (None => field = slot position)
    val: torch.Tensor | None        # f32 [B, F]   (None => 1.0)
    y: torch.Tensor | None          # f32 [B]

    @property
    def n(self) -> int:
        return self.idx.shape[0]

    def slice(self, s: int, e: int) -> "FFMBatch":
        f = lambda t: None if t is None else t[s:e]
        return FFMBatch(self.idx[s:e], f(self.fld), f(self.val), f(self.y))

    def to(self, device) -> "FFMBatch":
        f = lambda t: None if t is None else t.to(device, non_blocking=True).contiguous()
        return FFMBatch(f(self.idx), f(self.fld), f(self.val), f(self.y))


def csr_to_ffm_batch(csr: CSR, y: np.ndarray | None, width: int | None = None) -> FFMBatch:
    idx, val, fld = csr.to_ell(width)
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a))
    return FFMBatch(t(idx), t(fld), t(val), t(y))


# Data-parallel step-size scaling of the mixed replicas (docs/compat.md "Data-parallel
# quality"): N replicas that each run AdaGrad on 1/N of the rows and are averaged every mix move
# like ONE learner over all rows with its step size divided by sqrt(N) (drift and gradient
# noise both match at p = 0.5 in the small-step limit); the measured gap at the bench's shape,
# N = 8, fp32, vs one rank on the same total rows (benchmarks/dp_sim.py, profiles/r4/): p = 0
# (plain mean) +5.3e-3, 0.5 +1.5e-3, 0.75 +2.8e-4, 1.0 -6e-4.
DP_LR_POWER = 0.75

# Early-training ramp of the GPU kernel (train_batch).  In the first rows of a run every row
# moves the same hot (feature, field) slots, and the Hogwild kernel's concurrent read-modify-
# write of a slot keeps one of the racing rows' updates: held-out logloss after 500 K rows is
# 0.0195 above the sequential engine, 0.0107 even on 8 blocks, 0 on one
# (profiles/r4/ffm_early_grid_curve.jsonl).  Kernel variant 6 (fp32 state) adds every slot's
# update with float atomics instead (4 M rows/s: the hot addresses serialise): over the first
# 2^18 rows it takes the gap at 500 K rows to 0.0026 and at 2 M rows from 0.0069 to 0.0031
# (profiles/r4/ffm_early_ramp_atomic*.jsonl).  HM_FFM_RAMP_VARIANT=-1 runs the ramp rows on
# HM_FFM_RAMP_GRID blocks of the default kernel instead (0.017 at 256 blocks).
RAMP_ROWS = int(os.environ.get("HM_FFM_RAMP_ROWS", str(1 << 18)))
RAMP_GRID = int(os.environ.get("HM_FFM_RAMP_GRID", "1024"))
RAMP_VARIANT = int(os.environ.get("HM_FFM_RAMP_VARIANT", "6"))   # kernel variant of the ramp rows


# Divergence guard of the step rule (FFMTrainer._dp_guard): a rise of the mean training loss
# between two mix intervals by more than this fraction drops p to DP_GUARD_POWER.
DP_GUARD_RISE = 0.02
DP_GUARD_POWER = 0.5


def dp_lin_mode(world: int) -> int | None:
    """ops.ffm.ffm_step's ``lin_mode`` for a replica of ``world`` ranks (FFMTrainer.lin_mode)."""
    return 0 if world > 1 else None


def dp_lr_scale(world: int, power: float = DP_LR_POWER) -> float:
    """Step-size factor of a data-parallel replica (1.0 on one rank)."""
    return float(world) ** float(power) if world > 1 else 1.0


class FFMTrainer(Learner):
    NAME = "train_ffm"
    SQL_DP = "shard"
    ARROW_INPUT = True      # Arrow list<string> feature columns are parsed on the device
    OPTIONS = COMMON_ITER_OPTS + [
        flag("classification", "c", "Act as classification (logistic loss); labels 0/1 or -1/1"),
        opt("factors", "factor", 4, int, "The number of latent factors k", aliases=("k",)),
        opt("eta0", None, 0.2, float, "AdaGrad learning rate for V"),
        opt("eps", None, 1.0, float, "AdaGrad denominator constant"),
        opt("lambda", "lambda_v", 1e-4, float, "L2 regularization for V", aliases=("lambda0",)),
        opt("alpha", "alphaFTRL", 0.2, float, "FTRL alpha (learning rate) for w/w0"),
        opt("beta", "betaFTRL", 1.0, float, "FTRL beta (smoothing)"),
        opt("lambda1", None, 1e-3, float, "FTRL L1 regularization"),
        opt("lambda2", None, 1e-4, float, "FTRL L2 regularization"),
        flag("global_bias", "w0", "Include the global bias term w0"),
        flag("disable_wi", "no_coeff", "Do not include the linear term w_i"),
        flag("no_norm", "disable_norm", "Disable instance-wise L2 normalization"),
        flag("bf16_state", None, "[engine] keep V and the AdaGrad state in bf16 on the GPU "
                                 "(stochastic rounding); halves the HBM traffic"),
        flag("elementwise_adagrad", None, "[engine] one AdaGrad accumulator per V element "
                                          "instead of one per (feature, field) slot"),
        flag("split_state", None, "[engine] separate V and G tables on the GPU instead of the "
                                  "packed V|G slot layout (A/B)"),
        opt("feature_hashing", None, -1, int, "Hash feature indices into 2^bits"),
        opt("num_features", None, -1, int, "Number of (hashed) features; inferred when -1"),
        opt("num_fields", None, -1, int, "Number of fields; inferred from data when -1"),
        opt("init_v", None, "random", str, "V initialization: random (uniform) | gaussian"),
        opt("maxval", "max_init_value", 1.0, float, "uniform init: V ~ U[0, maxval/sqrt(k))"),
        opt("sigma", None, 0.1, float, "gaussian init stddev"),
        opt("min", "min_target", None, float, "Minimum target (regression clipping)"),
        opt("max", "max_target", None, float, "Maximum target (regression clipping)"),
        opt("grid", None, 0, int, "[engine] kernel workgroups: bounds the Hogwild rows in flight "
            "(0 = auto; 1 = one block, the sequential learner)"),
        opt("atomic_rows", None, None, int,
            "[engine] a learner's first N rows run on the kernel that adds every slot update with "
            "float atomics (no update lost to concurrent rows; ~4 M rows/s fp32): the quality / "
            "speed knob of the Hogwild learner; default 2^18, docs/compat.md)"),
        opt("dp_lr_power", None, DP_LR_POWER, float,
            "[engine] data-parallel training over N ranks: every rank's replica steps with "
            "eta0 * N^p and alpha * N^p, so the mean of the mixed replicas tracks one learner "
            "over the union of the ranks' rows (docs/compat.md)"),
    ]

    def __init__(self, options: str | None = None, device=None, num_features: int | None = None,
                 num_fields: int | None = None, **kw):
        super().__init__(options, device, **kw)
        c = self.cl
        self.k = int(c["factors"])
        if self.k <= 0:
            raise UDFArgumentException("-factors must be positive")
        self.kp = ((self.k + 3) // 4) * 4
        self.hyper = FFMHyper(
            eta0=c["eta0"], eps=c["eps"], lambda_v=c["lambda"], alpha=c["alpha"], beta=c["beta"],
            lambda1=c["lambda1"], lambda2=c["lambda2"],
            min_target=c["min"] if c["min"] is not None else -3.4e38,
            max_target=c["max"] if c["max"] is not None else 3.4e38,
            classification=bool(c["classification"]), use_linear=not c["disable_wi"],
            use_bias=bool(c["global_bias"]), norm=not c["no_norm"])
        # the N^p step rule was fitted for replicas mixed every few batches (benchmarks/dp_sim.py,
        # mix every 10); with the default -mix_interval 0 (average once at the end: Hivemall's
        # mappers, each on the plain eta0) the replicas keep the learner's step size
        self._dp_power = float(c["dp_lr_power"]) if (self._dp() and int(c["mix_interval"]) > 0) else 0.0
        self._base_eta0, self._base_alpha = self.hyper.eta0, self.hyper.alpha
        self._set_dp_power(self._dp_power)
        self._mix_loss = None      # device [sum, rows] of the training loss since the last mix
        self._prev_mix_loss = None
        nf = num_features
        if nf is None and c["feature_hashing"] > 0:
            nf = 1 << int(c["feature_hashing"])
        if nf is None and c["num_features"] > 0:
            nf = int(c["num_features"])
        self.num_features = nf
        self.num_fields = num_fields if num_fields is not None else (
            int(c["num_fields"]) if c["num_fields"] > 0 else None)
        self.state: dict | None = None
        self.cv = ConversionState(not c["disable_cv"], c["cv_rate"])
        self.rows_seen = 0
        self.grid = int(c["grid"])  # kernel grid override (0 = auto); bounds the Hogwild concurrency
        self.atomic_rows = RAMP_ROWS if c["atomic_rows"] is None else max(0, int(c["atomic_rows"]))
        self.dp_guard_tripped = False

    @property
    def dp_power(self) -> float:
        """The step rule's effective power p (eta0 * N^p), after any divergence-guard fallback;
        a checkpoint scalar (io/checkpoint.py), so a resumed run keeps the fallback."""
        return self._dp_power

    @dp_power.setter
    def dp_power(self, power: float) -> None:
        self._set_dp_power(float(power))

    def lin_mode(self) -> int | None:
        """The linear steps' form: the side table (module default) on one rank; the plain record
        stores for replicas that mix during training (the N^p step rule was calibrated with them,
        and an 8-rank rehearsal measured the side table no better there: +5.2e-3 vs +4.6e-3 against
        the N = 8 sequential reference, profiles/r6/dp_side/)."""
        return dp_lin_mode(self.mixer.world if self._dp() else 1)

    def _set_dp_power(self, power: float) -> None:
        sc = dp_lr_scale(self.mixer.world, power) if self._dp() else 1.0
        self.hyper.eta0 = self._base_eta0 * sc
        self.hyper.alpha = self._base_alpha * sc
        self._dp_power = float(power) if self._dp() else 0.0

    def _dp_guard(self) -> None:
        """Divergence guard of the N^p step rule, checked at every mix: the mean training loss
        of the interval since the last mix (over all ranks) must not rise by more than
        ``DP_GUARD_RISE`` relative to the previous interval's; if it does while p > 0.5, the
        replicas fall back to p = 0.5 (the drift-matching power, docs/compat.md) for the rest of
        the run."""
        if self._mix_loss is None or self._dp_power <= DP_GUARD_POWER:
            self._mix_loss = None
            return
        tot = self._mix_loss.clone()
        self._mix_loss = None
        self.mixer.all_reduce_sum([tot])
        s, n = (float(v) for v in tot.tolist())
        if n <= 0:
            return
        cur = s / n
        prev, self._prev_mix_loss = self._prev_mix_loss, cur
        if prev is not None and cur > prev * (1.0 + DP_GUARD_RISE):
            log.warning("%s: mixed-interval loss rose %.5f -> %.5f at N=%d, p=%.2f: falling back to p=%.2f",
                        self.NAME, prev, cur, self.mixer.world, self._dp_power, DP_GUARD_POWER)
            self._set_dp_power(DP_GUARD_POWER)
            self.dp_guard_tripped = True

    # ------------------------------------------------------------------ model state
    def init_state(self, num_features: int, num_fields: int) -> dict:
        self.num_features, self.num_fields = int(num_features), int(num_fields)
        g = torch.Generator(device="cpu").manual_seed(self.seed)
        dev = self.device
        sdt = torch.bfloat16 if (self.cl["bf16_state"] and dev.type == "cuda") else torch.float32
        # packed V|G slots on the GPU (csrc/kernels/ffm.hip); split tables on the CPU engine
        V, G = new_state_tables(self.num_features, self.num_fields, self.kp, sdt, dev,
                                packed=dev.type == "cuda" and not self.cl["split_state"],
                                slot_g=not self.cl["elementwise_adagrad"])
        if self.cl["init_v"] == "gaussian":
            init = lambda n: torch.randn(n, generator=g) * self.cl["sigma"]
        else:
            init = lambda n: torch.rand(n, generator=g) * (self.cl["maxval"] / math.sqrt(self.k))
        # fill in chunks (keeps host memory bounded for multi-GB tables)
        rows_per = max(1, (1 << 24) // (self.num_fields * self.k))
        for s in range(0, self.num_features, rows_per):
            e = min(self.num_features, s + rows_per)
            chunk = init((e - s) * self.num_fields * self.k).view(e - s, self.num_fields, self.k)
            V[s:e, :, : self.k].copy_(chunk.to(dev))
        # the GPU block layouts hold each feature's FTRL {w, z, n} in the 16-B chunk after its slots
        lin = lin_record_views(V, G) if LIN_IN_BLOCK else None
        if lin is None:
            lin = tuple(torch.zeros(self.num_features, dtype=torch.float32, device=dev) for _ in range(3))
        self.state = dict(
            V=V,
            G=G,
            w=lin[0],
            wz=lin[1],
            wn=lin[2],
            bias=torch.zeros(4, dtype=torch.float32, device=dev),
        )
        self.touched = torch.zeros(self.num_features, dtype=torch.bool, device=dev)
        return self.state

    def adopt_state(self, st: dict) -> dict:
        """Checkpoint load (io/checkpoint.py): the saved tensors copied into this device's layout
        (per-slot feature blocks with the linear records on the GPU)."""
        self.num_features, self.num_fields = int(st["V"].shape[0]), int(st["V"].shape[1])
        self.state = {k: v.to(self.device) for k, v in st.items()}
        self.pack_state()
        return self.state

    # ------------------------------------------------------------------ data
    def prepare(self, features, labels=None) -> FFMBatch:
        """Rows of ``field:index[:value]`` strings -> device-resident padded-ELL batch.

        On the GPU the strings are parsed and hashed there (io/ingest.py: Arrow buffers ->
        pinned double-buffered H2D -> hm_ffm_parse); on the CPU by the host parser."""
        nf = self.num_features if self.num_features is not None else (1 << 24)
        nfld = self.num_fields if self.num_fields is not None else 1 << 15
        y = None
        if labels is not None:
            y = parse_labels_binary(labels) if self.hyper.classification else \
                np.asarray(labels, dtype=np.float32).reshape(-1)
        if self.device.type == "cuda":
            from ..io import ingest

            idx, fld, val = ingest.ffm_ell_device(features, nf, nfld,
                                                  hash_ints=self.cl["feature_hashing"] > 0,
                                                  device=self.device)[:3]
            if self.num_features is None:
                self.num_features = int(tmax(idx)) + 1 if idx.numel() else 1
            if self.num_fields is None:
                self.num_fields = int(tmax(fld)) + 1 if fld.numel() else 1
            yt = None if y is None else torch.from_numpy(y).to(self.device)
            return FFMBatch(idx, fld, val, yt)
        # (an Arrow list<string> column is parsed from its buffers by parse_ffm_rows)
        csr = parse_ffm_rows(features, nf, nfld, hash_ints=self.cl["feature_hashing"] > 0)
        if self.num_features is None:
            self.num_features = int(csr.idx.max()) + 1 if csr.nnz else 1
        if self.num_fields is None:
            self.num_fields = int(csr.fld.max()) + 1 if csr.nnz else 1
        return csr_to_ffm_batch(csr, y).to(self.device)

    def _ensure_state(self):
        if self.state is None:
            # data-parallel: the replicas of every rank must have one shape (each rank infers
            # the sizes from its own shard otherwise)
            self.init_state(*self.agree_max(self.num_features, self.num_fields))

    # ------------------------------------------------------------------ training
    def train_batch(self, b: FFMBatch, loss_buf: torch.Tensor | None = None) -> None:
        self._ensure_state()
        bs = int(self.cl["batch_size"])
        for k in range(self.dp_batches(b.n, bs)):
            s = min(b.n, k * bs)
            sub = b.slice(s, min(b.n, s + bs))
            lb = None if loss_buf is None else loss_buf[s:s + sub.n]
            # the first RAMP_ROWS rows of a learner: the atomic-update kernel (RAMP_VARIANT), or
            # RAMP_GRID blocks unless -grid is given — early in training every row moves the same
            # few parameters and concurrent read-modify-writes lose the most
            cut = min(sub.n, max(0, self.atomic_rows - self.rows_seen))
            for r0, r1, ramp in ((0, cut, True), (cut, sub.n, False)):
                if r1 <= r0:
                    continue
                part = sub if (r0, r1) == (0, sub.n) else sub.slice(r0, r1)
                grid = self.grid or (RAMP_GRID if ramp and RAMP_VARIANT < 0 else 0)
                ffm_step(self.state, part.idx, part.fld, part.val, part.y, self.hyper, train=True,
                         loss=None if lb is None else lb[r0:r1], grid=grid,
                         # (an explicit HM_FFM_VARIANT selects the kernel for every row)
                         variant=RAMP_VARIANT if ramp and RAMP_VARIANT >= 0 and _ffm_ops._VARIANT == 0 else None,
                         lin_mode=self.lin_mode())
            self.rows_seen += sub.n
            mi = int(self.cl["mix_interval"])
            if self.mixer is not None and mi > 0:
                if lb is not None and self._dp_power > DP_GUARD_POWER:
                    part_sum = torch.stack([lb[:sub.n].double().sum(),
                                            torch.tensor(float(sub.n), dtype=torch.float64, device=lb.device)])
                    self._mix_loss = part_sum if self._mix_loss is None else self._mix_loss + part_sum
                self._nbatches = getattr(self, "_nbatches", 0) + 1
                if self._nbatches % mi == 0:
                    self._dp_guard()
                    self.mix()
        self._mark_touched(b)

    def _mark_touched(self, b: FFMBatch) -> None:
        mark_touched(self.touched, b.idx, self.num_features)

    def mix(self) -> None:
        self.mix_tensors([self.state["V"], *linear_mix_tensors(self.state), self.state["bias"]],
                         [self.touched])

    def fit(self, features=None, labels=None, batch: FFMBatch | None = None) -> "FFMTrainer":
        b = batch if batch is not None else self.prepare(features, labels)
        self._ensure_state()
        loss_buf = torch.empty(b.n, dtype=torch.float32, device=self.device)
        iters = int(self.cl["iters"])
        for ep in self.epochs(iters, data=(b.idx, b.fld, b.val, b.y)):
            if ep == 0:
                eb = b
            else:  # per-epoch device-side shuffle (replaces rand_amplify / spill replay)
                # seeded per epoch, so a resumed run draws the same order as an uninterrupted one
                g = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + ep)
                perm = torch.randperm(b.n, generator=g).to(self.device)
                f = lambda t: None if t is None else t.index_select(0, perm).contiguous()
                eb = FFMBatch(f(b.idx), f(b.fld), f(b.val), f(b.y))
            self.train_batch(eb, loss_buf)
            if self.epoch_converged(float(loss_buf.double().sum().item()), rows=b.n):
                log.info("%s converged at epoch %d", self.NAME, ep + 1)
                break
        if self.mixer is not None:
            self.mix()
        return self

    # ------------------------------------------------------------------ inference
    def predict_raw(self, features=None, batch: FFMBatch | None = None) -> torch.Tensor:
        b = batch if batch is not None else self.prepare(features, None)
        self._ensure_state()
        out = torch.empty(b.n, dtype=torch.float32, device=self.device)
        bs = int(self.cl["batch_size"])
        for s in range(0, b.n, bs):
            sub = b.slice(s, min(b.n, s + bs))
            ffm_step(self.state, sub.idx, sub.fld, sub.val, None, self.hyper, train=False,
                     pred=out[s:s + sub.n])
        return out

    def predict(self, features=None, batch: FFMBatch | None = None) -> np.ndarray:
        p = self.predict_raw(features, batch)
        if self.hyper.classification:
            p = torch.sigmoid(p)
        return p.cpu().numpy()

    # ------------------------------------------------------------------ model table
    def model_table(self, model_id: str | None = None) -> pd.DataFrame:
        """Rows keyed as in :mod:`models.ffm_keys` (bias, linear, and V(feature, field))."""
        self._ensure_state()
        # a mixed data-parallel model is one model: same id on every rank
        mid = model_id or f"ffm-{0 if self._dp() else self.rank}"
        ids = torch.nonzero(self.touched).flatten()
        NF, F, k = self.num_features, self.num_fields, self.k
        V = self.state["V"][ids][:, :, :k].float().reshape(len(ids) * F, k).cpu().numpy()
        W = self.state["w"][ids].cpu().numpy()
        ids = ids.cpu().numpy().astype(np.int64)
        vkeys = (NF + ids[:, None] * F + np.arange(F)[None, :]).reshape(-1)
        n_lin = len(ids)
        n = 1 + n_lin + len(vkeys)
        # columnar build (tens of millions of rows at 2^20 features x 39 fields): model_id is a
        # one-category categorical, Vi an Arrow list<float> over the V buffer (NULL for the bias
        # and linear rows) — no per-row Python objects
        import pyarrow as pa

        offs = np.concatenate([np.zeros(1 + n_lin, np.int32),
                               np.arange(1, len(vkeys) + 1, dtype=np.int64).astype(np.int32) * k])
        offs = np.concatenate([[0], offs]).astype(np.int32)
        valid = np.concatenate([np.zeros(1 + n_lin, bool), np.ones(len(vkeys), bool)])
        vi = pa.ListArray.from_arrays(pa.array(offs), pa.array(V.reshape(-1).astype(np.float32)),
                                      mask=pa.array(~valid))
        return pd.DataFrame({
            "model_id": pd.Categorical.from_codes(np.zeros(n, np.int8), [mid]),
            "i": np.concatenate([[-1], ids, vkeys]).astype(np.int64),
            "Wi": np.concatenate([[float(self.state["bias"][0].item())], W,
                                  np.full(len(vkeys), np.nan)]).astype(np.float32),
            "Vi": pd.Series(vi, dtype=pd.ArrowDtype(vi.type))})

    def state_dict(self) -> dict:
        return {k: v.detach().cpu().contiguous() for k, v in (self.state or {}).items()} | {
            "meta": torch.tensor([self.num_features, self.num_fields, self.k, self.kp])}

    def load_state_dict(self, sd: dict) -> None:
        nf, nfld, k, kp = [int(x) for x in sd["meta"].tolist()]
        assert k == self.k, "factor mismatch"
        self.num_features, self.num_fields = nf, nfld
        self.state = {k2: v.to(self.device) for k2, v in sd.items() if k2 != "meta"}
        self.pack_state()
        self.touched = torch.ones(nf, dtype=torch.bool, device=self.device)

    def pack_state(self) -> None:
        """Bring loaded V/G tables into this trainer's layout: the AdaGrad accumulator form
        (per slot: a per-element G is summed over the factors — the per-slot accumulator IS the
        sum of the squared gradients of the slot's k factors; per element: a per-slot G is
        spread evenly) and, on the GPU, the packed / block layout."""
        st = self.state
        if st is None:
            return
        slot_g = not self.cl["elementwise_adagrad"]
        V, G = st["V"], st["G"]
        if slot_g and G.dim() == 3:
            G = G.to(torch.float32).sum(-1)
        elif not slot_g and G.dim() == 2:
            G = (G / self.kp).unsqueeze(-1).expand(*G.shape, self.kp).to(V.dtype)
        packed = self.device.type == "cuda" and not self.cl["split_state"]
        keep = G is st["G"] and (not packed or (_is_block(V, G) if slot_g else is_packed(V, G)))
        if not keep:
            NF, NFLD, kp = V.shape
            V2, G2 = new_state_tables(NF, NFLD, kp, V.dtype, V.device, packed=packed, slot_g=slot_g)
            V2.copy_(V)
            G2.copy_(G)
            st["V"], st["G"] = V2, G2
        # the linear FTRL state into the feature blocks' 16-B records (init_state's layout)
        lin = lin_record_views(st["V"], st["G"]) if LIN_IN_BLOCK and "w" in st else None
        if lin is not None and lin[0].data_ptr() != st["w"].data_ptr():
            for dst, key in zip(lin, ("w", "wz", "wn")):
                dst.copy_(st[key])
                st[key] = dst


def _is_block(V: torch.Tensor, G: torch.Tensor) -> bool:
    """Per-slot G in a GPU layout: V's feature blocks (ops.ffm.slot_block_layout) or the 16-B
    bf16 slots {V | G | 0}."""
    es = V.element_size()
    if G.dim() != 2 or not V.is_cuda:
        return False
    if G.stride(1) in (3, 4):
        return G.data_ptr() - V.data_ptr() == 8 and V.dtype == torch.bfloat16
    return 0 < G.data_ptr() - V.data_ptr() < V.stride(0) * es and G.stride(0) * 4 == V.stride(0) * es


def train_ffm(features, labels, options: str | None = None, device=None, **kw) -> pd.DataFrame:
    """Functional UDTF form: returns the model table."""
    t = FFMTrainer(options, device, **kw)
    t.fit(features, labels)
    return t.model_table()
