"""Common learner machinery (the LearnerBaseUDTF / UDTFWithOptions layer).

A learner is created from a Hivemall option string, consumes rows (the UDTF ``process``
calls, here batched), trains for ``-iters`` epochs with the ``ConversionState`` convergence
check, and emits its model table (the UDTF ``close``/``forwardModel``) as a pandas frame
with the upstream column layout.
"""
from __future__ import annotations

import logging
import math
import os
import time
from typing import Any

import numpy as np
import torch

from ..utils.options import Options, opt, flag

log = logging.getLogger("hivemall_amd")


def default_device() -> torch.device:
    env = os.environ.get("HM_DEVICE")
    if env:
        return torch.device(env)
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def resolve_device(device) -> torch.device:
    if device is None:
        return default_device()
    return torch.device(device)


class ConversionState:
    """Epoch-level convergence check (hivemall.common.ConversionState).

    Training stops when the relative decrease of the cumulative loss between two epochs is
    below ``cv_rate`` (default 0.005), unless ``-disable_cv``.
    """

    def __init__(self, check: bool = True, cv_rate: float = 0.005):
        self.check = check
        self.cv_rate = cv_rate
        self.prev = math.inf
        self.curr = 0.0
        self.epoch = 0
        self.history: list[float] = []

    def incr_loss(self, v: float) -> None:
        self.curr += float(v)

    def is_converged(self) -> bool:
        self.history.append(self.curr)
        converged = False
        if self.check and self.prev < math.inf and self.prev > 0:
            change = (self.prev - self.curr) / self.prev
            if 0 <= change < self.cv_rate:
                converged = True
        self.prev = self.curr
        self.curr = 0.0
        self.epoch += 1
        return converged


# per-epoch checkpoint / resume of a learner's epoch loop
CKPT_OPTS = [
    opt("checkpoint", "checkpoint_dir", None, str,
        "[engine] directory for per-epoch checkpoints; a rerun of the same query resumes after "
        "the newest epoch every rank completed (parallel.elastic.ResumableLoop)"),
    opt("checkpoint_every", None, 1, int, "[engine] epochs between checkpoints"),
]

COMMON_ITER_OPTS = [
    opt("iters", "iterations", 1, int, "The maximum number of iterations (epochs)", aliases=("iter",)),
    opt("cv_rate", "convergence_rate", 0.005, float, "Threshold to determine convergence"),
    flag("disable_cv", "disable_cvtest", "Whether to disable convergence check"),
    opt("seed", None, -1, int, "Seed value for random number generator"),
    opt("batch_size", None, 65536, int, "[engine] rows per device kernel launch"),
    opt("mix_interval", None, 0, int, "[engine] RCCL model-mix every N batches (0 = at end only)"),
    flag("mix_sparse", None, "[engine] mix only the rows touched since the last mix: all-gather "
         "of (index, delta) instead of a dense all-reduce (parallel.mix.SparseDeltaMixer)"),
] + CKPT_OPTS

# data-parallel mixing (+ checkpoint) options of the learners that do not take COMMON_ITER_OPTS
MIX_OPTS = [COMMON_ITER_OPTS[-4], COMMON_ITER_OPTS[-3]] + CKPT_OPTS


def parse_labels_binary(y) -> np.ndarray:
    """0/1 or -1/+1 labels -> float32 {-1,+1} (BinaryOnlineClassifierUDTF label handling)."""
    a = np.asarray(y, dtype=np.float32).reshape(-1)
    out = np.where(a > 0, 1.0, -1.0).astype(np.float32)
    return out


class Learner:
    """Base for all learners; subclasses define OPTIONS, NAME and the train loop."""

    NAME = "learner"
    OPTIONS: list = []
    # data parallelism of the SQL UDTF in a distributed session (functions._learner_udtf):
    # "shard" (rows split over the ranks + RCCL mixing), "union" (ensemble members split over the
    # ranks) or "replicate" (no data-parallel formulation: every rank trains on all rows)
    SQL_DP = "replicate"

    @classmethod
    def options(cls) -> Options:
        return Options(cls.OPTIONS, cls.NAME)

    def __init__(self, options: str | None = None, device=None, **kw: Any):
        self.options_str = options or ""
        self.cl = self.options().parse(options)
        self.device = resolve_device(device)
        try:
            self.seed = self.cl.get("seed")
        except KeyError:  # learners without a -seed option
            self.seed = None
        if self.seed is None or self.seed < 0:
            self.seed = 31
        self.mixer = kw.pop("mixer", None)
        self.rank = kw.pop("rank", 0)
        self.kw = kw

    def opt(self, name: str, default=None):
        return self.cl.get(name, default)

    # ------------------------------------------------------------------ data parallel
    def _dp(self) -> bool:
        return self.mixer is not None and self.mixer.world > 1

    def agree_max(self, *sizes: int) -> tuple[int, ...]:
        """The max of each size over the ranks (data-parallel replicas must share one shape:
        every rank sizes its tables from its own shard's largest id otherwise)."""
        if not self._dp():
            return tuple(int(s) for s in sizes)
        return tuple(int(self.mixer.all_reduce_scalar(float(s), "max")) for s in sizes)

    def dp_sum(self, x: float) -> float:
        """``x`` summed over the ranks (an epoch loss, a row count); ``x`` itself when not
        data-parallel."""
        return self.mixer.all_reduce_scalar(float(x), "sum") if self._dp() else float(x)

    def epoch_converged(self, loss: float, reduced: bool = False, rows: int | None = None) -> bool:
        """ConversionState step on the job-wide epoch loss: every rank takes the same
        break decision, so no rank leaves the epoch loop while another still calls the mixing
        collectives.  With ``HM_METRICS`` set, also appends the epoch's metrics record."""
        total = loss if reduced else self.dp_sum(loss)
        self.cv.incr_loss(total)
        self._log_epoch(total, rows)
        return self.cv.is_converged()

    # ------------------------------------------------------------------ checkpoint / resume
    def run_fingerprint(self, n: int, data=()) -> dict:
        """What identifies a training run for ``-checkpoint`` resume: the learner, its option
        string, the epoch count, the seed, the world size, the model table shapes and a digest of
        the training rows (sizes + a strided sample of each array)."""
        import hashlib

        import numpy as np

        h = hashlib.sha1()
        for t in data:
            if t is None:
                h.update(b"-")
                continue
            a = t.detach().reshape(-1) if isinstance(t, torch.Tensor) else torch.as_tensor(np.asarray(t)).reshape(-1)
            step = max(1, a.numel() // 4096)
            smp = a[::step][:4096].cpu().contiguous()
            h.update(f"{a.numel()}:{a.dtype}:".encode())
            h.update(smp.view(torch.uint8).numpy().tobytes() if smp.numel() else b"")
        state = getattr(self, "state", None)
        shapes = {}
        if isinstance(state, dict):
            shapes = {k: list(v.shape) for k, v in state.items() if isinstance(v, torch.Tensor)}
        world = self.mixer.world if self.mixer is not None else 1
        return {"learner": self.NAME, "options": self.options_str, "epochs": int(n),
                "seed": self.seed, "world": int(world), "tables": shapes, "data": h.hexdigest()}

    def no_checkpoint(self, engine: str) -> None:
        """Warn that ``-checkpoint`` is not honoured by ``engine`` (its loop state lives outside
        the learner), instead of silently ignoring the option."""
        try:
            ckpt = self.cl.get("checkpoint")
        except KeyError:
            ckpt = None
        if ckpt:
            log.warning("%s: -checkpoint is not supported by %s; training without checkpoints",
                        self.NAME, engine)

    def epochs(self, n: int, data=()):
        """The epoch indices of a training loop.  With ``-checkpoint <dir>`` the learner's whole
        state is saved after every ``-checkpoint_every`` epochs (per rank, atomically), and a
        rerun resumes after the newest epoch that every rank completed — the same rows and
        options replay bit-identically on the deterministic engines.  A checkpoint written by a
        different run (other options, rows ``data``, table shapes, seed or world size:
        :meth:`run_fingerprint`) is never resumed: training starts fresh and overwrites it.
        ``HM_FAULT=rank:epoch`` injects a crash before that epoch (parallel.elastic)."""
        try:
            ckpt = self.cl.get("checkpoint")
        except KeyError:
            ckpt = None
        if not ckpt:
            yield from range(n)
            return
        from ..parallel.elastic import ResumableLoop, maybe_inject_fault

        loop = ResumableLoop(self, ckpt, every=int(self.cl.get("checkpoint_every") or 1),
                             ctx=getattr(self.mixer, "ctx", None),
                             fingerprint=self.run_fingerprint(n, data))
        start = loop.resume(self.device)
        if start > 0:
            keep = {"mixer": self.mixer, "rank": self.rank, "kw": self.kw}
            self.__dict__.update(loop.learner.__dict__)
            self.__dict__.update(keep)
            loop.learner = self
            log.info("%s: resumed from %s after epoch %d", self.NAME, ckpt, start - 1)
        for ep in range(start, n):
            maybe_inject_fault(loop.rank, ep)
            yield ep
            if (ep + 1) % loop.every == 0 or ep + 1 == n:
                loop.save(ep)

    # ------------------------------------------------------------------ metrics stream
    @property
    def metrics(self):
        """``prof.MetricsWriter`` when ``HM_METRICS=<path>`` is set (SURVEY.md §5.5 per-step
        JSONL), else None; rank-tagged with the mixer's rank."""
        if not os.environ.get("HM_METRICS"):
            return None
        m = getattr(self, "_metrics", None)
        if m is None:
            from ..prof import MetricsWriter
            m = self._metrics = MetricsWriter(rank=getattr(self.mixer, "rank", self.rank))
            self._m_t = time.perf_counter()
            self._m_epoch, self._m_mix_s, self._m_mix_bytes, self._m_mixes = 0, 0.0, 0, 0
        return m

    def _log_epoch(self, loss: float, rows: int | None) -> None:
        m = self.metrics
        if m is None:
            return
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        dt, self._m_t = now - self._m_t, now
        self._m_epoch += 1
        rec = dict(learner=self.NAME, epoch=self._m_epoch, loss=float(loss), epoch_s=round(dt, 6),
                   mixes=self._m_mixes, mix_ms=round(self._m_mix_s * 1e3, 3),
                   mixed_bytes=self._m_mix_bytes)
        if rows:
            rec["rows"] = int(rows)
            rec["rows_per_s"] = round(rows / max(dt, 1e-9), 1)
        if self._m_mix_s > 0:
            rec["mix_GBps"] = round(self._m_mix_bytes / self._m_mix_s / 1e9, 3)
        m.log(**rec)
        self._m_mix_s, self._m_mix_bytes, self._m_mixes = 0.0, 0, 0

    def dp_batches(self, n: int, bs: int) -> int:
        """Launches for ``n`` rows in batches of ``bs``; data-parallel learners that mix every
        few batches agree on the max over ranks (a rank with fewer rows runs empty batches), so
        every rank reaches the same number of mix points."""
        nb = (n + bs - 1) // bs if n > 0 else 0
        if self._dp() and int(self.cl.get("mix_interval", 0) or 0) > 0:
            nb = self.agree_max(nb)[0]
        return nb

    def mix_tensors(self, tensors: list, flags: list = ()) -> None:
        """Average this rank's replica with the other ranks' (the ``GROUP BY feature
        avg(weight)`` / MixServer step): a dense bucketed all-reduce, or the
        touched-row all-gather with ``-mix_sparse``.  ``flags`` (bool "seen" masks) are OR-ed
        over ranks so every rank emits the same model table."""
        if not self._dp():
            return
        timed = self.metrics is not None
        if timed:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            t0 = time.perf_counter()
        if self.cl.get("mix_sparse", False):
            if getattr(self, "_sparse_mixer", None) is None:
                from ..parallel.mix import SparseDeltaMixer
                self._sparse_mixer = SparseDeltaMixer(self.mixer)
            self._sparse_mixer.mix(list(tensors))
        else:
            self.mixer.average(list(tensors))
        if flags:
            f = [m.to(torch.float32) for m in flags]
            self.mixer.all_reduce_sum(f)
            for m, v in zip(flags, f):
                m.copy_(v > 0)
        if timed:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self._m_mix_s += time.perf_counter() - t0
            self._m_mix_bytes += sum(t.numel() * t.element_size() for t in tensors)
            self._m_mixes += 1
