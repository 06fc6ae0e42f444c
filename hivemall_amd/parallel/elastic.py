"""Failure detection, fault injection and checkpoint/resume for multi-rank training
(SURVEY.md §5.3-§5.4).

Upstream delegates failures to Hive/YARN (task retry from the split; ``-mix_cancel`` retracts
a dead attempt's MixServer contributions).  Here one job = one process per GPU, so:

* **detection** — every collective runs under the process group's timeout
  (``init_distributed(timeout_s=...)``); a dead or hung rank turns into an exception on the
  survivors instead of a silent hang;
* **recovery** — the launcher restarts the whole job (``torch.distributed.run --max-restarts``
  or any supervisor) and :class:`ResumableLoop` resumes every rank from the newest checkpoint
  step that *all* ranks completed (all-reduce MIN), so a replay is bit-identical to an
  uninterrupted run on the deterministic engines;
* **fault injection** — ``HM_FAULT="rank:step[:mode]"`` kills (``exit``) or raises in
  (``raise``) the given rank right before the given step: the test hook of
  ``tests/test_elastic.py``.
"""
from __future__ import annotations

import json
import logging
import os
import shutil

import torch

from ..io import checkpoint
from .dist import DistContext

log = logging.getLogger(__name__)


class InjectedFault(RuntimeError):
    pass


def maybe_inject_fault(rank: int, step: int) -> None:
    spec = os.environ.get("HM_FAULT")
    if not spec:
        return
    parts = spec.split(":")
    r, s = int(parts[0]), int(parts[1])
    mode = parts[2] if len(parts) > 2 else "exit"
    if r == rank and s == step:
        if mode == "raise":
            raise InjectedFault(f"injected fault at rank {rank} step {step}")
        os._exit(17)


class ResumableLoop:
    """Step loop with periodic per-rank checkpoints and consistent resume."""

    def __init__(self, learner, ckpt_dir: str, every: int = 1, ctx: DistContext | None = None,
                 keep: int = 2, fingerprint: dict | None = None):
        self.learner = learner
        self.dir = ckpt_dir
        self.every = max(1, int(every))
        self.ctx = ctx
        self.keep = keep
        # identity of the run (learner options, data digest, shapes, seed, world): a checkpoint
        # whose recorded fingerprint differs belongs to another run and is not resumed
        self.fingerprint = fingerprint
        self.rank = ctx.rank if ctx is not None else 0
        self.rank_dir = os.path.join(ckpt_dir, f"rank{self.rank}")
        os.makedirs(self.rank_dir, exist_ok=True)

    def _latest_local(self) -> int:
        p = os.path.join(self.rank_dir, "latest.json")
        if not os.path.exists(p):
            return -1
        with open(p) as f:
            meta = json.load(f)
        if self.fingerprint is not None and meta.get("fingerprint") != self.fingerprint:
            log.warning("checkpoint %s was written by a different run (options, rows, shapes, "
                        "seed or world size differ): starting fresh", self.rank_dir)
            return -1
        return int(meta["step"])

    def _agree(self, step: int) -> int:
        if self.ctx is None or not self.ctx.is_dist:
            return step
        t = torch.tensor([step], dtype=torch.int64, device=self.ctx.device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
        return int(t.item())

    def resume(self, device=None) -> int:
        """Load the newest step every rank has; returns the next step to run (0 = fresh)."""
        step = self._agree(self._latest_local())
        if step < 0:
            return 0
        path = os.path.join(self.rank_dir, f"step{step}")
        mixer, rank = getattr(self.learner, "mixer", None), getattr(self.learner, "rank", 0)
        self.learner = checkpoint.load(path, device=device or self.learner.device, restore_rng=True,
                                       mixer=mixer, rank=rank)
        return step + 1

    def save(self, step: int) -> None:
        path = os.path.join(self.rank_dir, f"step{step}")
        checkpoint.save(self.learner, path, model_table=False)
        tmp = os.path.join(self.rank_dir, "latest.json.tmp")
        with open(tmp, "w") as f:
            json.dump({"step": step, "fingerprint": self.fingerprint}, f)
        os.replace(tmp, os.path.join(self.rank_dir, "latest.json"))
        steps = sorted(int(d[4:]) for d in os.listdir(self.rank_dir) if d.startswith("step"))
        for s in steps[:-self.keep]:
            shutil.rmtree(os.path.join(self.rank_dir, f"step{s}"), ignore_errors=True)

    def run(self, n_steps: int, step_fn, device=None):
        start = self.resume(device)
        for step in range(start, n_steps):
            maybe_inject_fault(self.rank, step)
            step_fn(self.learner, step)
            if (step + 1) % self.every == 0 or step + 1 == n_steps:
                self.save(step)
        return self.learner
