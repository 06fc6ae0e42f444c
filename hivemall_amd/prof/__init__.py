"""Profiling and metrics.

* :class:`KernelTimer`  — HIP-event timing of a code region on the current stream
  (``with KernelTimer("ffm") as t: ...; t.ms``), host-sync free until read.
* :func:`rocprof_cmd`   — the ``rocprofv3`` command lines used for this repo's profiles
  (kernel trace + stats, or one PMC counter group per run — counters are never combined with
  the runtime/system traces).
* :func:`kernel_stats` / :func:`counter_summary` — parse rocprofv3's CSV output into
  per-kernel tables (what ``profiles/`` holds).
* :class:`MetricsWriter` — per-step JSONL metrics stream (rows/s, loss, bytes mixed, GB/s).
"""
from __future__ import annotations

import csv
import json
import os
import time
from collections import defaultdict

import torch


class KernelTimer:
    def __init__(self, name: str = "region", device=None):
        self.name = name
        self.device = device
        self._ms = None
        self.cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")

    def __enter__(self):
        if self.cuda:
            self.a = torch.cuda.Event(enable_timing=True)
            self.b = torch.cuda.Event(enable_timing=True)
            self.a.record()
        else:
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.cuda:
            self.b.record()
        else:
            self._ms = (time.perf_counter() - self.t0) * 1e3

    @property
    def ms(self) -> float:
        if self._ms is None and self.cuda:
            self.b.synchronize()
            self._ms = self.a.elapsed_time(self.b)
        return self._ms


COUNTER_GROUPS = [
    ["FETCH_SIZE"], ["WRITE_SIZE"],
    ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"],
    ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
    ["SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
]


def rocprof_cmd(out_dir: str, argv: list[str], counters: list[str] | None = None) -> list[str]:
    """rocprofv3 command: kernel trace + stats (counters None) or one PMC group."""
    base = ["rocprofv3", "--output-format", "csv", "-d", out_dir, "-o", "run"]
    if counters:
        base += ["--pmc", *counters]
    else:
        base += ["--kernel-trace", "--stats"]
    return base + ["--", *argv]


def kernel_stats(path: str) -> list[dict]:
    """Rows of ``*_kernel_stats.csv`` (Name, Calls, TotalDurationNs, AverageNs, Percentage)."""
    with open(path) as f:
        return [dict(r) for r in csv.DictReader(f)]


def counter_summary(paths: list[str], kernel_substr: str) -> dict:
    """Mean value per counter over the dispatches of the matching kernel."""
    acc = defaultdict(list)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                if kernel_substr in r["Kernel_Name"]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


class MetricsWriter:
    """Append-only JSONL metrics (one object per call), rank-tagged."""

    def __init__(self, path: str | None = None, rank: int = 0):
        self.path = path or os.environ.get("HM_METRICS")
        self.rank = rank
        self.t0 = time.time()

    def log(self, **kv) -> None:
        if not self.path:
            return
        rec = {"t": round(time.time() - self.t0, 6), "rank": self.rank}
        rec.update({k: (float(v) if isinstance(v, torch.Tensor) else v) for k, v in kv.items()})
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")
