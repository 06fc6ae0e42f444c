"""Profiling and metrics.

* :class:`KernelTimer`  — HIP-event timing of a code region on the current stream
  (``with KernelTimer("ffm") as t: ...; t.ms``), host-sync free until read.
* :func:`rocprof_cmd`   — the ``rocprofv3`` command lines used for this repo's profiles
  (kernel trace + stats, or one PMC counter group per run — counters are never combined with
  the runtime/system traces).
* :func:`kernel_stats` / :func:`counter_summary` — parse rocprofv3's CSV output into
  per-kernel tables (what ``profiles/`` holds).
* :class:`MetricsWriter` — per-step JSONL metrics stream (rows/s, loss, bytes mixed, GB/s).
* :func:`host_trace`    — torch.profiler host + device timeline of a region, exported as a
  Chrome trace (``HM_TRACE=<dir>`` makes ``bench.py`` write one per rank) plus a per-op table.
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


class host_trace:
    """``with host_trace("out_dir", name="ffm"):`` — torch.profiler over CPU + GPU activity of
    the region; writes ``<out_dir>/<name>.rank<r>.json`` (chrome://tracing / Perfetto) and
    ``<name>.rank<r>.txt`` (the ``key_averages`` table sorted by device time).  A no-op when
    ``out_dir`` is empty, so call sites can pass ``os.environ.get("HM_TRACE")``."""

    def __init__(self, out_dir: str | None, name: str = "trace", rank: int = 0, row_limit: int = 30):
        self.out_dir, self.name, self.rank, self.row_limit = out_dir, name, rank, row_limit
        self.prof = None

    def __enter__(self):
        if not self.out_dir:
            return self
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(ProfilerActivity.CUDA)
        self.prof = profile(activities=acts, record_shapes=False)
        self.prof.__enter__()
        return self

    def __exit__(self, *exc):
        if self.prof is None:
            return False
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.prof.__exit__(*exc)
        os.makedirs(self.out_dir, exist_ok=True)
        base = os.path.join(self.out_dir, f"{self.name}.rank{self.rank}")
        self.prof.export_chrome_trace(base + ".json")
        key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
        try:
            table = self.prof.key_averages().table(sort_by=key, row_limit=self.row_limit)
        except Exception:  # pragma: no cover - sort key naming differs across versions
            table = self.prof.key_averages().table(row_limit=self.row_limit)
        with open(base + ".txt", "w") as f:
            f.write(table)
        return False
