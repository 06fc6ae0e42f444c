"""Conflict-aware row order for the Hogwild FFM kernels (experiment).

``ffm_pipe_sg32_kernel`` (``csrc/kernels/ffm.hip``) runs block ``b`` over rows ``b, b + G,
b + 2G, ...`` (G = 8,192 blocks by default), with ~512 blocks resident on the 256 CUs.  To first
order, therefore, the rows whose read-modify-writes of the shared table overlap in time are the
512 consecutive indices ``p * G + g * 512 + [0, 512)`` of one *time slot* (generation
``g = b // 512``, position ``p``), and blocks ``b`` / ``b + 8`` share an XCD (round-robin
placement, MI355X_MICROARCH.md §Workgroup dispatch).  Which rows are in flight together is a
free choice of the batch's row order; these schedules choose it:

* ``none``   — stream order (the bench's default).
* ``spread`` — rows sharing a moderately hot feature (batch ranks 512 .. 8,192, the band the
  same-stream gap lives on: docs/perf_notes.md round 5) go to different time slots
  (``hm_ffm_schedule_slots``, greedy, C++).
* ``xcd``    — rows go to the XCD that owns most of their band features (features dealt to the
  8 XCDs by frequency), so a hot slot's read-modify-writes mostly stay inside one XCD's L2.

All return a permutation ``p`` of the batch (train on ``rows[p]``).  Offline (host) passes: the
measured outcome decides whether a device pass is worth building (docs/perf_notes.md round 6).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native

RESIDENT = 512          # blocks of the fp32 pipelined kernel resident at once (2 per CU)
GRID = 8192             # its default grid (csrc/kernels/ffm.hip default_blocks)
# feature frequency ranks of the band: 512 .. 8,192 carry ~85 % of the same-stream gap (float
# atomics on the top 512 took it from 2.30e-3 to 1.97e-3, on the top 8,192 to -4e-5: perf_notes)
BAND = (512, 8192)


def _band_ids(idx: np.ndarray, nf: int, band=None):
    c = np.bincount(idx.ravel()[idx.ravel() >= 0], minlength=nf)
    order = np.argsort(-c, kind="stable")
    lo, hi = BAND if band is None else band
    sel = order[lo:hi]
    sel = sel[c[sel] >= 2]
    bid = np.full(nf, -1, dtype=np.int32)
    bid[sel] = np.arange(sel.size, dtype=np.int32)
    return bid, sel, c


def slot_rows(B: int, grid: int = GRID, resident: int = RESIDENT) -> np.ndarray:
    """[S, resident] row indices of each time slot, in time order (S = B / resident)."""
    R = B // grid                       # rows per block
    gens = grid // resident
    t = np.arange(gens * R)
    g, p = t // R, t % R
    base = p * grid + g * resident
    return base[:, None] + np.arange(resident)[None, :]


def schedule_rows(idx: torch.Tensor, order: str, grid: int = GRID, resident: int = RESIDENT,
                  window: int = 0, nf: int | None = None, band=None) -> torch.Tensor:
    a = idx.cpu().numpy() if isinstance(idx, torch.Tensor) else np.asarray(idx)
    a = np.ascontiguousarray(a, dtype=np.int32)
    B, F = a.shape
    if order == "none":
        return torch.arange(B)
    nf = int(a.max()) + 1 if nf is None else nf
    if B % grid or grid % resident:
        raise ValueError(f"schedule needs B % grid == 0 and grid % resident == 0 ({B}, {grid}, {resident})")
    bid, sel, cnt = _band_ids(a, nf, band)
    if order == "spread":
        S = B // resident
        slot = np.empty(B, dtype=np.int32)
        lib = _native.host()
        kept = lib.hm_ffm_schedule_slots(a.ctypes.data, B, F, bid.ctypes.data, nf, int(sel.size), S,
                                         int(window), slot.ctypes.data)
        if kept < 0:
            raise RuntimeError("hm_ffm_schedule_slots failed")
        rows = slot_rows(B, grid, resident)          # [S, resident]
        perm = np.empty(B, dtype=np.int64)
        # rows of slot t in stream order -> the slot's indices
        o = np.argsort(slot, kind="stable")
        perm[rows.ravel()] = o
        return torch.from_numpy(perm)
    if order == "xcd":
        X = 8
        # deal band features to the XCDs by frequency (largest first onto the lightest XCD)
        load = np.zeros(X)
        grp = np.full(nf, -1, dtype=np.int64)
        for f in sel:
            x = int(np.argmin(load))
            grp[f] = x
            load[x] += cnt[f]
        g = grp[a]                                    # [B, F]
        w = np.where(g >= 0, cnt[a].astype(np.float64), 0.0)
        score = np.zeros((B, X))
        for x in range(X):
            score[:, x] = (w * (g == x)).sum(1)
        cap = np.full(X, B // X)
        pref = np.argsort(-score, axis=1)
        margin = np.sort(score, axis=1)[:, -1] - np.sort(score, axis=1)[:, -2]
        assign = np.empty(B, dtype=np.int64)
        for r in np.argsort(-margin, kind="stable"):
            for x in pref[r]:
                if cap[x] > 0:
                    cap[x] -= 1
                    assign[r] = x
                    break
        perm = np.empty(B, dtype=np.int64)
        for x in range(X):
            perm[x::X] = np.nonzero(assign == x)[0]
        return torch.from_numpy(perm)
    raise ValueError(f"unknown row order {order!r}")


def conflict_pairs(idx: torch.Tensor, perm: torch.Tensor, grid: int = GRID, resident: int = RESIDENT,
                   nf: int | None = None, band=None) -> dict:
    """Same-slot pairs of rows sharing a band feature under ``perm`` (the objective, for tables)."""
    a = (idx.cpu().numpy() if isinstance(idx, torch.Tensor) else np.asarray(idx))[np.asarray(perm)]
    B, F = a.shape
    nf = int(a.max()) + 1 if nf is None else nf
    bid, sel, _ = _band_ids(a, nf, band)
    rows = slot_rows(B, grid, resident)
    slot_of = np.empty(B, dtype=np.int64)
    slot_of[rows.ravel()] = np.repeat(np.arange(rows.shape[0]), resident)
    b = bid[a]
    m = b >= 0
    key = b[m].astype(np.int64) * rows.shape[0] + np.repeat(slot_of, F).reshape(B, F)[m]
    c = np.bincount(key)
    xk = b[m].astype(np.int64) * 8 + (np.repeat(np.arange(B) % 8, F).reshape(B, F)[m])
    cx = np.bincount(xk, minlength=sel.size * 8).reshape(-1, 8).astype(np.float64)
    tot = cx.sum(1)
    return {"same_slot_pairs": int((c * (c - 1) // 2).sum()),
            "xcd_share_max": float((cx.max(1) / np.maximum(tot, 1)).mean())}
