"""FM train/predict op: gfx950 kernel (``csrc/kernels/fm.hip``) on ``cuda`` tensors, sequential
C++ engine (``csrc/host/fm_cpu.cpp``) on CPU tensors."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import os

import numpy as np
import torch

from .. import _native


@dataclass
class FMHyper:
    eta0: float = 0.05
    power_t: float = 0.1
    total_steps: float = -1.0
    eta_kind: int = 2              # 0 fixed, 1 simple, 2 inverse
    lambda0: float = 0.01
    lambda_w: float = 0.01
    lambda_v: float = 0.01
    min_target: float = -3.4e38
    max_target: float = 3.4e38
    classification: bool = False
    use_w0: bool = True
    seed: int = 31


# rows between a wave's re-reads of the 64 global-bias shards (csrc/kernels/fm.hip fm_pipe_kernel);
# each re-read is 64 lines the other waves' atomics have just dropped from L2.  Measured on the
# Criteo-shaped 2^24 bench (profiles/r4/fm_w0_every_ab.log, two reps each): every row 145 M rows/s
# (held-out 0.4757), every 8 rows 234 M (0.4762), every 32 rows 300 M but 0.54-0.74 (the bias
# drifts between refreshes) -> 8.  Early in training the bias is far from its optimum and the
# delayed view turns the waves' bias steps into an overshoot (200 K rows, bf16 V: held-out 0.546
# vs 0.486 for the 8-mapper average), so a pass that starts within the first W0_WARM_ROWS rows of
# the stream re-reads every row.
# Round 5: HM_FM_W0_EVERY overrides the row bound, clamped to W0_EVERY_MAX, so the 32-row setting
# of the cliff above is not reachable.  An adaptive re-read (also re-read as soon as the wave's
# own bias steps since the last re-read add up to more than W0_TOL x eta) was measured and is off
# by default: on 3 M rows (2^20 features, bf16 V; benchmarks/fm_w0_probe.py,
# profiles/r5/fm_w0_probe.jsonl) held-out logloss vs the 8-mapper average is +2.87e-3 re-reading
# every row, +2.89e-3 every 8 rows after the warm rows, +3.5e-3 with tol 2 and +3.2e-3 with tol 0.5
# from row 0 — the bias schedule is not what separates the GPU from the mapper average there, and
# the adaptive rule alone from row 0 lost early (200 K rows fp32: 0.510 vs 0.486,
# profiles/r5/pytest_gpu_a.log).  The first W0_WARM_ROWS rows re-read every row.
W0_EVERY = 8
W0_EVERY_MAX = 16
W0_WARM_ROWS = 1 << 20
W0_TOL = float(os.environ.get("HM_FM_W0_TOL", "0"))


# w inside each feature's V record (new_state_tables): measured and not the default.  Config 2
# (2^24 features, k = 8, bf16), same box, 3 interleaved pairs (profiles/r5/fm_w_record_ab.log):
# 249-254 M rows/s vs 233-237 M (+7.5 %), but held-out 0.4773-0.4777 vs 0.4753-0.4759; against
# the 8-mapper average (benchmarks/fm_grid_parity_probe.py, grid 256, 3 reps) +4.0e-3 .. +4.5e-3
# vs +2.9e-3 .. +3.7e-3.  One line per feature instead of two stays longer in each XCD's L2, and
# the non-coherent L2s then serve older copies to the other XCDs (docs/perf_notes.md).
W_RECORD = os.environ.get("HM_FM_W_RECORD", "0") == "1"
# waves per launched workgroup (csrc/kernels/fm.hip launch): the grid's 4-wave workgroups
# (rows in flight / 4) are launched as 4 / WPB workgroups of WPB waves, so the 512 rows in flight
# of the default grid spread over all 256 CUs instead of 128.  Config 2, same box, 2 reps
# (profiles/r5/fm_wpb_ab.log): 1 wave 165.7-166.4 M rows/s, 2 waves 166.2-166.6 M, 4 waves
# 162.0-163.0 M; parity vs the 8-mapper average unchanged (+1.8e-3 .. +2.1e-3 vs +1.5e-3 .. +1.9e-3)
WPB = int(os.environ.get("HM_FM_WPB", "2"))


def new_state_tables(dims: int, KP: int, dtype: torch.dtype, device) -> tuple:
    """(w, V) for the GPU kernel.  Default: a separate w array and a contiguous V.  With
    HM_FM_W_RECORD=1 each feature's w lives in the padding of its V row (a 16-B aligned record
    {V[0..KP), w}), so a row's gather and its update store touch one line per feature instead of
    two; w is then a strided fp32 view and V a row-strided view, ordinary tensors to everything
    else (mixing, model tables, checkpoints)."""
    es = torch.empty(0, dtype=dtype).element_size()
    if not W_RECORD:
        return (torch.zeros(dims, dtype=torch.float32, device=device),
                torch.zeros((dims, KP), dtype=dtype, device=device))
    rec = (KP * es + 4 + 15) // 16 * 16                       # bytes per feature record
    buf = torch.zeros((dims, rec // 4), dtype=torch.float32, device=device)
    w = buf[:, KP * es // 4]
    V = buf.view(dtype)[:, :KP]
    return w, V


# Hot features' stores go out write-through (csrc/kernels/fm.hip P.hot): the per-XCD L2s are not
# coherent, and with plain stores each XCD kept training its own copy of the hottest lines.  Every
# store write-through (A/B variant 2) moved the grid-256 held-out gap vs Hivemall's 8-mapper average
# from +3.1e-3 .. +3.7e-3 to -3.2e-3 .. -3.1e-3 (one learner over all rows loses nothing) at 0.4x
# the rate (profiles/r6/fm_wt_parity.jsonl); a feature in at least HOT_FRAC of a batch's rows
# (sampled) is hot.  HM_FM_HOT_WT=0: plain stores everywhere (A/B).
HOT_FRAC = float(os.environ.get("HM_FM_HOT_FRAC", "0"))
# a hot feature's store goes out write-through on one row in HOT_EVERY (a power of two; per-row
# hash): the line is dropped from the writer's L2 that often, which bounds how many of its own
# XCD's updates a stale copy can absorb while the memory side serialises 1 / HOT_EVERY of them
HOT_EVERY = int(os.environ.get("HM_FM_HOT_EVERY", "1"))
HOT_WT = os.environ.get("HM_FM_HOT_WT", "1") != "0"
# waves on this many of the 8 XCDs (csrc/kernels/fm.hip P.xcds; 8 = all).  6 with the auto grid
# (256 workgroups there): +17 % on config 2 at the same parity as 8 XCDs at 128 (round 6,
# profiles/r6/fm_xcd/)
XCDS = 6
# ... except over a learner's first RAMP_ROWS rows (a launch that starts there), which run on ONE
# XCD at grid 128: early training is the most staleness-sensitive regime.  On the 200 K early
# rows of test_fm_gpu_logloss_parity vs the 8-mapper average (profiles/r6/fm_xcd/fm_ramp_*):
# 6 XCDs at 256 +0.0133; 8 XCDs at 128 +0.009 .. +0.0105 (fp32 / bf16); 2 XCDs at 128 +2.6e-3 ..
# +6.6e-3; 1 XCD at 128 +0.0 .. +1.4e-3 fp32, +4.3e-3 .. +4.4e-3 bf16 — at ~31 M rows/s, i.e.
# ~30 ms once per learner
RAMP_ROWS = int(os.environ.get("HM_FM_RAMP_ROWS", str(1 << 20)))
RAMP_GRID = int(os.environ.get("HM_FM_RAMP_GRID", "128"))
RAMP_XCDS = int(os.environ.get("HM_FM_RAMP_XCDS", "1"))


def hot_flags(state: dict, idx: torch.Tensor, n_rows: int, frac: float = None,
              buf: torch.Tensor | None = None) -> torch.Tensor | None:
    """uint8 [dims] flags of the features in >= ``frac`` of the rows, from a strided sample of the
    indices (written into ``buf`` when it fits, else a new tensor)."""
    V = state["V"]
    dims = V.shape[0]
    frac = HOT_FRAC if frac is None else frac
    if not (HOT_WT and V.is_cuda) or n_rows <= 0 or idx.numel() == 0 or frac <= 0:
        return None
    stride = 17 if idx.numel() >= (1 << 20) else 1     # prime: every field position is sampled
    ids = idx[::stride]
    ids = ids[(ids >= 0) & (ids < dims)].long()
    cnt = torch.bincount(ids, minlength=dims)
    thr = max(2.0, frac * n_rows / stride)
    hot = buf
    if hot is None or hot.numel() != dims or hot.device != V.device:
        hot = torch.zeros(dims, dtype=torch.uint8, device=V.device)
    torch.ge(cnt, thr, out=hot.view(torch.bool))
    return hot


def fm_step(state: dict, indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor | None,
            y: torch.Tensor | None, h: FMHyper, k: int, train: bool = True, t0: int = 0,
            pred: torch.Tensor | None = None, loss: torch.Tensor | None = None, grid: int = 0,
            hot: torch.Tensor | None = None) -> None:
    """One fused pass over CSR rows.  state: w f32 [dims], V bf16|f32 [dims, KP], w0 f32:
    on the GPU the global bias is the SUM of S = numel/32 shards at stride 32 floats (every
    row's update is an atomic add into shard (wave % S) instead of one contended address);
    the CPU engine keeps a single w0 (numel 1)."""
    w, V, w0 = state["w"], state["V"], state["w0"]
    dims, KP = V.shape
    n = indptr.numel() - 1
    dev = V.device
    for t in (indptr, idx, val, y, pred, loss):
        if t is not None:
            assert t.device == dev and t.is_contiguous(), "tensor device/layout mismatch"
    assert indptr.dtype == torch.int64 and idx.dtype == torch.int32
    if y is not None:
        assert y.dtype == torch.float32 and y.numel() >= n
    for t in (pred, loss):
        if t is not None:
            assert t.numel() >= n
    bf16 = V.dtype == torch.bfloat16
    xcds = int(os.environ.get("HM_FM_XCDS", str(XCDS)))
    if train and grid <= 0 and t0 < RAMP_ROWS and "HM_FM_XCDS" not in os.environ:
        xcds, grid = RAMP_XCDS, RAMP_GRID
    ip = np.array([dims, k, KP, int(h.classification), int(train), h.eta_kind, int(h.use_w0),
                   int(bf16), grid, h.seed & 0x7FFFFFFF, max(1, w0.numel() // 32),
                   int(os.environ.get("HM_FM_VARIANT", "0")),
                   max(1, min(W0_EVERY_MAX, int(os.environ.get(
                       "HM_FM_W0_EVERY", str(W0_EVERY if t0 >= W0_WARM_ROWS else 1))))),
                   V.stride(0), w.stride(0), WPB, max(1, HOT_EVERY) - 1,
                   xcds],
                  dtype=np.int32)
    assert V.stride(1) == 1 and V.stride(0) >= KP, "V rows must be contiguous"
    assert (dev.type == "cuda" and w0.numel() % 32 == 0 and w0.numel() // 32 <= 64) or w0.numel() == 1
    hp = np.array([h.eta0, h.power_t, h.total_steps, h.lambda0, h.lambda_w, h.lambda_v,
                   h.min_target, h.max_target, W0_TOL], dtype=np.float32)
    p = _native.ptr
    args = [ip.ctypes.data, hp.ctypes.data, C.c_int64(n), C.c_int64(t0), p(indptr), p(idx), p(val),
            p(y), p(w), p(V), p(w0), p(pred), p(loss)]
    if dev.type == "cuda":
        if hot is not None:
            assert hot.dtype == torch.uint8 and hot.numel() == dims and hot.device == dev
        rc = _native.hip().hm_fm_step(*args, p(hot if train else None), _native.stream_of(dev))
        _native.check(rc, "hm_fm_step")
    else:
        assert not bf16, "CPU FM engine keeps V in fp32"
        assert V.is_contiguous() and w.is_contiguous(), "CPU FM engine: contiguous w and V"
        rc = _native.host().hm_fm_step_cpu(*args)
        if rc != 0:
            raise RuntimeError(f"hm_fm_step_cpu failed: {rc}")


_P = _native.c_p
_native.register_hip("hm_fm_step", [_P, _P, _native.c_i64, _native.c_i64] + [_P] * 10 + [_P])
_native.register_host("hm_fm_step_cpu", [_P, _P, _native.c_i64, _native.c_i64] + [_P] * 9)
