"""Fused join-predict reductions: gfx950 kernels
``csrc/kernels/join_predict.hip`` on a GPU session, numpy on a CPU session.

Inputs are the executor's resolved join/group (see ``sql/fused.py``): ``tm`` int32 [n] model row
of every exploded test row (-1 = no match), ``g`` int32 [n] group code, values ``v`` f32 [n],
model weights ``W`` f32 [R] (NaN = NULL) and, for FM, factors ``V`` f32 [R, k] with ``vmask``.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native

_P = _native.c_p
_native.register_hip("hm_join_dot", [_P, _P, _P, _P, _native.c_i64, _P, _P, _P])
_native.register_hip("hm_join_fm", [_P, _P, _P, _P, _P, _P, _native.c_i64, _native.c_int, _P, _P, _P, _P])
_native.register_hip("hm_join_ffm", [_P] * 10 + [_native.c_i64, _native.c_int, _P, _P])


def _dev(a: np.ndarray, dev) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=False)


def join_dot(tm, v, g, W, n_groups: int, device=None):
    """Per group: (sum of W[tm] * v over matched non-NULL products, their count)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda":
        p = _native.ptr
        t_tm, t_v, t_g, t_W = (_dev(tm, dev), _dev(v, dev), _dev(g, dev), _dev(W, dev))
        s = torch.zeros(n_groups, dtype=torch.float64, device=dev)
        c = torch.zeros(n_groups, dtype=torch.int32, device=dev)
        rc = _native.hip().hm_join_dot(p(t_tm), p(t_v), p(t_g), p(t_W), len(tm), p(s), p(c),
                                       _native.stream_of(dev))
        _native.check(rc, "hm_join_dot")
        return s.cpu().numpy(), c.cpu().numpy()
    ok = tm >= 0
    w = np.where(ok, W[np.where(ok, tm, 0)], np.nan).astype(np.float64)
    prod = w * v.astype(np.float64)
    good = ~np.isnan(prod)
    s = np.bincount(g[good], weights=prod[good], minlength=n_groups)
    c = np.bincount(g[good], minlength=n_groups).astype(np.int32)
    return s, c


def join_fm(tm, x, g, W, V, vmask, n_groups: int, device=None):
    """Per group: fm_predict = Σ W x + ½ Σ_f [(Σ V_f x)² − Σ (V_f x)²]."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    k = V.shape[1]
    if dev.type == "cuda":
        p = _native.ptr
        ts = [_dev(a, dev) for a in (tm, x, g, W, V, vmask.astype(np.uint8))]
        lin = torch.zeros(n_groups, dtype=torch.float64, device=dev)
        S = torch.zeros((n_groups, k), dtype=torch.float64, device=dev)
        Q = torch.zeros_like(S)
        rc = _native.hip().hm_join_fm(*[p(t) for t in ts], len(tm), k, p(lin), p(S), p(Q),
                                      _native.stream_of(dev))
        _native.check(rc, "hm_join_fm")
        return (lin + 0.5 * (S * S - Q).sum(1)).cpu().numpy()
    ok = tm >= 0
    r = np.where(ok, tm, 0)
    xd = x.astype(np.float64)
    w = W[r].astype(np.float64)
    lw = ok & ~np.isnan(w)
    lin = np.bincount(g[lw], weights=w[lw] * xd[lw], minlength=n_groups)
    vm = ok & vmask[r].astype(bool)
    vv = V[r[vm]].astype(np.float64) * xd[vm, None]
    S = np.zeros((n_groups, k))
    Q = np.zeros((n_groups, k))
    np.add.at(S, g[vm], vv)
    np.add.at(Q, g[vm], vv * vv)
    return lin + 0.5 * (S * S - Q).sum(1)


def join_ffm(ti, tj, xi, xj, g, W1, V1, m1, V2, m2, n_groups: int, device=None):
    """Per group: ffm_predict = Σ <V1[ti], V2[tj]> xi xj over rows with both V rows, plus
    Σ W1[ti] xi over the other matched rows (NaN W = NULL)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    k = V1.shape[1]
    if V2.shape[1] != k:
        raise ValueError("join_ffm: the two model tables disagree on k")
    if dev.type == "cuda":
        p = _native.ptr
        ts = [_dev(a, dev) for a in (ti, tj, xi, xj, g, W1, V1, m1.astype(np.uint8), V2, m2.astype(np.uint8))]
        out = torch.zeros(n_groups, dtype=torch.float64, device=dev)
        rc = _native.hip().hm_join_ffm(*[p(t) for t in ts], len(ti), k, p(out), _native.stream_of(dev))
        _native.check(rc, "hm_join_ffm")
        return out.cpu().numpy()
    c = lambda a, dt: np.ascontiguousarray(a, dtype=dt)   # noqa: E731
    ts = (c(ti, np.int32), c(tj, np.int32), c(xi, np.float32), c(xj, np.float32), c(W1, np.float32),
          c(V1, np.float32), c(m1, np.uint8), c(V2, np.float32), c(m2, np.uint8))
    val = np.empty(len(ti), dtype=np.float64)
    _native.host().hm_join_ffm_rows_cpu(*[t.ctypes.data for t in ts], len(ti), k, val.ctypes.data)
    return np.bincount(g, weights=val, minlength=n_groups)
