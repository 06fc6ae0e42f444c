"""Model-table "seen" masks of the factorization learners (csrc/kernels/util.hip)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import _native

_native.register_hip("hm_mark_touched", [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p])


def mark_touched(flags: torch.Tensor, idx: torch.Tensor, dims: int) -> None:
    """flags[i] = True for every id i of ``idx`` with 0 <= i < dims (flags: bool [dims])."""
    assert flags.dtype == torch.bool and flags.device == idx.device
    if idx.numel() == 0:
        return
    if idx.is_cuda and idx.dtype == torch.int32 and flags.is_contiguous():
        i = idx.contiguous().reshape(-1)
        _native.check(_native.hip().hm_mark_touched(_native.ptr(i), C.c_int64(i.numel()), int(dims),
                                                     _native.ptr(flags), _native.stream_of(idx.device)),
                      "hm_mark_touched")
        return
    if not idx.is_cuda and flags.is_contiguous():
        a = idx.reshape(-1).numpy()
        f = flags.numpy()
        f[a[(a >= 0) & (a < dims)]] = True
        return
    i = idx.reshape(-1).long()
    flags[i[(i >= 0) & (i < dims)]] = True
