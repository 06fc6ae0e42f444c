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


_native.register_hip("hm_int_strlen", [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p])
_native.register_hip("hm_int_format", [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p])


def int_strings(ids: torch.Tensor):
    """Arrow string array of the decimal text of int ``ids`` (a model table's integer-named
    "feature" column).  CUDA tensors are formatted on the device (csrc/kernels/util.hip
    hm_int_strlen / hm_int_format: lengths, a scan, the digits, one D2H of the bytes), host
    tensors by pyarrow's cast."""
    import numpy as np
    import pyarrow as pa

    if not ids.is_cuda:
        return pa.array(ids.numpy().astype(np.int64)).cast(pa.string())
    v = ids.to(torch.int64).contiguous()
    n = v.numel()
    if n == 0:
        return pa.array([], type=pa.string())
    st = _native.stream_of(v.device)
    ln = torch.empty(n, dtype=torch.int32, device=v.device)
    _native.check(_native.hip().hm_int_strlen(v.data_ptr(), C.c_int64(n), ln.data_ptr(), st), "hm_int_strlen")
    off = torch.zeros(n + 1, dtype=torch.int32, device=v.device)
    torch.cumsum(ln, 0, dtype=torch.int32, out=off[1:])
    total = int(off[-1].item())
    out = torch.empty(max(1, total), dtype=torch.uint8, device=v.device)
    _native.check(_native.hip().hm_int_format(v.data_ptr(), C.c_int64(n), off.data_ptr(), out.data_ptr(), st),
                  "hm_int_format")
    ob, db = off.cpu().numpy(), out[:total].cpu().numpy()
    return pa.StringArray.from_buffers(n, pa.py_buffer(ob), pa.py_buffer(db))
