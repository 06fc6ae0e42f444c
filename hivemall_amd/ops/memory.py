"""Device tensors in memory of an explicit HIP coherence type (csrc/kernels/util.hip
hm_malloc_flags), for tables that many XCDs read-modify-write inside one kernel.

MI355X has 8 XCDs, each with its own L2.  Default (coarse-grained) allocations let an XCD's L2
keep a line it has read while another XCD updates the same line in memory, until the line is
evicted or the kernel ends.  Fine-grained memory keeps the XCDs' views coherent at a cost.
``fine_grained_zeros(shape, dtype, device)`` returns a torch tensor over such memory (zeroed),
freed when the tensor is collected."""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native

FLAGS = {"default": 0, "fine": 1, "uncached": 3}

_native.register_hip("hm_malloc_flags", [C.c_size_t, C.c_uint], restype=C.c_void_p)
_native.register_hip("hm_free", [C.c_void_p])


class _DevBuf:
    """A raw device allocation exposed through ``__cuda_array_interface__``."""

    def __init__(self, ptr: int, shape, typestr: str):
        self.ptr = ptr
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}

    def __del__(self):
        if self.ptr:
            _native.hip().hm_free(C.c_void_p(self.ptr))
            self.ptr = 0


def zeros(shape, dtype: torch.dtype, device, kind: str = "fine") -> torch.Tensor:
    """Zeroed tensor of ``shape`` / ``dtype`` on ``device`` in ``kind`` memory ("default",
    "fine", "uncached")."""
    dev = torch.device(device)
    assert dev.type == "cuda"
    n = 1
    for s in shape:
        n *= int(s)
    es = torch.empty(0, dtype=dtype).element_size()
    with torch.cuda.device(dev):
        ptr = _native.hip().hm_malloc_flags(C.c_size_t(max(1, n * es)), C.c_uint(FLAGS[kind]))
    if not ptr:
        raise MemoryError(f"hm_malloc_flags({n * es} B, {kind}) failed")
    # wrap the bytes as uint8, then view as the dtype (uint8's typestr is portable)
    buf = _DevBuf(ptr, (n * es,), "|u1")
    t = torch.as_tensor(buf, device=dev)
    t._hm_buf = buf                      # keep the allocation alive with the tensor
    return t.view(dtype).view(*shape)
