"""ctypes bindings to the in-tree native libraries (see ``_build.py``).

``hip()`` returns the gfx950 kernel library.  It is loaded *after* torch so that the HIP
runtime torch already mapped (soname ``libamdhip64.so.7``) is reused — one runtime per
process.  On a GPU box a missing or stale kernel library is an error, never a silent
fallback: ``require_hip()`` raises.

``host()`` returns the CPU data-plane library (hashing, parsing, CPU learner engine).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

from . import _build

_lock = threading.Lock()
_hip = None
_host = None

c_int = C.c_int
c_i32 = C.c_int32
c_i64 = C.c_int64
c_u32 = C.c_uint32
c_f32 = C.c_float
c_p = C.c_void_p


def _autobuild() -> bool:
    return os.environ.get("HM_NO_AUTOBUILD", "0") != "1"


def host():
    """Load (building if needed) the CPU native library."""
    global _host
    if _host is not None:
        return _host
    with _lock:
        if _host is None:
            if _autobuild():
                _build.build_host()
            lib = C.CDLL(str(_build.HOST_LIB))
            _check_build_id(lib, "host", _build.HOST_LIB)
            _declare_host(lib)
            _host = lib
    return _host


def hip():
    """Load (building if needed) the gfx950 kernel library."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            import torch  # noqa: F401  -- map torch's HIP runtime first

            if _autobuild():
                _build.build_hip()
            if not _build.HIP_LIB.exists():
                raise RuntimeError(f"HIP kernel library missing: {_build.HIP_LIB} (run build())")
            lib = C.CDLL(str(_build.HIP_LIB))
            _check_build_id(lib, "hip", _build.HIP_LIB)
            _declare_hip(lib)
            _hip = lib
    return _hip


BUILD_IDS: dict = {}   # kind -> source hash embedded in the loaded library


def _check_build_id(lib, kind: str, path) -> None:
    """The loaded library must have been built from the sources in this tree: its embedded
    hm_build_id() (the content hash of csrc + flags, _build.source_hash) must equal the hash of
    the sources here.  A library from another tree, or one whose sources changed without a
    rebuild, is an error (HM_SKIP_BUILD_ID=1 skips the check; so does an out-of-tree library
    chosen by HM_HIP_LIB / HM_HOST_LIB)."""
    fn = getattr(lib, "hm_build_id", None)
    got = None
    if fn is not None:
        fn.restype = C.c_char_p
        fn.argtypes = []
        got = fn().decode()
    BUILD_IDS[kind] = got
    in_tree = str(path) == str(_build.LIBDIR / ("libhm_hip.so" if kind == "hip" else "libhm_host.so"))
    if os.environ.get("HM_SKIP_BUILD_ID") == "1" or not in_tree:
        # an explicitly chosen library (HM_HIP_LIB / HM_HOST_LIB, e.g. the sanitizer build with
        # its own flags) is the caller's responsibility
        return
    want = _build.expected_hash(kind)
    if got != want:
        raise RuntimeError(f"{path}: built from other sources (build id {got}, this tree {want}); "
                           "rebuild with `python -m hivemall_amd._build`")


def hip_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"HIP kernel launch {what} failed: hipError_t={rc}")


def ptr(t) -> int:
    """Raw device/host pointer of a torch tensor or numpy array (None -> NULL)."""
    if t is None:
        return 0
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def stream_of(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def i32arr(vals):
    a = np.asarray(vals, dtype=np.int32)
    return a, a.ctypes.data


def f32arr(vals):
    a = np.asarray(vals, dtype=np.float32)
    return a, a.ctypes.data


# ------------------------------------------------------------------ declarations
_HIP_SIGS: dict[str, tuple] = {}
_HOST_SIGS: dict[str, tuple] = {
    "hm_murmur3": (c_u32, [c_p, c_int, c_u32]),
    "hm_murmur3_batch": (None, [c_p, c_p, c_i64, c_u32, c_p]),
    "hm_mhash_batch": (None, [c_p, c_p, c_i64, c_u32, c_i32, c_p]),
    "hm_feature_hash_strs": (c_i64, [c_p, c_p, c_i64, c_i32, c_u32, c_p, c_p]),
    "hm_list_append_str": (c_i64, [c_p, c_p, c_p, c_p, c_i64, c_p, c_i32, c_p, c_p, c_p]),
    "hm_format_feature_index": (c_i64, [c_p, c_p, c_p, c_i64, c_p, c_p]),
    "hm_normalize_features": (c_i64, [c_p, c_p, c_p, c_i64, c_int, c_p, c_p, c_p]),
    "hm_sigmoid_f64": (None, [c_p, c_i64, c_p]),
    "hm_oht_probe": (c_i64, [c_p, c_i64, c_p, c_i64, c_p, c_int]),
    "hm_oht_get_i64": (None, [c_p, c_p, c_i64, c_p, c_i64, c_i64, c_p]),
    "hm_join_ffm_rows_cpu": (None, [c_p] * 9 + [c_i64, c_int, c_p]),
    "hm_dict_new": (c_p, []),
    "hm_dict_free": (None, [c_p]),
    "hm_dict_size": (c_i64, [c_p]),
    "hm_dict_encode": (None, [c_p, c_p, c_p, c_i64, c_int, c_p]),
    "hm_dict_dump": (c_i64, [c_p, c_p, c_p]),
    "hm_parse_features": (c_i64, [c_p, c_p, c_i64, c_int, c_p, c_int, c_i32, c_u32, c_i64, c_p, c_p]),
    "hm_parse_ffm_features": (c_i64, [c_p, c_p, c_i64, c_i32, c_i32, c_int, c_u32, c_p, c_p, c_p]),
    "hm_ffm_schedule_slots": (c_i64, [c_p, c_int, c_int, c_p, c_int, c_int, c_int, c_int, c_p]),
}


def register_hip(name: str, argtypes: list, restype=c_int) -> None:
    _HIP_SIGS[name] = (restype, argtypes)
    if _hip is not None:
        _apply(_hip, {name: (restype, argtypes)})


def register_host(name: str, argtypes: list, restype=c_int) -> None:
    _HOST_SIGS[name] = (restype, argtypes)
    if _host is not None:
        _apply(_host, {name: (restype, argtypes)})


def _apply(lib, sigs):
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def _declare_host(lib):
    _apply(lib, _HOST_SIGS)


def _declare_hip(lib):
    _apply(lib, _HIP_SIGS)


# Kernel launchers: every one returns hipError_t and takes the stream last.
register_hip("hm_ffm_step", [c_p] * 16)
register_host("hm_ffm_step_cpu", [c_p] * 14)
