"""Checkpoint / resume of any learner.

Upstream the model table *is* the checkpoint (plus ``-loadmodel`` warm start); multi-epoch
state lives in a task-local spill file and is not resumable.  Here a checkpoint directory holds

* ``model.parquet``  — the learner's model table (Hivemall layout; loadable by SQL / -loadmodel),
* ``state.pt``       — every device tensor of the learner (weights *and* optimizer state:
                       AdaGrad G, FTRL z/n, Adam moments, covariances, touched masks, replica
                       scalars), saved with ``torch.save`` and read back with
                       ``torch.load(weights_only=True)`` (tensors and primitives only),
* ``meta.json``      — learner class, option string, counters (step t, rows seen, epoch,
                       convergence history), label / vocabulary encoders and the RNG cursor.

``save(learner, dir)`` / ``load(dir, device)`` round-trip bit-exactly; writes are atomic
(temp directory + rename) so a rank killed mid-write never leaves a torn checkpoint.
"""
from __future__ import annotations

import dataclasses
import importlib
import glob
import json
import os
import shutil
import tempfile
import time

import numpy as np
import torch

_SCALARS = ("t", "rows_seen", "num_features", "num_fields", "dims", "n_users", "n_items", "labels",
            "classes", "k", "kp", "grid", "K", "dp_power", "dp_guard_tripped")


def _collect_tensors(learner) -> dict:
    out = {}
    st = getattr(learner, "state", None)
    if isinstance(st, dict):
        for k, v in st.items():
            if torch.is_tensor(v):
                out[f"state.{k}"] = v
    elif dataclasses.is_dataclass(st):
        for f in dataclasses.fields(st):
            v = getattr(st, f.name)
            if torch.is_tensor(v):
                out[f"state.{f.name}"] = v
    for k, v in vars(learner).items():
        if torch.is_tensor(v) and not k.startswith("_"):
            out[f"attr.{k}"] = v
    return out


def _encoder_meta(enc):
    if enc is None:
        return None
    return {"mode": enc.mode, "num_features": enc.num_features, "seed": enc.seed,
            "int_base": enc.int_base, "vocab": enc.vocab() if enc.mode in ("dict", "auto") else [],
            "string_names": bool(getattr(enc, "string_names", False))}


def _restore_encoder(m):
    if m is None:
        return None
    from ..utils.features import FeatureEncoder
    enc = FeatureEncoder(m["mode"], m["num_features"], m["int_base"], m["seed"])
    enc.string_names = m.get("string_names", False)
    if m["vocab"]:
        enc.encode([m["vocab"]], add_new=True)
    return enc


def _jsonable(v):
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    return v


def save(learner, path: str, model_table: bool = True) -> str:
    parent = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(parent, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix=".ckpt-", dir=parent)
    try:
        tensors = {k: v.detach().cpu() for k, v in _collect_tensors(learner).items()}
        torch.save(tensors, os.path.join(tmp, "state.pt"))
        st = getattr(learner, "state", None)
        meta = {
            "class": f"{type(learner).__module__}:{type(learner).__qualname__}",
            "name": getattr(learner, "NAME", None),
            "options": getattr(learner, "options_str", ""),
            "scalars": {k: _jsonable(getattr(learner, k)) for k in _SCALARS
                        if hasattr(learner, k) and isinstance(getattr(learner, k), (int, float, str, list, tuple, type(None), np.integer, np.floating))},
            "state_kind": "dataclass" if dataclasses.is_dataclass(st) else ("dict" if isinstance(st, dict) else None),
            # JSON scalars only: tensors kept in meta are scratch buffers the engines rebuild
            # (ops/linear.py train_pass_minibatch), caches (the hot set) are recomputed
            "state_meta": ({k: v for k, v in st.meta.items() if isinstance(v, (bool, int, float, str))}
                           if dataclasses.is_dataclass(st) and hasattr(st, "meta") else None),
            "state_covar": bool(getattr(st, "covar", False)) if dataclasses.is_dataclass(st) else None,
            "encoder": _encoder_meta(getattr(learner, "encoder", None)),
            "cv": vars(learner.cv) if hasattr(learner, "cv") else None,
            "hyper": dataclasses.asdict(learner.hyper) if dataclasses.is_dataclass(getattr(learner, "hyper", None)) else None,
            "torch_rng": torch.get_rng_state().tolist(),
            "saved_ns": time.time_ns(),       # orders checkpoints (the .old-* fallback)
        }
        with open(os.path.join(tmp, "meta.json"), "w") as f:
            json.dump(meta, f, default=lambda o: None)
        if model_table and hasattr(learner, "model_table"):
            try:
                from .model_table import write_table
                write_table(learner.model_table(), os.path.join(tmp, "model.parquet"))
            except Exception:  # pragma: no cover - the tensors are the authoritative state
                pass
        for name in os.listdir(tmp):
            _fsync_file(os.path.join(tmp, name))
        _fsync_dir(tmp)
        # swap: the old checkpoint is renamed aside (never deleted first), the new one moved in,
        # the parent directory synced, and only then the old one removed — a crash at any point
        # leaves a complete checkpoint at ``path`` or at ``path``.old-*
        old = None
        if os.path.exists(path):
            old = tempfile.mkdtemp(prefix=os.path.basename(path) + ".old-", dir=parent)
            os.rmdir(old)
            os.replace(path, old)
        os.replace(tmp, path)
        _fsync_dir(parent)
        if old is not None:
            shutil.rmtree(old, ignore_errors=True)
        # a crash between the final rename and this cleanup in an EARLIER save left a stale
        # .old-* behind: ``path`` is complete now, so none of them is needed any more
        for stale in glob.glob(glob.escape(path.rstrip("/")) + ".old-*"):
            shutil.rmtree(stale, ignore_errors=True)
    except BaseException:
        shutil.rmtree(tmp, ignore_errors=True)
        raise
    return path


def _fsync_file(p: str) -> None:
    if os.path.isfile(p):
        fd = os.open(p, os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)


def _fsync_dir(d: str) -> None:
    try:
        fd = os.open(d, os.O_RDONLY)
    except OSError:  # pragma: no cover - platforms without directory fds
        return
    try:
        os.fsync(fd)
    except OSError:  # pragma: no cover
        pass
    finally:
        os.close(fd)


def load(path: str, device=None, restore_rng: bool = False, **kw):
    """Rebuild a learner from ``save``.  ``restore_rng``: also restore the process-global torch
    CPU RNG to its state at save time (off by default: loading must not reseed the caller)."""
    if not os.path.exists(os.path.join(path, "meta.json")):
        # a crash between the two renames of save(): take the newest complete .old-* (by the
        # save time written into its meta; the mkdtemp suffixes are random, not ordered)
        best = None
        for cand in glob.glob(glob.escape(path.rstrip("/")) + ".old-*"):
            try:
                with open(os.path.join(cand, "meta.json")) as f:
                    t = json.load(f).get("saved_ns") or os.path.getmtime(os.path.join(cand, "meta.json"))
            except (OSError, ValueError):
                continue
            if best is None or t > best[0]:
                best = (t, cand)
        if best is not None:
            path = best[1]
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    mod, qual = meta["class"].split(":")
    m = importlib.import_module(mod)
    try:
        cls = m
        for part in qual.split("."):
            cls = getattr(cls, part)
    except AttributeError:  # classes generated per SQL function (models.linear.LEARNERS)
        cls = getattr(m, "LEARNERS")[meta["name"]]
    learner = cls(meta["options"] or None, device=device, **kw)
    tensors = torch.load(os.path.join(path, "state.pt"), weights_only=True)
    dev = learner.device
    for k, v in meta["scalars"].items():
        setattr(learner, k, v)
    kind = meta["state_kind"]
    st_t = {k[6:]: v.to(dev) for k, v in tensors.items() if k.startswith("state.")}
    if kind == "dict":
        # learners whose device state lives in a layout of views into one table (FFM's feature
        # blocks, FM's V records) rebuild that layout and copy the saved values in: torch.save of
        # each view on its own wrote plain contiguous tensors, which would otherwise send the
        # resumed learner down the generic kernels
        if hasattr(learner, "adopt_state"):
            learner.adopt_state(st_t)
        else:
            learner.state = st_t
    elif kind == "dataclass":
        from ..ops.linear import LinearState
        learner.state = LinearState(st_t["S"], st_t["touched"], st_t["RS"], bool(meta["state_covar"]),
                                    st_t.get("gacc"), st_t.get("tlist"), meta.get("state_meta") or {})
    for k, v in tensors.items():
        if k.startswith("attr."):
            setattr(learner, k[5:], v.to(dev))
    if meta.get("encoder") is not None:
        learner.encoder = _restore_encoder(meta["encoder"])
    if meta.get("cv") is not None and hasattr(learner, "cv"):
        for k, v in meta["cv"].items():
            setattr(learner.cv, k, v if v is not None else float("inf"))
    if meta.get("hyper") is not None and hasattr(learner, "hyper"):
        for k, v in meta["hyper"].items():
            setattr(learner.hyper, k, v)
    if getattr(learner, "labels", None) is not None and hasattr(learner, "P"):
        learner.P.n_labels = len(learner.labels)
    if restore_rng:
        torch.set_rng_state(torch.tensor(meta["torch_rng"], dtype=torch.uint8))
    return learner
