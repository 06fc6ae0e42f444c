"""Host model of train_fm's Hogwild gap (round 6, CPU only): the early-training parity fixture of
tests/test_fm.py (200 K criteo_like rows, 2^18 features, k = 8, eta0 0.01) trained with W rows in
flight, each row's w / V writes landing as plain stores (lost when a concurrent row stored the same
feature) or as added deltas, per feature class (``probes/fm_hogwild_sim.cpp``).  Which part of the
state carries the gap to the sequential engine / the 8-mapper average?

    python benchmarks/fm_hogwild_sim.py --W 1024 --hot 0:32:5
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.fm import FMTrainer  # noqa: E402
from hivemall_amd.models.linear import SparseRows  # noqa: E402

SRC = os.path.join(ROOT, "benchmarks", "probes", "fm_hogwild_sim.cpp")
LIB = "/tmp/fm_hogwild_sim.so"


def rows_of(idx, y=None):
    n, F = idx.shape
    return SparseRows(torch.arange(0, n * F + 1, F, dtype=torch.int64), idx.reshape(-1).contiguous(), None, y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--W", type=int, default=1024)
    ap.add_argument("--modes", type=int, default=0)
    ap.add_argument("--hot", default="")
    ap.add_argument("--rows", type=int, default=200000)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    torch.set_num_threads(1)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["g++", "-O3", "-march=native", "-shared", "-fPIC", "-o", LIB, SRC])
    L = ctypes.CDLL(LIB)
    L.fm_hogwild_sim.restype = ctypes.c_int
    L.fm_hogwild_sim.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 6
    idx, y = criteo_like(a.rows, 18, seed=5)
    eidx, ey = criteo_like(20000, 18, seed=77)
    opts = "-c -factors 8 -num_features 262144 -eta0 0.01 -sigma 0.01"
    t = FMTrainer(opts, device="cpu")
    t._ensure(rows_of(idx, y))
    st = t.state
    dims, KP = st["V"].shape
    cnt = torch.bincount(idx.reshape(-1).long(), minlength=dims)
    order = torch.argsort(cnt, descending=True)
    mode = torch.full((dims,), a.modes, dtype=torch.uint8)
    for spec in filter(None, a.hot.split(",")):
        lo, hi, bits = (int(v) for v in spec.split(":"))
        mode[order[lo:hi]] = bits
    h = t.h
    ip = np.array([dims, t.k, KP, h.eta_kind, int(h.use_w0), a.W, idx.shape[1]], dtype=np.int32)
    hp = np.array([h.eta0, h.power_t, h.total_steps, h.lambda0, h.lambda_w, h.lambda_v], dtype=np.float32)
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    rc = L.fm_hogwild_sim(ip.ctypes.data, hp.ctypes.data, idx.shape[0], 0, p(idx.contiguous()), p(y.contiguous()),
                          p(mode), p(st["w"]), p(st["V"]), p(st["w0"]))
    assert rc == 0
    ll = torch.nn.functional.binary_cross_entropy_with_logits(t.predict_raw(rows=rows_of(eidx)), (ey > 0).float()).item()
    print(json.dumps({"W": a.W, "modes": a.modes, "hot": a.hot, "heldout": round(ll, 5), "tag": a.tag}), flush=True)


if __name__ == "__main__":
    main()
