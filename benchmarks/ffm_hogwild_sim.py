"""Host model of the FFM headline's Hogwild gap (round 6, CPU only, no GPU minutes).

Replays bench.py's exact N = 1 stream (8 resident 262,144-row ``criteo_ffm`` batches, seed 1000,
cycled for warmup + steps; held-out rows seed 999,999) through ``probes/ffm_hogwild_sim.cpp``: W
rows in flight, each row reading the state W rows stale and its write landing as a plain store
(lost updates) or an added delta (atomic), chosen per feature class and per state part (V, G,
linear).  W = 1 is the sequential engine.  The point is attribution: which part of the state and
which features carry the +2e-3 same-stream gap the GPU measures, and how it moves with W.

    python benchmarks/ffm_hogwild_sim.py --W 1024 --modes 0 --steps 20 --warmup 5
    --hot A:B:bits  features of frequency rank [A, B) get mode bits (1 V, 2 G, 4 linear)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402

SRC = os.path.join(ROOT, "benchmarks", "probes", "ffm_hogwild_sim.cpp")
LIB = "/tmp/ffm_hogwild_sim.so"


def lib():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["g++", "-O3", "-march=native", "-shared", "-fPIC", "-o", LIB + ".tmp", SRC])
        os.replace(LIB + ".tmp", LIB)
    L = ctypes.CDLL(LIB)
    L.ffm_hogwild_sim.restype = ctypes.c_int
    L.ffm_hogwild_sim.argtypes = [ctypes.c_void_p] * 13
    return L


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def predict(st, idx, val, norm=True, chunk=8192):
    V, w, bias = st["V"], st["w"], st["bias"]
    out = torch.empty(idx.shape[0])
    F = idx.shape[1]
    iu = torch.triu_indices(F, F, 1)
    for s in range(0, idx.shape[0], chunk):
        i = idx[s:s + chunk].long()
        x = val[s:s + chunk]
        if norm:
            x = x / x.norm(dim=1, keepdim=True)
        Vs = V[i]                                  # [n, F(a), F(b), 4]: V[i_a, f_b]
        u = Vs[:, iu[0], iu[1]]                    # V[i_a, f_b]
        v = Vs[:, iu[1], iu[0]]                    # V[i_b, f_a]
        pair = ((u * v).sum(-1) * x[:, iu[0]] * x[:, iu[1]]).sum(1)
        out[s:s + chunk] = pair + (w[i] * x).sum(1) + bias[0]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--W", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--resident", type=int, default=8)
    ap.add_argument("--modes", type=int, default=0, help="mode bits of every feature")
    ap.add_argument("--hot", default="", help="A:B:bits[,A:B:bits]: frequency-rank ranges")
    ap.add_argument("--ramp-steps", type=int, default=1, help="steps at the start with every write atomic")
    ap.add_argument("--lin-delay", type=int, default=0, help="added linear steps land this many rows late")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    torch.set_num_threads(1)
    hb, F = 20, 39
    tr = FFMTrainer(f"-classification -factors 4 -feature_hashing {hb} -num_fields {F} -seed 31 "
                    f"-batch_size {a.batch}", device="cpu")
    tr.init_state(1 << hb, F)
    st = {k: v.contiguous().clone() for k, v in tr.state.items()}
    hp = np.ascontiguousarray(tr.hyper.hp()[:7], dtype=np.float32)
    idx, _, val, y = criteo_ffm(a.batch * a.resident, hb, seed=1000)
    NF = 1 << hb
    cnt = torch.bincount(idx[: a.batch].reshape(-1).long(), minlength=NF)
    order = torch.argsort(cnt, descending=True)
    mode = torch.full((NF,), a.modes, dtype=torch.uint8)
    for spec in filter(None, a.hot.split(",")):
        lo, hi, bits = (int(t) for t in spec.split(":"))
        mode[order[lo:hi]] = bits
    allm = torch.full((NF,), 7, dtype=torch.uint8)
    L = lib()
    t0 = time.time()
    losses = []
    for i in range(a.warmup + a.steps):
        s = (i % a.resident) * a.batch
        ip = np.array([a.batch, F, NF, a.W, int(tr.hyper.use_linear), int(tr.hyper.use_bias),
                       int(tr.hyper.norm), a.lin_delay], dtype=np.int32)
        lo = torch.empty(a.batch)
        m = allm if i < a.ramp_steps else mode
        L.ffm_hogwild_sim(ip.ctypes.data, hp.ctypes.data, ptr(idx[s:s + a.batch]), ptr(val[s:s + a.batch]),
                          ptr(y[s:s + a.batch]), ptr(m), ptr(st["V"]), ptr(st["G"]), ptr(st["w"]),
                          ptr(st["wz"]), ptr(st["wn"]), ptr(st["bias"]), ptr(lo))
        losses.append(float(lo.mean()))
    dt = time.time() - t0
    eidx, _, evl, ey, elogit = criteo_ffm(262144, hb, seed=999_999, return_logit=True)
    p = predict(st, eidx, evl, norm=bool(tr.hyper.norm))
    yy = (ey > 0).float()
    ll = torch.nn.functional.binary_cross_entropy_with_logits(p, yy).item()
    rec = {"W": a.W, "lin_delay": a.lin_delay, "modes": a.modes, "hot": a.hot, "ramp_steps": a.ramp_steps, "steps": a.steps,
           "warmup": a.warmup, "heldout": round(ll, 6), "train_loss_last": round(losses[-1], 5),
           "sim_s": round(dt, 1), "tag": a.tag}
    ref = json.load(open(os.path.join(ROOT, "resources", "bench_seq_ref.json"))).get(
        f"criteo_ffm/n1/s{a.steps}/w{a.warmup}/b{a.batch}/h{hb}/k4/r{a.resident}/e262144/onone")
    if ref:
        rec["gap_vs_seq"] = round(ll - ref["logloss_seq"], 6)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
