"""Sequential CPU reference for the ML-20M-shaped explicit-MF probe (benchmarks/mf_coherence_probe.py
ml20m case): the same planted data shape and options, trained by the C++ sequential engine, to
separate "the GPU's Hogwild schedule loses the factors" from "4 epochs at -eta0 0.01 do not leave
the near-zero init on this data".  Prints held-out RMSE per epoch and the bias-only level.
    python benchmarks/mf_ml20m_cpu_ref.py [--epochs 4] [--device cpu]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from hivemall_amd.io.synthetic import movielens_like  # noqa: E402
from hivemall_amd.models.mf import MatrixFactorization, MatrixFactorizationAdaGrad  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--opts", default="-factors 16 -iters 1 -mu 3.5 -eta0 0.01 -lambda 0.01 -rankinit gaussian")
    ap.add_argument("--model", default="sgd")
    a = ap.parse_args()
    dev = torch.device(a.device)
    us, its = movielens_like(device=dev, k=16)
    g = torch.Generator(device=dev).manual_seed(0)
    P = torch.randn(138493, 8, device=dev, generator=g) * 0.5
    Q = torch.randn(27278, 8, device=dev, generator=g) * 0.5
    r = (3.5 + (P[us.long()] * Q[its.long()]).sum(1) + 0.3 * torch.randn(us.numel(), device=dev, generator=g)).clamp(1, 5)
    nt = 500000
    cls = MatrixFactorization if a.model == "sgd" else MatrixFactorizationAdaGrad
    m = cls(a.opts, device=dev)
    for ep in range(a.epochs):
        t0 = time.perf_counter()
        m.fit(us[:-nt], its[:-nt], r[:-nt])
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        pred = torch.as_tensor(m.predict(us[-nt:].cpu().numpy(), its[-nt:].cpu().numpy()), device=dev)
        rmse = float(((pred - r[-nt:]) ** 2).mean().sqrt())
        print(json.dumps({"case": "ml20m", "model": cls.NAME, "device": a.device, "opts": a.opts, "epoch": ep + 1,
                          "ratings_per_s": round((us.numel() - nt) / dt), "heldout_rmse": round(rmse, 4)}), flush=True)
    rb = r[:-nt]
    mu = rb.mean()
    bu = torch.zeros(138493, device=dev).index_add_(0, us[:-nt].long(), rb - mu)
    cu = torch.zeros(138493, device=dev).index_add_(0, us[:-nt].long(), torch.ones_like(rb))
    bi = torch.zeros(27278, device=dev).index_add_(0, its[:-nt].long(), rb - mu)
    ci = torch.zeros(27278, device=dev).index_add_(0, its[:-nt].long(), torch.ones_like(rb))
    pb = mu + (bu / cu.clamp_min(1))[us[-nt:].long()] + (bi / ci.clamp_min(1))[its[-nt:].long()]
    print(json.dumps({"case": "ml20m", "model": "bias-only (user+item means)",
                      "heldout_rmse": round(float(((pb - r[-nt:]) ** 2).mean().sqrt()), 4)}), flush=True)


if __name__ == "__main__":
    main()
