"""Explicit MF on the GPU: Hogwild with plain read-modify-write stores (concurrent updates of one
row overwrite each other) vs component-wise atomic delta adds (every update lands, reads stale),
on the ML-20M-shaped planted data of benchmarks/mf_coherence_probe.py and the small-catalogue
test fixture.  Held-out RMSE per epoch; compare with the sequential CPU engine
(benchmarks/mf_ml20m_cpu_ref.py).
    python benchmarks/mf_atomic_probe.py [fixture] [ml20m]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from hivemall_amd.io.synthetic import movielens_like  # noqa: E402
from hivemall_amd.models.mf import MatrixFactorization, MatrixFactorizationAdaGrad  # noqa: E402


def fixture():
    from tests.test_mf import _ratings

    u, i, r = _ratings()
    for atomic in ("0", "1", "2"):
        os.environ["HM_MF_ATOMIC"] = atomic
        for grid in (1, 2, 3, 9, 36):
            m = MatrixFactorization(f"-factors 10 -eta0 0.01 -update_mean -disable_cv -iters 20 -grid {grid}",
                                    device="cuda").fit(u[:35000], i[:35000], r[:35000])
            pr = np.asarray(m.predict(u[35000:], i[35000:]))
            print(json.dumps({"case": "fixture", "atomic": ["stores", "users+items", "items"][int(atomic)], "grid": grid, "epochs": 20,
                              "rmse": round(float(np.sqrt(((pr - r[35000:]) ** 2).mean())), 4)}), flush=True)


def ml20m(epochs=12):
    dev = torch.device("cuda")
    us, its = movielens_like(device=dev, k=16)
    g = torch.Generator(device=dev).manual_seed(0)
    P = torch.randn(138493, 8, device=dev, generator=g) * 0.5
    Q = torch.randn(27278, 8, device=dev, generator=g) * 0.5
    r = (3.5 + (P[us.long()] * Q[its.long()]).sum(1) + 0.3 * torch.randn(us.numel(), device=dev, generator=g)).clamp(1, 5)
    nt = 500000
    for cls in (MatrixFactorization, MatrixFactorizationAdaGrad):
        for atomic, grid in (("0", 0), ("1", 0), ("2", 0), ("2", 848)):
            os.environ["HM_MF_ATOMIC"] = atomic
            m = cls("-factors 16 -iters 1 -mu 3.5 -eta0 0.01 -lambda 0.01 -rankinit gaussian"
                    + (f" -grid {grid}" if grid else ""), device=dev)
            curve, tt = [], 0.0
            for ep in range(epochs):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                m.fit(us[:-nt], its[:-nt], r[:-nt])
                torch.cuda.synchronize()
                tt += time.perf_counter() - t0
                pred = torch.as_tensor(m.predict(us[-nt:].cpu().numpy(), its[-nt:].cpu().numpy()), device=dev)
                curve.append(round(float(((pred - r[-nt:]) ** 2).mean().sqrt()), 4))
            print(json.dumps({"case": "ml20m", "model": cls.NAME, "atomic": ["stores", "users+items", "items"][int(atomic)], "grid": m._grid(),
                              "ratings_per_s": round(epochs * (us.numel() - nt) / tt), "heldout_rmse_per_epoch": curve}),
                  flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["fixture", "ml20m"]
    if "fixture" in which:
        fixture()
    if "ml20m" in which:
        ml20m()
