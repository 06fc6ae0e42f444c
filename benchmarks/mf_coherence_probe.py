"""does explicit MF on the GPU stop learning the factors above grid 1 because
of Hogwild staleness, or because plain loads hit the CU's non-coherent L1 (each CU keeps reading
its own stale copy of L1-resident factor rows while other CUs update them in L2)?

A/B on the same box: L1-bypassing agent-scope loads (default) vs plain loads
(HM_MF_PLAIN_LOADS=1), on (1) the 300-item test fixture at grids 1/2/3/9/36 with the convergence
test off, and (2) ML-20M-shaped planted ratings (k=8 planted, k=16 fitted) at the default grid
and wider, where the bias-only held-out RMSE is the reference level to beat.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import movielens_like  # noqa: E402
from hivemall_amd.models.mf import MatrixFactorization, MatrixFactorizationAdaGrad  # noqa: E402
from tests.test_mf import _ratings  # noqa: E402


def fixture():
    u, i, r = _ratings()
    for plain in ("0", "1"):
        os.environ["HM_MF_PLAIN_LOADS"] = plain
        for g in (1, 2, 3, 9, 36):
            m = MatrixFactorization(f"-factors 10 -eta0 0.01 -update_mean -disable_cv -iters 20 "
                                    f"-grid {g}", device="cuda").fit(u[:35000], i[:35000], r[:35000])
            pr = m.predict(u[35000:], i[35000:])
            print(json.dumps({"case": "fixture", "plain_loads": plain == "1", "grid": g,
                              "rmse": round(float(np.sqrt(((pr - r[35000:]) ** 2).mean())), 4),
                              "P_abs_mean": round(float(m.state["P"].abs().mean()), 4)}), flush=True)


def ml20m():
    us, its = movielens_like(device="cuda", k=16)
    g = torch.Generator(device="cuda").manual_seed(0)
    P = torch.randn(138493, 8, device="cuda", generator=g) * 0.5
    Q = torch.randn(27278, 8, device="cuda", generator=g) * 0.5
    r = (3.5 + (P[us.long()] * Q[its.long()]).sum(1)
         + 0.3 * torch.randn(us.numel(), device="cuda", generator=g)).clamp(1, 5)
    nt = 500000
    for plain in ("0", "1"):
        os.environ["HM_MF_PLAIN_LOADS"] = plain
        for cls in (MatrixFactorization, MatrixFactorizationAdaGrad):
            for grid in (0, 848):
                m = cls("-factors 16 -iters 1 -mu 3.5 -eta0 0.01 -lambda 0.01 -rankinit gaussian"
                        + (f" -grid {grid}" if grid else ""), device="cuda")
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(4):
                    m.fit(us[:-nt], its[:-nt], r[:-nt])
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                pred = torch.as_tensor(m.predict(us[-nt:].cpu().numpy(), its[-nt:].cpu().numpy()),
                                       device="cuda")
                rmse = float(((pred - r[-nt:]) ** 2).mean().sqrt())
                print(json.dumps({"case": "ml20m", "model": cls.NAME, "plain_loads": plain == "1",
                                  "grid": m._grid(), "epochs": 4,
                                  "ratings_per_s": round(4 * (us.numel() - nt) / dt),
                                  "heldout_rmse": round(rmse, 4)}), flush=True)
    # bias-only reference: user + item means
    rb = r[:-nt]
    mu = rb.mean()
    bu = torch.zeros(138493, device="cuda").index_add_(0, us[:-nt].long(), rb - mu)
    cu = torch.zeros(138493, device="cuda").index_add_(0, us[:-nt].long(), torch.ones_like(rb))
    bi = torch.zeros(27278, device="cuda").index_add_(0, its[:-nt].long(), rb - mu)
    ci = torch.zeros(27278, device="cuda").index_add_(0, its[:-nt].long(), torch.ones_like(rb))
    pb = mu + (bu / cu.clamp_min(1))[us[-nt:].long()] + (bi / ci.clamp_min(1))[its[-nt:].long()]
    print(json.dumps({"case": "ml20m", "model": "bias-only (user+item means)",
                      "heldout_rmse": round(float(((pb - r[-nt:]) ** 2).mean().sqrt()), 4)}),
          flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["fixture", "ml20m"]
    if "fixture" in which:
        fixture()
    if "ml20m" in which:
        ml20m()
