#!/bin/bash
# MF (explicit ratings, SGD and AdaGrad) Hogwild concurrency sweep on MI355X: ratings/s and
# held-out RMSE per launch grid on planted low-rank ML-20M-shaped ratings; plus the BPR
# default after the ROWS_PER_BLOCK change.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u - > gpurun_out/mf_grid.log 2>&1 <<'PY'
import json, sys, time
import numpy as np
import torch
sys.path.insert(0, "benchmarks")
from bench_configs import bench_bprmf
from hivemall_amd.io.synthetic import movielens_like
from hivemall_amd.models.mf import MatrixFactorization, MatrixFactorizationAdaGrad

print(json.dumps(bench_bprmf()), flush=True)
us, its = movielens_like(device="cuda", k=16)
g = torch.Generator(device="cuda").manual_seed(0)
P = torch.randn(138493, 8, device="cuda", generator=g) * 0.5
Q = torch.randn(27278, 8, device="cuda", generator=g) * 0.5
r = (3.5 + (P[us.long()] * Q[its.long()]).sum(1) + 0.3 * torch.randn(us.numel(), device="cuda", generator=g)).clamp(1, 5)
nt = 500000
for cls in (MatrixFactorization, MatrixFactorizationAdaGrad):
    for grid in (0, 212, 424, 848, 1696):
        m = cls(f"-factors 16 -iters 1 -mu 3.5 -eta0 0.01 -lambda 0.01" + (f" -grid {grid}" if grid else ""), device="cuda")
        m.fit(us[:-nt], its[:-nt], r[:-nt])           # warm-up epoch (also allocates)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(3):
            m.fit(us[:-nt], its[:-nt], r[:-nt])
        torch.cuda.synchronize(); dt = time.perf_counter() - t0
        pred = torch.as_tensor(m.predict(us[-nt:].cpu().numpy(), its[-nt:].cpu().numpy()), device="cuda")
        rmse = float(((pred - r[-nt:]) ** 2).mean().sqrt())
        print(json.dumps({"model": cls.NAME, "grid": m._grid(), "ratings_per_s": round(3 * (us.numel() - nt) / dt),
                          "heldout_rmse": round(rmse, 4)}), flush=True)
PY
echo done
