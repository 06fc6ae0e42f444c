#!/bin/bash
# round 6: explicit MF's grid (rule: 1 block per 32 items = 852 on ML-20M, the same grid BPR ran
# slow at): rate and held-out RMSE after 6 epochs at 852 / 1,024 / 2,048 blocks, SGD and AdaGrad
set -o pipefail
O=gpurun_out/r6bi
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python - > $O/mf_grid.jsonl 2> $O/mf_grid.err <<'PY' || { tail -5 $O/mf_grid.err; exit 1; }
import json, sys, time
import torch
sys.path.insert(0, ".")
from hivemall_amd.io.synthetic import movielens_like
from hivemall_amd.models.mf import MatrixFactorization, MatrixFactorizationAdaGrad
dev = torch.device("cuda")
us, its = movielens_like(device=dev, k=16)
g = torch.Generator(device=dev).manual_seed(0)
P = torch.randn(138493, 8, device=dev, generator=g) * 0.5
Q = torch.randn(27278, 8, device=dev, generator=g) * 0.5
r = (3.5 + (P[us.long()] * Q[its.long()]).sum(1) + 0.3 * torch.randn(us.numel(), device=dev, generator=g)).clamp(1, 5)
nt = 500000
for rep in range(2):
    for cls in (MatrixFactorization, MatrixFactorizationAdaGrad):
        for grid in (852, 1024, 2048):
            m = cls(f"-factors 16 -iters 1 -mu 3.5 -eta0 0.01 -lambda 0.01 -rankinit gaussian -grid {grid}", device=dev)
            tt = 0.0
            for ep in range(6):
                torch.cuda.synchronize(); t0 = time.perf_counter()
                m.fit(us[:-nt], its[:-nt], r[:-nt])
                torch.cuda.synchronize(); tt += time.perf_counter() - t0
            pred = torch.as_tensor(m.predict(us[-nt:].cpu().numpy(), its[-nt:].cpu().numpy()), device=dev)
            print(json.dumps({"model": cls.NAME, "grid": grid, "rep": rep, "ratings_per_s": round(6 * (us.numel() - nt) / tt),
                              "rmse": round(float(((pred - r[-nt:]) ** 2).mean().sqrt()), 4)}), flush=True)
PY
cat $O/mf_grid.jsonl
echo ok
