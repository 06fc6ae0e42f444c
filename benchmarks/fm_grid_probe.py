"""train_fm at the config-2 shape (2M Criteo-1TB-shaped rows, 2^24 features, k=8, bf16 V):
rows/s and held-out logloss vs launch grid, with and without the per-row global-bias atomic
(use_w0), to locate the FM throughput limit."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.fm import FMTrainer  # noqa: E402
from hivemall_amd.models.linear import SparseRows  # noqa: E402

dev = torch.device("cuda")
n, bits = 2 * 1024 * 1024, 24
idx, y = criteo_like(n, bits, seed=5, device=dev)
rows = SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64, device=dev), idx.reshape(-1).contiguous(), None, y)
eidx, ey = criteo_like(200000, bits, seed=77, device=dev)
er = SparseRows(torch.arange(0, 200000 * 39 + 1, 39, dtype=torch.int64, device=dev), eidx.reshape(-1).contiguous(), None, None)
for w0 in (True, False):
    for grid in (int(g) for g in os.environ.get("FM_GRIDS", "64,128,256,512,1024").split(",")):
        t = FMTrainer(f"-c -factors 8 -num_features {1 << bits} -eta0 0.01 -sigma 0.01", device=dev)
        t.grid = grid
        t.h.use_w0 = w0
        t.fit(rows=rows)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.train_rows(rows)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ll = torch.nn.functional.binary_cross_entropy_with_logits(t.predict_raw(rows=er), (ey > 0).float()).item()
        print(json.dumps({"use_w0": w0, "grid": grid, "rows_per_s": round(n / dt), "logloss": round(ll, 5)}), flush=True)
