"""Kernel rate of train_fm under non-default options (the config-2 bench runs only the default):
criteo_like rows, 2^22 features, one timed epoch of 2 M rows after a warm epoch.

    python benchmarks/fm_option_rate_sweep.py
"""
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
n, bits = 8 * 262144, 22
idx, y = criteo_like(n, bits, seed=5, device=dev)
rows = SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64, device=dev), idx.reshape(-1).contiguous(), None, y)
yr = SparseRows(rows.indptr, rows.idx, None, (y > 0).float())
cases = ["-c", "-c -fp32", "", "-c -adareg", "-c -factors 16", "-c -factors 4", "-c -eta fixed", "-c -factors 32"]
for extra in cases:
    t = FMTrainer(f"-factors 8 -num_features {1 << bits} -eta0 0.01 -sigma 0.01 {extra}".replace("-factors 8 -num", "-num")
                  if "-factors" in extra else f"-factors 8 -num_features {1 << bits} -eta0 0.01 -sigma 0.01 {extra}", device=dev)
    r = rows if "-c" in extra.split() else yr
    t.fit(rows=r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t.train_rows(r)
    torch.cuda.synchronize()
    print(json.dumps({"opts": extra or "(regression)", "rows_per_s": round(n / (time.perf_counter() - t0) / 1e6, 2)}), flush=True)
