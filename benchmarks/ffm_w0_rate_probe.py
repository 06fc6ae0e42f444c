"""Rate of the fp32 FFM kernel with and without the global bias (-w0) at the bench's config
(criteo_ffm rows, 262,144 per step, 2^20 features, fp32 V + per-slot G).

    python benchmarks/ffm_w0_rate_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

dev = torch.device("cuda")
B, NRES = 262144, 4
idx, fld, val, y = criteo_ffm(B * NRES, 20, seed=3, device=dev)
for rep in range(2):
    for extra in ("", " -w0"):
        t = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 20" + extra, device=dev)
        t.init_state(1 << 20, 39)
        for i in range(4):
            s = (i % NRES) * B
            ffm_step(t.state, idx[s:s + B], fld[s:s + B], val[s:s + B], y[s:s + B], t.hyper)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 20
        for i in range(n):
            s = (i % NRES) * B
            ffm_step(t.state, idx[s:s + B], fld[s:s + B], val[s:s + B], y[s:s + B], t.hyper)
        torch.cuda.synchronize()
        print(json.dumps({"opts": extra.strip() or "default", "rep": rep,
                          "rows_per_s": round(B * n / (time.perf_counter() - t0) / 1e6, 2)}), flush=True)
