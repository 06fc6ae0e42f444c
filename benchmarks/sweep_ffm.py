"""Sweep the FFM kernel launch geometry / batch on one GPU (rows/s per config)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

dev = torch.device("cuda")
bits = int(os.environ.get("BITS", "20"))
B = 262144
idx, y = criteo_like(B * 4, bits, seed=3, device=dev)
tr = FFMTrainer(f"-c -factors 4 -num_fields 39 -feature_hashing {bits}", device=dev)
tr.init_state(1 << bits, 39)
res = []
for grid, rl in [(g, r) for g in [0, 4096, 65536] for r in (0, 1)]:
    tr.hyper.reload = bool(rl)
    for _ in range(2):
        ffm_step(tr.state, idx[:B], None, None, y[:B], tr.hyper, grid=grid)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 8
    for i in range(n):
        s = (i % 4) * B
        ffm_step(tr.state, idx[s:s + B], None, None, y[s:s + B], tr.hyper, grid=grid)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res.append({"grid": grid, "reload": rl, "rows_per_s": B * n / dt, "ms_per_batch": dt / n * 1e3})
    print(json.dumps(res[-1]), flush=True)
# predict-only throughput
pred = torch.empty(B, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(8):
    ffm_step(tr.state, idx[:B], None, None, None, tr.hyper, train=False, pred=pred)
torch.cuda.synchronize()
print(json.dumps({"predict_rows_per_s": B * 8 / (time.perf_counter() - t0)}))
