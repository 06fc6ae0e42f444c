"""A/B of FFM kernel variants (state dtype x batched gathers x reload) on one GPU: rows/s."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

bits = 20
dev = torch.device("cuda")
B = 262144
idx, y = criteo_like(B * 4, bits, seed=3, device=dev)
for state in ("bf16", "fp32"):
    t = FFMTrainer(f"-c -factors 4 -num_fields 39 -feature_hashing {bits}" +
                   (" -bf16_state" if state == "bf16" else ""), device=dev)
    t.init_state(1 << bits, 39)
    for batched in (False, True):  # batched -> pair kernel (True) vs staged kernel (False)
        for reload in (True, False):
            t.hyper.reload = reload
            for i in range(3):
                ffm_step(t.state, idx[:B], None, None, y[:B], t.hyper)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 12
            for i in range(n):
                s = (i % 4) * B
                ffm_step(t.state, idx[s:s + B], None, None, y[s:s + B], t.hyper)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"state": state, "pairs": batched, "reload": reload,
                              "rows_per_s": round(B * n / dt), "ms_per_step": round(dt / n * 1e3, 3)}),
                  flush=True)
