"""FFM: fp32 vs bf16 (stochastic-rounded) V/G state — throughput and logloss."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

bits = 20
dev = torch.device("cuda")
idx, y = criteo_like(500000, bits, seed=5)
eidx, ey = criteo_like(100000, bits, seed=99)
yy = (ey > 0).float()
B = 262144
bidx, by = criteo_like(B * 4, bits, seed=3, device=dev)
for extra in ("", " -bf16_state"):
    for reload in (True, False):
        t = FFMTrainer(f"-c -factors 4 -num_fields 39 -feature_hashing {bits} -seed 1" + extra, device=dev)
        t.hyper.reload = reload
        t.fit(batch=FFMBatch(idx, None, None, y).to(dev))
        p = t.predict_raw(batch=FFMBatch(eidx, None, None, None).to(dev)).cpu()
        ll = torch.nn.functional.binary_cross_entropy_with_logits(p, yy).item()
        for i in range(2):
            ffm_step(t.state, bidx[:B], None, None, by[:B], t.hyper)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(8):
            s = (i % 4) * B
            ffm_step(t.state, bidx[s:s + B], None, None, by[s:s + B], t.hyper)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"state": "bf16" if extra else "fp32", "reload": reload, "logloss_500k": round(ll, 5),
                          "rows_per_s": round(B * 8 / dt)}), flush=True)
