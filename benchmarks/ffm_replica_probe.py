"""Hypothesis probe: does averaging R Hogwild replicas (touched-only average, Hivemall's
GROUP BY avg semantics) close the logloss gap to the sequential engine?  Emulated with the
existing kernel: each batch is split into R sub-batches, replica r trains on sub-batch r with
a grid of G/R blocks, then V/w/z/n are averaged over the replicas that touched the feature."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

bits = 20
N = int(os.environ.get("ROWS", "500000"))
dev = torch.device("cuda")
idx, y = criteo_like(N, bits, seed=5, device=dev)
eidx, ey, el = criteo_like(200000, bits, seed=999_999, return_logit=True, device=dev)
yy = (ey > 0).float()
for R, grid, B in [(1, 0, 65536), (4, 1536, 65536), (8, 768, 65536), (8, 768, 16384), (16, 384, 65536)]:
    trs = []
    for r in range(R):
        t = FFMTrainer(f"-c -factors 4 -num_fields 39 -feature_hashing {bits} -seed 1", device=dev)
        t.init_state(1 << bits, 39)
        if r:
            for k in t.state:
                t.state[k].copy_(trs[0].state[k])
        trs.append(t)
    keys = ["V", "w", "wz", "wn"]
    for s in range(0, N, B):
        e = min(N, s + B)
        cnt = torch.zeros(1 << bits, device=dev)
        masks = []
        for r in range(R):
            a = s + (e - s) * r // R
            b = s + (e - s) * (r + 1) // R
            ffm_step(trs[r].state, idx[a:b], None, None, y[a:b], trs[r].hyper, grid=grid)
            m = torch.zeros(1 << bits, device=dev)
            m[idx[a:b].reshape(-1).long()] = 1.0
            masks.append(m)
            cnt += m
        if R > 1:
            hit = cnt > 0
            for k in keys:
                acc = None
                for r in range(R):
                    x = trs[r].state[k]
                    m = masks[r].view(-1, *([1] * (x.dim() - 1)))
                    acc = x * m if acc is None else acc + x * m
                c = cnt.view(-1, *([1] * (acc.dim() - 1))).clamp_min(1)
                avg = acc / c
                h = hit.view(-1, *([1] * (acc.dim() - 1)))
                for r in range(R):
                    trs[r].state[k].copy_(torch.where(h, avg, trs[r].state[k]))
    p = trs[0].predict_raw(batch=FFMBatch(eidx, None, None, None))
    ll = torch.nn.functional.binary_cross_entropy_with_logits(p, yy).item()
    print(json.dumps({"rows": N, "R": R, "grid": grid, "mix_batch": B, "logloss": round(ll, 5)}), flush=True)
