"""Logloss parity probe: sequential C++ engine (Hivemall per-row semantics) vs the gfx950
Hogwild kernel at several launch geometries and data sizes.  Prints one JSON line per run."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer  # noqa: E402

bits = int(os.environ.get("BITS", "20"))
sizes = [int(s) for s in os.environ.get("SIZES", "60000,500000").split(",")]
grids = [int(g) for g in os.environ.get("GRIDS", "0,256").split(",")]
eidx, ey, el = criteo_like(200000, bits, seed=999_999, return_logit=True)
yy = (ey > 0).float()
floor = torch.nn.functional.binary_cross_entropy_with_logits(el, yy).item()
for n in sizes:
    idx, y = criteo_like(n, bits, seed=5)
    for dev, grid, rl in [("cpu", 0, 1)] + [("cuda", g, r) for g in grids for r in (0, 1)]:
        if dev == "cpu" and n > int(os.environ.get("CPU_MAX", "600000")):
            continue
        t = FFMTrainer(f"-c -factors 4 -num_fields 39 -feature_hashing {bits} -iters 1 -seed 1",
                       device=dev)
        t.grid = grid
        t.hyper.reload = bool(rl)
        t0 = time.time()
        t.fit(batch=FFMBatch(idx, None, None, y).to(dev))
        if dev == "cuda":
            torch.cuda.synchronize()
        dt = time.time() - t0
        p = t.predict_raw(batch=FFMBatch(eidx, None, None, None).to(dev)).cpu()
        ll = torch.nn.functional.binary_cross_entropy_with_logits(p, yy).item()
        print(json.dumps({"rows": n, "dev": dev, "grid": grid, "reload": rl, "logloss": round(ll, 5),
                          "floor": round(floor, 5), "fit_s": round(dt, 2)}), flush=True)
