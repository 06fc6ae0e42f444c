"""train_fm on the GPU: logloss and rows/s vs launch grid (Hogwild concurrency) against the
sequential engine and the M-mapper-average reference (Hivemall's execution model)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.fm import FMTrainer  # noqa: E402
from tests.test_fm import _rows, mapper_average_fm  # noqa: E402

idx, y = criteo_like(200000, 18, seed=5)
eidx, ey = criteo_like(20000, 18, seed=77)
yy = (ey > 0).float()
opts = "-c -factors 8 -num_features 262144 -eta0 0.01 -sigma 0.01"


def ll(t, dev):
    return torch.nn.functional.binary_cross_entropy_with_logits(
        t.predict_raw(rows=_rows(eidx).to(dev)).cpu(), yy).item()


print(json.dumps({"ref": "sequential", "logloss": ll(FMTrainer(opts, device="cpu").fit(rows=_rows(idx, y)), "cpu")}), flush=True)
for M in (4, 8):
    print(json.dumps({"ref": f"mappers{M}", "logloss": ll(mapper_average_fm(opts, idx, y, M, 262144), "cpu")}), flush=True)
rows = _rows(idx, y).to("cuda")
for grid in (1, 4, 16, 64, 256, 1024, 0):
    for extra in ("", " -fp32"):
        t = FMTrainer(opts + extra, device="cuda")
        t.grid = grid
        t.fit(rows=rows)
        # throughput on a bigger resident set
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.train_rows(rows)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"grid": grid, "dtype": "fp32" if extra else "bf16", "logloss": ll(t, "cuda"),
                          "rows_per_s": rows.n / dt}), flush=True)
