"""train_fm's stale global bias (ops/fm.py W0_*): held-out logloss of the GPU learner on a stream
past 2^20 rows against Hivemall's 8-mapper CPU average on the same rows, for bias re-read
schedules (every row / every 8 rows / adaptive tolerance / the warm-rows rule).

    python benchmarks/fm_w0_probe.py [n_rows] [configs...]     config = every:tol:warm, e.g. 8:2:1048576
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.fm import FMTrainer  # noqa: E402
from hivemall_amd.ops import fm as fm_ops  # noqa: E402
from tests.test_fm import _rows, mapper_average_fm  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3 << 20
    cfgs = sys.argv[2:] or ["1:0:0", "8:0:1048576", "8:2:1048576", "8:2:0", "8:0.5:0"]
    idx, y = criteo_like(n, 20, seed=5)
    eidx, ey = criteo_like(100000, 20, seed=77)
    yy = (ey > 0).float()
    opts = "-c -factors 8 -num_features 1048576 -eta0 0.01 -sigma 0.01"
    ll = lambda t, dev: torch.nn.functional.binary_cross_entropy_with_logits(  # noqa: E731
        t.predict_raw(rows=_rows(eidx).to(dev)).cpu(), yy).item()
    t0 = time.time()
    ref = mapper_average_fm(opts, idx, y, 8, 1 << 20)
    m8 = ll(ref, "cpu")
    print(json.dumps({"mappers8": round(m8, 5), "rows": n, "cpu_s": round(time.time() - t0, 1)}), flush=True)
    rows = _rows(idx, y).to("cuda")
    for c in cfgs:
        every, tol, warm = c.split(":")
        fm_ops.W0_EVERY, fm_ops.W0_TOL, fm_ops.W0_WARM_ROWS = int(every), float(tol), int(warm)
        torch.cuda.synchronize()
        t = time.perf_counter()
        g = FMTrainer(opts, device="cuda").fit(rows=rows)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        v = ll(g, "cuda")
        print(json.dumps({"every": int(every), "tol": float(tol), "warm_rows": int(warm), "gpu": round(v, 5),
                          "delta_vs_mappers8": round(v - m8, 5), "rows_per_s": round(n / dt)}), flush=True)


if __name__ == "__main__":
    main()
