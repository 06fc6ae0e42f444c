"""Explicit MF atomic-update throughput on the ML-20M shape: which hot line bounds it?
Compares atomic mode with and without biases (the item-bias array packs 16 items per 64-B line,
so the 16 most popular items' bias adds share one line) and at k = 16 / 32 / 64.
    python benchmarks/mf_contention_probe.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from hivemall_amd.io.synthetic import movielens_like  # noqa: E402
from hivemall_amd.models.mf import MatrixFactorization  # noqa: E402


def main():
    dev = torch.device("cuda")
    us, its = movielens_like(device=dev, k=16)
    r = 3.5 + 0.5 * torch.randn(us.numel(), device=dev)
    for atomic in ("1", "0"):
        os.environ["HM_MF_ATOMIC"] = atomic
        for opts in ("-factors 16", "-factors 16 -disable_bias", "-factors 32", "-factors 64",
                     "-factors 16 -grid 3392"):
            m = MatrixFactorization(f"{opts} -iters 1 -mu 3.5 -eta0 0.01", device=dev)
            m.fit(us, its, r)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                m.fit(us, its, r)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"atomic": atomic, "opts": opts, "grid": m._grid(),
                              "ratings_per_s": round(3 * us.numel() / dt)}), flush=True)


if __name__ == "__main__":
    main()
