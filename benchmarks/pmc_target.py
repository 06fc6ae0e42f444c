"""Short, fixed-shape runs of the non-FFM hot kernels for rocprofv3 counter passes
(``scripts/gpu_r3k.sh``): each pass replays the same dispatches, so per-dispatch counter means
line up with the ``--kernel-trace --stats`` durations of a separate run.

    python benchmarks/pmc_target.py gbdt|fm|bprmf|mf
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from benchmarks import bench_configs as bc  # noqa: E402

SHAPES = {
    # HIGGS-shaped, depth 8: per level one hist_kernel (smaller child) + sibling + finalize
    "gbdt": lambda: bc.bench_gbdt(n=2_000_000, trees=3),
    "fm": lambda: bc.bench_fm(n_rows=4 * 262144, bits=24),
    "bprmf": lambda: bc.bench_bprmf(k=64, epochs=1),
}


def mf():
    from hivemall_amd.io.synthetic import movielens_like
    from hivemall_amd.models.mf import MatrixFactorization
    us, its = movielens_like(device="cuda", k=16)
    r = (torch.rand(us.numel(), device="cuda") * 4 + 1)
    m = MatrixFactorization("-factors 64 -iters 1 -eta0 0.005", device="cuda")
    m.fit(us, its, r)
    torch.cuda.synchronize()
    return {"bench": "mf", "ratings": us.numel()}


if __name__ == "__main__":
    name = sys.argv[1]
    res = mf() if name == "mf" else SHAPES[name]()
    print(json.dumps(res), flush=True)
