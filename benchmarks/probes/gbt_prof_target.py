"""rocprofv3 target: GBT fit on HIGGS-shaped 11M x 28 (depth 8), wall time per tree printed, so the
kernel-stats total can be set against the wall clock (kernel-bound vs host/launch-bound).
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gbt -o run -- python3 benchmarks/probes/gbt_prof_target.py
"""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
from hivemall_amd.io.synthetic import higgs_like  # noqa: E402
from hivemall_amd.models.trees import GradientTreeBoostingClassifier  # noqa: E402

trees = int(sys.argv[1]) if len(sys.argv) > 1 else 20
X, y = higgs_like(11_000_000, device="cuda")
GradientTreeBoostingClassifier("-trees 2 -max_depth 8", device="cuda").fit(X[:100000], y[:100000].long())
torch.cuda.synchronize()
gb = GradientTreeBoostingClassifier(f"-trees {trees} -eta 0.1 -max_depth 8 -subsample 1.0", device="cuda")
t0 = time.perf_counter()
gb.fit(X, y.long())
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"gbt fit {trees} trees: {dt:.3f} s, {dt * 1e3 / trees:.2f} ms/tree", flush=True)
