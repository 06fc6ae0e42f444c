"""rocprofv3 target: RandomForest fit on HIGGS-shaped 11M x 28 (depth 12), wall time per tree.
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rf -o run -- python3 benchmarks/probes/rf_prof_target.py
"""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
from hivemall_amd.io.synthetic import higgs_like  # noqa: E402
from hivemall_amd.models.trees import RandomForestClassifier  # noqa: E402

trees = int(sys.argv[1]) if len(sys.argv) > 1 else 10
X, y = higgs_like(11_000_000, device="cuda")
RandomForestClassifier("-trees 2 -max_depth 12", device="cuda").fit(X[:100000], y[:100000].long())
torch.cuda.synchronize()
rf = RandomForestClassifier(f"-trees {trees} -max_depth 12", device="cuda")
t0 = time.perf_counter()
rf.fit(X, y.long())
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"rf fit {trees} trees: {dt:.3f} s, {dt * 1e3 / trees:.2f} ms/tree", flush=True)
