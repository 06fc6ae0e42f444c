"""Kernel rate of train_ffm under its non-default options (the bench config runs only the default):
a cliff like -w0's (5.5 M rows/s before round 5) shows up here.  criteo_ffm rows, 262,144 per step,
2^20 features, 20 timed steps after 4 warm.

    python benchmarks/ffm_option_rate_sweep.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

dev = torch.device("cuda")
B, NRES = 262144, 4
idx, fld, val, y = criteo_ffm(B * NRES, 20, seed=3, device=dev)
yr = torch.where(y > 0, 1.0, 0.0)      # regression targets
base = "-factors 4 -num_fields 39 -feature_hashing 20"
cases = sys.argv[1:] or ["-c", "-c -w0", "-c -disable_wi", "-c -no_norm", "", "-c -elementwise_adagrad", "-c -bf16_state",
         "-c -bf16_state -w0", "-c -factors 8", "-c -w0 -disable_wi"]
for extra in cases:
    opts = base + " " + extra
    if "-factors 8" in extra:
        opts = opts.replace("-factors 4 ", "")
    t = FFMTrainer(opts, device=dev)
    t.init_state(1 << 20, 39)
    yy = y if "-c" in extra.split() else yr
    for i in range(24):
        if i == 4:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        s = (i % NRES) * B
        ffm_step(t.state, idx[s:s + B], fld[s:s + B], val[s:s + B], yy[s:s + B], t.hyper)
    torch.cuda.synchronize()
    print(json.dumps({"opts": extra or "(regression)", "rows_per_s": round(B * 20 / (time.perf_counter() - t0) / 1e6, 2)}),
          flush=True)
