"""the generic FFM kernel's (ffm_row_kernel, variant 1) early-training Hogwild gap vs the
sequential engine moved 0.0117 -> 0.0164 when the linear FTRL {w, z, n} records moved into the
feature blocks.  This runs test_ffm_gpu_hogwild_logloss_parity_with_sequential's setup (500 K
criteo_like rows, 2^20 features, full grid) for the generic and the pipelined kernel with the
linear state as records (default) or separate arrays (``--separate``, set before import), each
``--reps`` times, and prints the gap to the CPU engine.

    python benchmarks/ffm_generic_lin_probe.py [--separate] [--reps 3]
"""
import argparse
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--separate", action="store_true")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--variants", default="1,0")
a = ap.parse_args()
if a.separate:
    os.environ["HM_FFM_LIN_SEPARATE"] = "1"

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models import ffm as ffm_model  # noqa: E402
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer  # noqa: E402
from hivemall_amd.ops import ffm as ffm_op  # noqa: E402


def run(dev, variant):
    ffm_op._VARIANT = variant
    ffm_model.RAMP_ROWS = 0
    t = FFMTrainer("-classification -factors 4 -num_fields 39 -feature_hashing 20 -seed 1", device=dev)
    t.fit(batch=FFMBatch(idx, None, None, y).to(dev))
    ffm_op._VARIANT = 0
    p = t.predict_raw(batch=FFMBatch(eidx, None, None, None).to(dev)).cpu()
    return torch.nn.functional.binary_cross_entropy_with_logits(p, yy).item()


idx, y = criteo_like(500000, hash_bits=20, seed=5)
eidx, ey = criteo_like(100000, hash_bits=20, seed=99)
yy = (ey > 0).float()
seq = run("cpu", 0)
for v in [int(x) for x in a.variants.split(",")]:
    for r in range(a.reps):
        g = run("cuda", v)
        print(json.dumps({"lin": "separate" if a.separate else "records", "variant": v, "rep": r,
                          "seq": round(seq, 5), "gpu": round(g, 5), "gap": round(g - seq, 5)}), flush=True)
