"""Held-out logloss of train_ffm -w0 (the global bias) on the GPU vs the sequential engine, on 1 M
criteo_ffm rows (2 passes), for the sharded bias state re-read every HM_FFM_BIAS_EVERY rows and the
single-address state (HM_FFM_BIAS_SHARDS=0).

    python benchmarks/ffm_w0_quality_probe.py [every ...]     # 64 shards at each re-read interval
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer  # noqa: E402
from hivemall_amd.ops import ffm as ffm_ops  # noqa: E402

n, BITS = 1 << 20, 20
idx, fld, val, y = criteo_ffm(n, BITS, seed=1000)
eidx, efld, evl, ey, _ = criteo_ffm(200000, BITS, seed=999_999, return_logit=True)
yy = (ey > 0).float()
opts = f"-c -factors 4 -num_fields 39 -feature_hashing {BITS} -w0 -iters 2 -disable_cv"


def run(dev):
    t = FFMTrainer(opts, device=dev)
    t0 = time.time()
    t.fit(batch=FFMBatch(idx, fld, val, y).to(dev))
    p = t.predict_raw(batch=FFMBatch(eidx, efld, evl, None).to(dev)).cpu()
    return torch.nn.functional.binary_cross_entropy_with_logits(p, yy).item(), time.time() - t0, float(t.state["bias"][0])


seq, dt, b = run("cpu")
print(json.dumps({"engine": "cpu sequential", "logloss": round(seq, 5), "w0": round(b, 4), "s": round(dt, 1)}), flush=True)
cases = [(64, int(a)) for a in sys.argv[1:]] or [(64, 8), (64, 16), (64, 1), (0, 1)]
for shards, every in cases:
    ffm_ops.BIAS_SHARDS, ffm_ops.BIAS_EVERY = shards, every
    ll, dt, b = run("cuda")
    print(json.dumps({"bias_shards": shards, "bias_every": every, "logloss": round(ll, 5), "gap": round(ll - seq, 5),
                      "w0": round(b, 4), "s": round(dt, 2)}), flush=True)
