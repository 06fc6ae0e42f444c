"""One block (-grid 1) of an FFM kernel variant vs the sequential CPU engine on field-disjoint
criteo_like rows (test_ffm_gpu_single_block_is_exactly_sequential's setup), for A/B variants.

    python benchmarks/ffm_variant_exact.py 0 9
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models import ffm as ffm_model  # noqa: E402
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer  # noqa: E402
from hivemall_amd.ops import ffm as ffm_op  # noqa: E402

idx, y = criteo_like(20000, hash_bits=16, seed=5)
eidx, ey = criteo_like(5000, hash_bits=16, seed=99)
fid = torch.arange(39, dtype=idx.dtype)
idx = idx % 1024 + fid * 1024
eidx = eidx % 1024 + fid * 1024
yy = (ey > 0).float()
ffm_model.RAMP_ROWS = 0
res = {}
for dev, v in [("cpu", 0)] + [("cuda", int(a)) for a in sys.argv[1:]]:
    for k in (4, 8):
        ffm_op._VARIANT = v
        t = FFMTrainer(f"-classification -factors {k} -num_fields 39 -feature_hashing 16 -seed 1", device=dev)
        t.grid = 1
        t.fit(batch=FFMBatch(idx, None, None, y).to(dev))
        ffm_op._VARIANT = 0
        p = t.predict_raw(batch=FFMBatch(eidx, None, None, None).to(dev)).cpu()
        res[(dev, v, k)] = torch.nn.functional.binary_cross_entropy_with_logits(p, yy).item()
for (dev, v, k), ll in res.items():
    print(json.dumps({"dev": dev, "variant": v, "k": k, "logloss": ll, "delta_vs_cpu": ll - res[("cpu", 0, k)]}))
