"""XCD replicas for the fp32 FFM kernel on the bench's exact stream (12,582,912 rows of
criteo_ffm, seed 1000, 8 resident batches of 262,144, the atomic ramp in step 0; sequential engine
0.44501, profiles/r4/ffm_parity_bench_scale_ffmdata.log).  After the ramp the model gets R
replicas (ops/ffm.py xcd_replicate: block b trains replica b % R, i.e. one per XCD), averaged
every K steps (xcd_merge) with every replica's step size scaled by R^p (as data-parallel ranks,
docs/compat.md).  Prints held-out logloss and timed rows/s (steps 8..47, merges included).

    python benchmarks/ffm_xrep_probe.py [R:K:p ...]      (R = 1: the default single table)
"""
import copy
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models import ffm as ffm_model  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step, xcd_merge, xcd_replicate  # noqa: E402

B, NRES, BITS, F = 262144, 8, 20, 39
OPTS = f"-classification -factors 4 -feature_hashing {BITS} -num_fields {F} -seed 31 -batch_size {B}"
SEQ = 0.44501


def main():
    cfgs = sys.argv[1:] or ["1:0:0", "8:10:0.75", "8:10:0.5", "8:5:0.75", "8:20:0.75"]
    steps, warmup = 48, 8
    dev = torch.device("cuda")
    idx, fld, val, y = (t.to(dev) for t in criteo_ffm(B * NRES, BITS, seed=1000))
    eidx, efld, evl, ey, _ = (t.to(dev) for t in criteo_ffm(B, BITS, seed=999_999, return_logit=True))
    yy = (ey > 0).float()
    for c in cfgs:
        R, K, p = c.split(":")
        R, K, p = int(R), int(K), float(p)
        tr = FFMTrainer(OPTS, device=dev)
        tr.init_state(1 << BITS, F)
        h0 = tr.hyper
        hx = copy.copy(h0)
        hx.eta0 *= R ** p
        hx.alpha *= R ** p
        torch.cuda.synchronize()
        t0 = None
        for i in range(steps):
            if i == warmup:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            s = (i % NRES) * B
            if i == 0:
                ffm_step(tr.state, idx[s:s + B], fld[s:s + B], val[s:s + B], y[s:s + B], h0,
                         variant=ffm_model.RAMP_VARIANT)
                if R > 1:
                    xcd_replicate(tr.state, R)
                continue
            ffm_step(tr.state, idx[s:s + B], fld[s:s + B], val[s:s + B], y[s:s + B], hx if R > 1 else h0)
            if R > 1 and (i % K == 0 or i == steps - 1):
                xcd_merge(tr.state)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        pred = torch.empty(B, device=dev)
        ffm_step(tr.state, eidx, efld, evl, None, h0, train=False, pred=pred)
        ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
        print(json.dumps({"R": R, "merge_every": K, "power": p, "logloss_heldout": round(ll, 5),
                          "gap_vs_seq": round(ll - SEQ, 5),
                          "rows_per_s": round(B * (steps - warmup) / dt / 1e6, 2)}), flush=True)
        del tr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
