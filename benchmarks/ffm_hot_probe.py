"""How much of the fp32 FFM kernel's same-stream logloss gap comes from its hottest features?

Replays bench.py's exact 1-rank stream (``--gen-device cpu``: 8 resident batches of 262,144
criteo_ffm rows, seed 1000, 48 steps = 12,582,912 rows, the first step on the atomic ramp
kernel) and varies which (feature, field) slots are updated by float atomics (kernel variant 8:
slots of the features flagged hot) instead of the Hogwild read-modify-write store.  The hot set
is the top-H features by frequency in the resident rows.  Prints one JSON line per H: timed
rows/s of steps 8..47 and held-out logloss (sequential engine on this stream: 0.44501,
profiles/r4/ffm_parity_bench_scale_ffmdata.log).

    python benchmarks/ffm_hot_probe.py [--hs 0,32,128,512,2048] [--steps 48] [--variant 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models import ffm as ffm_model  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

B, NRES, BITS, F = 262144, 8, 20, 39
OPTS = f"-classification -factors 4 -feature_hashing {BITS} -num_fields {F} -seed 31 -batch_size {B}"
SEQ = 0.44501


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hs", default="0,32,128,512,2048,8192")
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--variant", type=int, default=8)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--plain", default="", help="kernel variants without a hot set, e.g. 0,10")
    ap.add_argument("--grid", type=int, default=0, help="plain runs: blocks (0 = the kernel's default)")
    ap.add_argument("--ramp-steps", type=int, default=1, help="plain runs: steps on the atomic ramp kernel")
    a = ap.parse_args()
    dev = torch.device("cuda")
    idx, fld, val, y = (t.to(dev) for t in criteo_ffm(B * NRES, BITS, seed=1000))
    eidx, efld, evl, ey, elogit = (t.to(dev) for t in criteo_ffm(B, BITS, seed=999_999, return_logit=True))
    cnt = torch.bincount(idx.flatten().long(), minlength=1 << BITS)
    order = torch.argsort(cnt, descending=True)
    tot = float(cnt.sum())
    yy = (ey > 0).float()
    def run(H, var, hot):
        tr = FFMTrainer(OPTS, device=dev)
        tr.init_state(1 << BITS, F)
        torch.cuda.synchronize()
        t0 = None
        for i in range(a.steps):
            if i == a.warmup:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            s = (i % NRES) * B
            if i % 8 == 0:
                print(f"step {i}", file=sys.stderr, flush=True)
            v = ffm_model.RAMP_VARIANT if i < a.ramp_steps else var
            ffm_step(tr.state, idx[s:s + B], fld[s:s + B], val[s:s + B], y[s:s + B], tr.hyper,
                     train=True, variant=v, hot=hot, grid=a.grid)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        pred = torch.empty(B, device=dev)
        ffm_step(tr.state, eidx, efld, evl, None, tr.hyper, train=False, pred=pred)
        ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
        return B * (a.steps - a.warmup) / dt / 1e6, ll

    for rep in range(a.reps):
        for v in [int(x) for x in a.plain.split(",") if x]:
            rate, ll = run(0, v, None)
            print(json.dumps({"mode": "plain", "variant": v, "grid": a.grid, "ramp_steps": a.ramp_steps,
                              "rep": rep, "rows_per_s": round(rate, 2),
                              "logloss_heldout": round(ll, 5), "gap_vs_seq": round(ll - SEQ, 5)}), flush=True)
        for H in [int(h) for h in a.hs.split(",") if h]:
            hot = torch.zeros(1 << BITS, dtype=torch.uint8, device=dev)
            if H > 0:
                hot[order[:H]] = 1
            cover = float(cnt[order[:H]].sum()) / tot if H > 0 else 0.0
            tr = FFMTrainer(OPTS, device=dev)
            tr.init_state(1 << BITS, F)
            torch.cuda.synchronize()
            t0 = None
            for i in range(a.steps):
                if i == a.warmup:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                s = (i % NRES) * B
                var = ffm_model.RAMP_VARIANT if i == 0 else (a.variant if H > 0 else 0)
                ffm_step(tr.state, idx[s:s + B], fld[s:s + B], val[s:s + B], y[s:s + B], tr.hyper,
                         train=True, variant=var, hot=hot if H > 0 else None)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            pred = torch.empty(B, device=dev)
            ffm_step(tr.state, eidx, efld, evl, None, tr.hyper, train=False, pred=pred)
            ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
            print(json.dumps({"H": H, "row_cover": round(cover, 4), "rep": rep,
                              "rows_per_s": round(B * (a.steps - a.warmup) / dt / 1e6, 2),
                              "logloss_heldout": round(ll, 5), "gap_vs_seq": round(ll - SEQ, 5)}),
                  flush=True)
            del tr


if __name__ == "__main__":
    main()
