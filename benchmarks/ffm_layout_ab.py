"""A/B of the FFM state layouts on one GPU: packed V|G slots (default) vs split V / G tables,
x reload on/off, x bf16 / fp32 state.

Shape = bench.py: 262,144-row launches, 2^20 hashed features, 39 fields, k=4.  Every variant
trains the same rows from the same init, then scores held-out rows, so a faster variant that
loses more Hogwild updates shows up in the logloss column.

    python benchmarks/ffm_layout_ab.py [--states bf16,fp32] [--steps 24]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", default="bf16,fp32")
    ap.add_argument("--layouts", default="packed,split")
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--batch", type=int, default=262144)
    args = ap.parse_args()
    bits, B, nres = 20, args.batch, 8
    dev = torch.device("cuda")
    idx, y = criteo_like(B * nres, bits, seed=3, device=dev)
    eidx, ey = criteo_like(B, bits, seed=999_999, device=dev)
    yy = (ey > 0).float()
    for state in args.states.split(","):
        for layout in args.layouts.split(","):
            for reload in (True, False):
                opts = f"-c -factors 4 -num_fields 39 -feature_hashing {bits} -seed 31"
                opts += " -bf16_state" if state == "bf16" else ""
                opts += " -split_state" if layout == "split" else ""
                t = FFMTrainer(opts, device=dev)
                t.init_state(1 << bits, 39)
                t.hyper.reload = reload
                for i in range(2):
                    ffm_step(t.state, idx[i * B:(i + 1) * B], None, None, y[i * B:(i + 1) * B], t.hyper)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    s = ((i + 2) % nres) * B
                    ffm_step(t.state, idx[s:s + B], None, None, y[s:s + B], t.hyper)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                pred = torch.empty(B, device=dev)
                ffm_step(t.state, eidx, None, None, None, t.hyper, train=False, pred=pred)
                ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
                print(json.dumps({"state": state, "layout": layout, "reload": reload,
                                  "rows_per_s": round(B * args.steps / dt),
                                  "ms_per_step": round(dt / args.steps * 1e3, 3),
                                  "heldout_logloss": round(ll, 5),
                                  "rows_trained": B * (args.steps + 2)}), flush=True)
                del t
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
