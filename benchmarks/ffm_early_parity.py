"""FFM held-out logloss after the first rows of training (an early-training regime): the GPU
kernel at full concurrency and with the first rows on fewer blocks (HM_FFM_RAMP_ROWS /
HM_FFM_RAMP_GRID, models/ffm.py), against the sequential CPU engine.

    python benchmarks/ffm_early_parity.py [rows] [ramp_grid ...]
"""
import json
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OPTS = "-classification -factors 4 -num_fields 39 -feature_hashing 20 -seed 1"


def one(dev, n):
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.ffm import FFMBatch, FFMTrainer
    idx, y = criteo_like(n, hash_bits=20, seed=5)
    eidx, ey = criteo_like(100000, hash_bits=20, seed=99)
    t = FFMTrainer(OPTS, device=dev)
    t.fit(batch=FFMBatch(idx, None, None, y).to(dev))
    p = t.predict_raw(batch=FFMBatch(eidx, None, None, None).to(dev)).cpu()
    return torch.nn.functional.binary_cross_entropy_with_logits(p, (ey > 0).float()).item()


def main():
    if sys.argv[1:2] == ["--one"]:
        print(json.dumps({"ll": one(sys.argv[2], int(sys.argv[3]))}), flush=True)
        return
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500000
    # each argument: a ramp grid for all n rows ("0": none), or "vV:R" = kernel variant V for the
    # first R rows at the default grid
    grids = sys.argv[2:] or ["0", "256", "1024", "2048"]
    seq = one("cpu", n)
    for g in grids:
        if g.startswith("v"):
            v, r = g[1:].split(":")
            env = dict(os.environ, HM_FFM_RAMP_ROWS=r, HM_FFM_RAMP_VARIANT=v)
        else:
            g = int(g)
            env = dict(os.environ, HM_FFM_RAMP_ROWS=str(n if g else 0), HM_FFM_RAMP_GRID=str(g or 1))
        r = subprocess.run([sys.executable, __file__, "--one", "cuda", str(n)], env=env, capture_output=True,
                           text=True, timeout=600)
        ll = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["ll"]
        print(json.dumps({"rows": n, "ramp_grid": g or "none", "seq_cpu": round(seq, 5), "gpu": round(ll, 5),
                          "delta": round(ll - seq, 5)}), flush=True)


if __name__ == "__main__":
    main()
