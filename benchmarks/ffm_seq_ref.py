"""Sequential-engine reference logloss for bench.py's OWN row stream.

bench.py (``--gen-device cpu``, the default since round 6) trains each rank r on 8 resident
batches of 262,144 ``criteo_ffm`` rows drawn with seed 1000 + r, cycling over them for
``warmup + steps`` steps, and evaluates the mixed model on 262,144 held-out rows (seed 999,999).
This script replays exactly those rows through the sequential C++ engine (Hivemall's per-row
FFM semantics, fp32 state, ``csrc/host/ffm_cpu.cpp``) as ONE learner — for N ranks the rows of
step i are taken rank 0, 1, .., N-1 in turn, i.e. one learner over the union of the ranks'
shards, which is what the mixed replicas track (docs/compat.md) — and records its held-out
logloss in ``resources/bench_seq_ref.json``.  bench.py looks its own configuration up there and
prints ``logloss_seq_ref`` and ``logloss_gap`` next to ``logloss_heldout``, so every driver
record carries the parity half of the headline metric.

    python benchmarks/ffm_seq_ref.py --gpus 1 --steps 20 --warmup 5

CPU only; the sequential engine trains ~20-60 K rows/s on one core.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hivemall_amd.io.synthetic import criteo_ffm  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

REF_PATH = os.path.join(ROOT, "resources", "bench_seq_ref.json")


def ref_key(gpus: int, steps: int, warmup: int, batch: int, hash_bits: int, factors: int,
            resident: int, eval_rows: int, data: str = "criteo_ffm", order: str = "none") -> str:
    """The lookup key bench.py and this script agree on (every knob that changes the rows, the
    order they are trained in, or the model)."""
    return (f"{data}/n{gpus}/s{steps}/w{warmup}/b{batch}/h{hash_bits}/k{factors}/r{resident}"
            f"/e{eval_rows}/o{order}")


def load_refs() -> dict:
    try:
        with open(REF_PATH) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def run(gpus, steps, warmup, batch, hash_bits, factors, resident, eval_rows, order="none"):
    F = 39
    opts = (f"-classification -factors {factors} -feature_hashing {hash_bits} -num_fields {F} "
            f"-seed 31 -batch_size {batch}")
    tr = FFMTrainer(opts, device="cpu")
    tr.init_state(1 << hash_bits, F)
    shards = [criteo_ffm(batch * resident, hash_bits, seed=1000 + r) for r in range(gpus)]
    if order != "none":
        from hivemall_amd.ops.ffm_sched import schedule_rows

        for r, (idx, fld, val, y) in enumerate(shards):
            for b in range(resident):
                s = slice(b * batch, (b + 1) * batch)
                p = schedule_rows(idx[s], order)
                idx[s], fld[s], val[s], y[s] = idx[s][p], fld[s][p], val[s][p], y[s][p]
    t0 = time.time()
    for i in range(warmup + steps):
        s = (i % resident) * batch
        for idx, fld, val, y in shards:
            ffm_step(tr.state, idx[s:s + batch], fld[s:s + batch], val[s:s + batch],
                     y[s:s + batch], tr.hyper, train=True)
    dt = time.time() - t0
    eidx, efld, evl, ey, elogit = criteo_ffm(eval_rows, hash_bits, seed=999_999, return_logit=True)
    pred = torch.empty(eval_rows)
    for s in range(0, eval_rows, batch):
        e = min(eval_rows, s + batch)
        ffm_step(tr.state, eidx[s:e], efld[s:e], evl[s:e], None, tr.hyper, train=False, pred=pred[s:e])
    yy = (ey > 0).float()
    ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
    floor = torch.nn.functional.binary_cross_entropy_with_logits(elogit, yy).item()
    rows = batch * gpus * (warmup + steps)
    return {"logloss_seq": round(ll, 6), "floor": round(floor, 6), "rows": rows,
            "train_s": round(dt, 1), "engine": "sequential C++ (csrc/host/ffm_cpu.cpp), fp32"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--hash-bits", type=int, default=20)
    ap.add_argument("--factors", type=int, default=4)
    ap.add_argument("--resident-batches", type=int, default=8)
    ap.add_argument("--eval-rows", type=int, default=262144)
    ap.add_argument("--order", default="none", help="row schedule inside each batch (bench.py --row-order)")
    ap.add_argument("--write", type=int, default=1)
    a = ap.parse_args()
    torch.set_num_threads(int(os.environ.get("HM_REF_THREADS", "2")))
    key = ref_key(a.gpus, a.steps, a.warmup, a.batch, a.hash_bits, a.factors,
                  a.resident_batches, a.eval_rows, order=a.order)
    rec = run(a.gpus, a.steps, a.warmup, a.batch, a.hash_bits, a.factors, a.resident_batches,
              a.eval_rows, a.order)
    print(json.dumps({"key": key, **rec}), flush=True)
    if a.write:
        # re-read right before the write: several of these runs go in parallel
        refs = load_refs()
        refs[key] = rec
        with open(REF_PATH, "w") as f:
            json.dump(dict(sorted(refs.items())), f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
