"""Logloss parity at the headline bench's scale.

Replays EXACTLY the row stream that ``bench.py --gen-device cpu`` (1 rank, defaults) trains on
— 8 resident batches of 262,144 Criteo-shaped rows (seed 1000; ``--data`` as bench.py), 48 steps (8 warmup + 40 timed) cycling over
them: 12,582,912 rows — through

* the sequential C++ engine (Hivemall's per-row FFM semantics, fp32 state): ``seq``;
* an M-mapper average (Hivemall DP-1: M independent learners over contiguous shards of the
  stream, then ``avg(weight) GROUP BY feature``): ``avgM``;

and reports held-out logloss on bench.py's evaluation rows (262,144 rows, seed 999,999) next to
the planted-model floor.  The GPU numbers come from bench.py's own JSON (``logloss_heldout``,
bf16 and fp32 state).  CPU only; ~5 minutes per full pass on 8 cores.

    python benchmarks/ffm_parity_bench_scale.py [--mappers 8] [--rows 12582912]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm, criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

B, NRES, BITS, F = 262144, 8, 20, 39
OPTS = f"-classification -factors 4 -feature_hashing {BITS} -num_fields {F} -seed 31 -batch_size {B}"
DATA = "criteo_ffm"       # bench.py --data (explicit fields + values; criteo_like = rounds 1-3)


def gen(n, seed, logit=False):
    """(idx, fld, val, y[, logit]) exactly as bench.py --gen-device cpu draws them."""
    if DATA == "criteo_ffm":
        return criteo_ffm(n, BITS, seed=seed, return_logit=logit)
    out = criteo_like(n, BITS, seed=seed, return_logit=logit)
    return (out[0], None, None) + tuple(out[1:])


def stream_batches(n_rows):
    idx, fld, val, y = gen(B * NRES, 1000)
    steps = n_rows // B
    sl = lambda t, s: None if t is None else t[s:s + B]  # noqa: E731
    for i in range(steps):
        s = (i % NRES) * B
        yield idx[s:s + B], sl(fld, s), sl(val, s), y[s:s + B]


def heldout(tr):
    eidx, efld, evl, ey, elogit = gen(B, 999_999, logit=True)
    pred = torch.empty(B)
    ffm_step(tr.state, eidx, efld, evl, None, tr.hyper, train=False, pred=pred)
    yy = (ey > 0).float()
    ll = torch.nn.functional.binary_cross_entropy_with_logits(pred, yy).item()
    floor = torch.nn.functional.binary_cross_entropy_with_logits(elogit, yy).item()
    return ll, floor


def run_seq(n_rows):
    tr = FFMTrainer(OPTS, device="cpu")
    tr.init_state(1 << BITS, F)
    t0 = time.time()
    for idx, fld, val, y in stream_batches(n_rows):
        ffm_step(tr.state, idx, fld, val, y, tr.hyper, train=True)
    return tr, time.time() - t0


def run_avg(n_rows, M):
    """M learners from the same init, each over a contiguous 1/M of the stream, then averaged
    (V, w and the FTRL state, as the mixer does)."""
    base = FFMTrainer(OPTS, device="cpu")
    base.init_state(1 << BITS, F)
    init = {k: v.clone() for k, v in base.state.items()}
    acc = {k: torch.zeros_like(v, dtype=torch.float64) for k, v in init.items() if k in ("V", "w", "wz", "wn", "bias")}
    batches = list(stream_batches(n_rows))
    per = len(batches) * B // M                     # rows per mapper
    flat_idx = torch.cat([b[0] for b in batches])
    flat_fld = None if batches[0][1] is None else torch.cat([b[1] for b in batches])
    flat_val = None if batches[0][2] is None else torch.cat([b[2] for b in batches])
    flat_y = torch.cat([b[3] for b in batches])
    sl = lambda t, q, e: None if t is None else t[q:min(e, q + B)]  # noqa: E731
    t0 = time.time()
    for m in range(M):
        for k in base.state:
            base.state[k].copy_(init[k])
        s, e = m * per, (m + 1) * per
        for q in range(s, e, B):
            ffm_step(base.state, sl(flat_idx, q, e), sl(flat_fld, q, e), sl(flat_val, q, e),
                     sl(flat_y, q, e), base.hyper)
        for k in acc:
            acc[k] += base.state[k].double()
    for k in acc:
        base.state[k].copy_((acc[k] / M).to(base.state[k].dtype))
    return base, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=48 * B)
    ap.add_argument("--mappers", type=int, default=8)
    ap.add_argument("--skip-seq", action="store_true")
    ap.add_argument("--data", choices=("criteo_ffm", "criteo_like"), default="criteo_ffm")
    a = ap.parse_args()
    global DATA
    DATA = a.data
    torch.set_num_threads(os.cpu_count() or 8)
    if not a.skip_seq:
        tr, dt = run_seq(a.rows)
        ll, floor = heldout(tr)
        print(json.dumps({"engine": "seq (C++ per-row, fp32)", "data": DATA, "rows": a.rows, "logloss_heldout": round(ll, 5),
                          "floor": round(floor, 5), "train_s": round(dt, 1),
                          "rows_per_s": round(a.rows / dt)}), flush=True)
    if a.mappers > 0:
        tr, dt = run_avg(a.rows, a.mappers)
        ll, floor = heldout(tr)
        print(json.dumps({"engine": f"avg{a.mappers} (M-mapper average, fp32)", "data": DATA, "rows": a.rows,
                          "logloss_heldout": round(ll, 5), "floor": round(floor, 5), "train_s": round(dt, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
