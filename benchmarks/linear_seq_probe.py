"""Near-sequential engine (``-engine seq``, csrc/kernels/linear.hip linear_seq_kernel) vs the
sequential CPU engine at Hivemall's default ``-mini_batch 1 -dims 2^24``.

For each rule: one epoch over N Criteo-shaped hashed rows (39 nnz), held-out logloss of the CPU
engine (one replica: the sequential learner) and of the GPU seq engine at each rows-in-flight W
and XCD spread, with the GPU pass's rows/s (fit time, device-synchronised).

    python benchmarks/linear_seq_probe.py [--rows 1000000] [--waves 8,16,32,64] [--spread 8,1]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

RULES = ["-opt adam -eta0 0.01", "-opt sgd -eta0 0.05", "-opt rmsprop -eta0 0.01", "-opt adadelta",
         "-opt momentum -eta0 0.005"]


def rows_of(n, bits, seed):
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.linear import SparseRows

    idx, y = criteo_like(n, hash_bits=bits, seed=seed)
    return SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64), idx.reshape(-1).contiguous(),
                      None, y.contiguous())


def heldout(m, test, dev):
    s = m.decision_function(rows=test.to(dev)).cpu()
    yy = (test.y > 0).float()
    return torch.nn.functional.binary_cross_entropy_with_logits(s, yy).item()


def fit(opts, rows, dev, timed=True):
    """``opts``: train_classifier options, or "<learner>: options" for another SQL learner."""
    from hivemall_amd.models.linear import LEARNERS

    name, _, o = opts.partition(":") if ":" in opts else ("train_classifier", "", opts)
    base = "-loss logloss " if name == "train_classifier" else ""
    m = LEARNERS[name.strip()](f"{base}{o} -dims 16777216 -iters 1", device=dev)
    r = rows.to(dev)
    m._ensure_state(r)
    if dev == "cuda":
        torch.cuda.synchronize()
    t = time.perf_counter()
    m.fit(rows=r)
    if dev == "cuda":
        torch.cuda.synchronize()
    return m, rows.n / (time.perf_counter() - t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--waves", default="8,16,32,64")
    ap.add_argument("--spread", default="8,1")
    ap.add_argument("--rules", default=None, help="';'-separated option strings")
    ap.add_argument("--shared", type=int, default=1, help="also the shared engine at its rule waves")
    ap.add_argument("--seed", type=int, default=5, help="training rows' seed")
    a = ap.parse_args()
    rules = a.rules.split(";") if a.rules else RULES
    rows = rows_of(a.rows, 24, a.seed)
    test = rows_of(100_000, 24, 99)
    for opts in rules:
        mc, rc = fit(opts, rows, "cpu")
        ll_c = heldout(mc, test, "cpu")
        print(json.dumps({"opts": opts, "engine": "cpu-seq", "rows": a.rows, "seed": a.seed, "logloss": round(ll_c, 5),
                          "rows_per_s": round(rc)}), flush=True)
        if a.shared:
            m, r = fit(opts + " -engine shared", rows, "cuda")
            ll = heldout(m, test, "cuda")
            print(json.dumps({"opts": opts, "engine": "shared", "waves": int(m.state.RS.shape[0]),
                              "logloss": round(ll, 5), "delta": round(ll - ll_c, 5),
                              "rows_per_s": round(r)}), flush=True)
        for sp in [int(x) for x in a.spread.split(",")]:
            for w in [int(x) for x in a.waves.split(",")]:
                m, r = fit(f"{opts} -engine seq -shared_waves {w} -seq_spread {sp}", rows, "cuda")
                ll = heldout(m, test, "cuda")
                print(json.dumps({"opts": opts, "engine": "seq", "waves": w, "spread": sp,
                                  "logloss": round(ll, 5), "delta": round(ll - ll_c, 5),
                                  "rows_per_s": round(r)}), flush=True)


if __name__ == "__main__":
    main()
