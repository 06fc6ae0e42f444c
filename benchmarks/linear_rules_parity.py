"""Held-out logloss of every train_classifier -opt on the GPU shared-table engine at Hivemall's
default -dims 2^24 vs the sequential CPU engine.

For each rule: one epoch over Criteo-shaped hashed rows (39 nnz) on the CPU (sequential, one
replica) and on the GPU shared-table engine at each ``HM_RULE_WAVES`` rows in flight.

    python benchmarks/linear_rules_parity.py [rows] [opts...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# every rule at a step size where the sequential learner converges on these rows (held-out
# 0.476-0.487 at 300 K rows; a diverging or oscillating sequential run, e.g. momentum at eta0 0.05
# or Adam at eta0 0.1, has no trajectory for a parallel engine to match)
RULES = ["-opt sgd -eta0 0.05", "-opt momentum -eta0 0.005", "-opt nesterov -eta0 0.005", "-opt adagrad",
         "-opt adagrad -reg l1 -lambda 1e-6", "-opt rmsprop -eta0 0.01", "-opt rmspropgraves -eta0 0.001",
         "-opt adadelta", "-opt adam -eta0 0.01", "-opt nadam -eta0 0.01", "-opt eve -eta0 0.01",
         "-opt adamhd -eta0 0.01"]


def rows_of(n, bits, seed):
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.linear import SparseRows

    idx, y = criteo_like(n, hash_bits=bits, seed=seed)
    return SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64), idx.reshape(-1).contiguous(),
                      None, y.contiguous())


def run(opts, rows, test, dev, hot=True, waves=0):
    from hivemall_amd.models.linear import TrainClassifier

    os.environ["HM_LINEAR_HOT"] = "1" if hot else "0"
    extra = f" -shared_waves {waves}" if waves else ""
    m = TrainClassifier(f"-loss logloss {opts} -dims 16777216 -iters 1{extra}", device=dev)
    r = rows.to(dev)
    if dev == "cuda":
        torch.cuda.synchronize()
    t = time.perf_counter()
    m.fit(rows=r)
    if dev == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t
    s = m.decision_function(rows=test.to(dev)).cpu()
    yy = (test.y > 0).float()
    return torch.nn.functional.binary_cross_entropy_with_logits(s, yy).item(), rows.n / dt


def main():
    """argv: rows, then rule option strings; HM_RULE_WAVES="512,128,32" sweeps the rows in flight
    of the GPU engine (default: the engine's own choice for the rule)."""
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    rules = sys.argv[2:] or RULES
    waves = [int(w) for w in os.environ.get("HM_RULE_WAVES", "0").split(",")]
    rows = rows_of(n, 24, 5)
    test = rows_of(100_000, 24, 99)
    for opts in rules:
        ll_c, _ = run(opts, rows, test, "cpu")
        for w in waves:
            ll_g, rps = run(opts, rows, test, "cuda", waves=w)
            print(json.dumps({"opts": opts, "rows": n, "waves": w or "auto", "seq_cpu": round(ll_c, 5),
                              "gpu": round(ll_g, 5), "delta": round(ll_g - ll_c, 5),
                              "rows_per_s": round(rps)}), flush=True)


if __name__ == "__main__":
    main()
