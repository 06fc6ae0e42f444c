"""Private-replica engine (Hivemall's per-mapper semantics) for the general learner's non-AdaGrad
rules at -dims 2^24.

For each rule and replica count R: one epoch of Criteo-shaped hashed rows (39 nnz) through
  * the sequential CPU engine (one learner over every row),
  * the R-mapper CPU average (R learners over contiguous shards, averaged: Hivemall's DP-1),
  * the GPU replica engine (-engine replica -replicas R: one wave per replica, the same per-row
    arithmetic as the CPU engine, averaged by hm_linear_mix),
  * the GPU shared-table engine at its default rows in flight (the round-4 routing),
and prints held-out logloss and rows/s as JSON lines.

    python benchmarks/linear_replica_probe.py [rows] [R,...] [opts...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from linear_rules_parity import rows_of  # noqa: E402

RULES = ["-opt adam -eta0 0.01", "-opt sgd -eta0 0.05", "-opt rmsprop -eta0 0.01", "-opt adadelta"]


def fit(opts, rows, test, dev):
    from hivemall_amd.models.linear import TrainClassifier

    m = TrainClassifier(f"-loss logloss {opts} -dims 16777216 -iters 1", device=dev)
    r = rows.to(dev)
    if dev == "cuda":
        torch.cuda.synchronize()
    t = time.perf_counter()
    m.fit(rows=r)
    if dev == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t
    s = m.decision_function(rows=test.to(dev)).cpu()
    ll = torch.nn.functional.binary_cross_entropy_with_logits(s, (test.y > 0).float()).item()
    eng = ("minibatch" if m.state.meta.get("minibatch") else
           "shared" if m.state.meta.get("shared") else f"replica{m.state.R}")
    del m
    if dev == "cuda":
        torch.cuda.empty_cache()
    return ll, rows.n / dt, eng


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    Rs = [int(r) for r in (sys.argv[2] if len(sys.argv) > 2 else "64,128").split(",") if r]
    rules = sys.argv[3:] or RULES
    Ms = [int(m) for m in os.environ.get("HM_PROBE_MB", "").split(",") if m]
    rows = rows_of(n, 24, 5)
    test = rows_of(100_000, 24, 99)
    # -mini_batch M: the sequential mini-batch learner (CPU, one replica) vs the GPU mini-batch engine
    for opts in rules:
        for M in Ms:
            o = f"{opts} -mini_batch {M}"
            seqm, seqm_rate, _ = fit(o + " -replicas 1", rows, test, "cpu")
            g, rate, eng = fit(o, rows, test, "cuda")
            print(json.dumps({"opts": o, "rows": n, "engine": eng, "seq_cpu_minibatch": round(seqm, 5),
                              "gpu": round(g, 5), "delta": round(g - seqm, 5), "rows_per_s": round(rate),
                              "seq_rows_per_s": round(seqm_rate)}), flush=True)
    if not Rs:
        return
    for opts in rules:
        seq, seq_rate, _ = fit(opts, rows, test, "cpu")
        sh, sh_rate, sh_eng = fit(opts, rows, test, "cuda")
        print(json.dumps({"opts": opts, "rows": n, "engine": sh_eng, "seq_cpu": round(seq, 5),
                          "gpu": round(sh, 5), "delta_seq": round(sh - seq, 5),
                          "rows_per_s": round(sh_rate), "seq_rows_per_s": round(seq_rate)}), flush=True)
        for R in Rs:
            avg, _, _ = fit(f"{opts} -engine replica -replicas {R}", rows, test, "cpu")
            g, rate, eng = fit(f"{opts} -engine replica -replicas {R}", rows, test, "cuda")
            print(json.dumps({"opts": opts, "rows": n, "engine": eng, "seq_cpu": round(seq, 5),
                              f"avg{R}_cpu": round(avg, 5), "gpu": round(g, 5),
                              "delta_seq": round(g - seq, 5), "delta_avg": round(g - avg, 5),
                              "rows_per_s": round(rate)}), flush=True)


if __name__ == "__main__":
    main()
