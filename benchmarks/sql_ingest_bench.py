"""End-to-end HiveQL ``train_ffm`` over Criteo-like STRING rows.

Builds an Arrow-backed table ``t(features array<string>, label int)`` of N rows with 39
Criteo-shaped ``field:index[:value]`` strings per row (13 numeric fields with a value, 26
categorical without), registers it in a ``Session`` and runs

    SELECT train_ffm(features, label, '-c -feature_hashing 20 -num_fields 39 -iters E ...') FROM t

The learner gets the Arrow column as is (functions._column), ingest.ffm_ell_device stages
its buffers through pinned double-buffered H2D and parses/hashes them with ``hm_ffm_parse``.
Reports end-to-end rows/s and the host/device split (ingest.LAST_STATS), and optionally the
same statement with the host parser (HM_INGEST_HOST=1) on a smaller table.

    python benchmarks/sql_ingest_bench.py --rows 5000000 --host-rows 200000
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.compute as pc

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NUM, CAT = 13, 26


def criteo_strings(n: int, seed: int = 0) -> tuple[pa.Array, np.ndarray]:
    """n rows x 39 strings; built column-wise with Arrow compute (C++), no per-string Python."""
    rng = np.random.default_rng(seed)
    F = NUM + CAT
    # large_string: 39 strings x 5M rows is more than the 2 GiB a 32-bit-offset string array holds
    fields = pa.array(np.tile(np.arange(F, dtype=np.int64), n)).cast(pa.large_string())
    # categorical ids: Zipf-ish per-field vocabularies; numeric fields: log-binned ids
    ids = np.empty((n, F), dtype=np.int64)
    ids[:, :NUM] = np.minimum(rng.geometric(0.05, size=(n, NUM)), 200) + np.arange(NUM) * 1000
    ids[:, NUM:] = np.minimum(rng.zipf(1.3, size=(n, CAT)), 1 << 22) * 131 + np.arange(CAT) * 7919
    idx = pa.array(ids.reshape(-1)).cast(pa.large_string())
    vals = np.round(rng.lognormal(0.0, 1.0, size=(n, F)), 3)
    vstr = pa.array(vals.reshape(-1)).cast(pa.large_string())
    sep = pa.scalar(":", pa.large_string())
    fi = pc.binary_join_element_wise(fields, idx, sep)
    with_val = pc.binary_join_element_wise(fi, vstr, sep)
    is_num = pa.array(np.tile(np.arange(F) < NUM, n))
    flat = pc.if_else(is_num, with_val, fi)
    offs = pa.array(np.arange(0, n * F + 1, F, dtype=np.int32))
    lists = pa.ListArray.from_arrays(offs, flat)
    logit = (ids[:, NUM:] % 7 - 3).sum(1) * 0.05 - 1.0
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.int32)
    return lists, y


def run(n: int, iters: int, host: bool) -> dict:
    import torch

    from hivemall_amd.io import ingest
    from hivemall_amd.models.ffm import FFMTrainer
    from hivemall_amd.sql import Session

    phases = {}

    def timed(name, fn):
        def w(*a, **k):
            sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
            sync()
            t = time.perf_counter()
            r = fn(*a, **k)
            sync()
            phases[name] = phases.get(name, 0.0) + time.perf_counter() - t
            return r
        return w

    orig = {k: getattr(FFMTrainer, k) for k in ("prepare", "fit", "model_table")}
    for k, f in orig.items():
        setattr(FFMTrainer, k, timed(k, f))

    t0 = time.perf_counter()
    lists, y = criteo_strings(n)
    df = pd.DataFrame({"features": pd.Series(lists, dtype=pd.ArrowDtype(lists.type)), "label": y})
    gen_s = time.perf_counter() - t0
    s = Session(device="cuda" if torch.cuda.is_available() else "cpu")
    s.register("t", df)
    if host:
        os.environ["HM_INGEST_HOST"] = "1"
    try:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        tab = s.sql(f"SELECT train_ffm(features, label, '-c -feature_hashing 20 -num_fields 39 "
                    f"-iters {iters} -disable_cv -seed 3') FROM t")
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        total_s = time.perf_counter() - t1
    finally:
        os.environ.pop("HM_INGEST_HOST", None)
        for k, f in orig.items():
            setattr(FFMTrainer, k, f)
    phases = {k: round(v, 3) for k, v in phases.items()}
    phases["train_s"] = round(phases.get("fit", 0) - phases.get("prepare", 0), 3)
    st = ingest.LAST_STATS.as_dict()
    return {"rows": n, "iters": iters, "parser": "host" if host else "device", "gen_s": round(gen_s, 2),
            "sql_total_s": round(total_s, 3), "rows_per_s_end_to_end": round(n / total_s),
            "ingest": st, "ingest_rows_per_s": round(n / max(st["wall_s"], 1e-9)),
            "ingest_GBps": round(st["bytes"] / max(st["wall_s"], 1e-9) / 1e9, 3),
            "phases_s": phases, "train_rows_per_s": round(n * iters / max(phases["train_s"], 1e-9)),
            "model_rows": len(tab)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=5_000_000)
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--host-rows", type=int, default=0, help="also time the host parser on this many rows")
    a = ap.parse_args()
    print(json.dumps(run(a.rows, a.iters, host=False)), flush=True)
    if a.host_rows:
        print(json.dumps(run(a.host_rows, a.iters, host=True)), flush=True)
        print(json.dumps(run(a.host_rows, a.iters, host=False)), flush=True)


if __name__ == "__main__":
    main()
