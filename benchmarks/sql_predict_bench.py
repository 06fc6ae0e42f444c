"""Hivemall's SQL prediction pipeline, fused vs generic.

    CREATE TABLE test_exploded AS SELECT rowid, label, extract_feature(fv) AS feature,
           extract_weight(fv) AS value FROM test LATERAL VIEW explode(features) t AS fv;
    SELECT t.rowid, sigmoid(sum(m.weight * t.value)) AS prob, max(t.label) AS label
    FROM test_exploded t LEFT OUTER JOIN model m ON (t.feature = m.feature) GROUP BY t.rowid

Test rows carry 39 ``"feature:value"`` strings (Zipf feature ids over 2^20), the model table has
one weight per feature.  Times the explode step and the join-predict step separately, with the
fused operator (on the session device) and the generic join + GROUP BY path (HM_SQL_FUSED=0, on
fewer rows: it is the slow one), and checks that both give the same predictions.

    python benchmarks/sql_predict_bench.py --rows 1000000 --generic-rows 100000 [--device cuda]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NF, F = 1 << 20, 39


def tables(n, seed=0):
    rng = np.random.default_rng(seed)
    ids = np.minimum(rng.zipf(1.2, size=(n, F)), NF - 1)
    vals = np.round(rng.random((n, F)) * 2, 3)
    flat = (pd.Series(ids.reshape(-1).astype(str), dtype=object) + ":" +
            pd.Series(vals.reshape(-1).astype(str), dtype=object)).to_numpy()
    feats = [list(flat[i * F:(i + 1) * F]) for i in range(n)]
    test = pd.DataFrame({"rowid": np.arange(n), "features": feats, "label": rng.integers(0, 2, n)})
    model = pd.DataFrame({"feature": np.arange(0, NF, 3).astype(str),
                          "weight": rng.normal(size=len(range(0, NF, 3))).astype(np.float32)})
    return test, model


def run(n, fused, device):
    import torch

    from hivemall_amd.sql import Session

    os.environ["HM_SQL_FUSED"] = "1" if fused else "0"
    test, model = tables(n)
    s = Session(device=device)
    s.register("test", test)
    s.register("model", model)
    t0 = time.perf_counter()
    s.sql("""CREATE TABLE test_exploded AS SELECT rowid, label, extract_feature(fv) AS feature,
             extract_weight(fv) AS value FROM test LATERAL VIEW explode(features) t AS fv""")
    t1 = time.perf_counter()
    s.last_plan = None
    out = s.sql("""SELECT t.rowid, sigmoid(sum(m.weight * t.value)) AS prob, max(t.label) AS label
                   FROM test_exploded t LEFT OUTER JOIN model m ON (t.feature = m.feature)
                   GROUP BY t.rowid""")
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t2 = time.perf_counter()
    return out, {"rows": n, "exploded_rows": n * F, "fused": fused, "plan": s.last_plan, "device": str(s.device),
                 "explode_s": round(t1 - t0, 3), "join_predict_s": round(t2 - t1, 3),
                 "join_predict_rows_per_s": round(n / (t2 - t1)), "end_to_end_rows_per_s": round(n / (t2 - t0))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--generic-rows", type=int, default=50_000)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    out_f, r = run(a.rows, True, a.device)
    print(json.dumps(r), flush=True)
    if a.generic_rows:
        small_f, _ = run(a.generic_rows, True, a.device)
        small_g, rg = run(a.generic_rows, False, a.device)
        print(json.dumps(rg), flush=True)
        d = np.abs(small_f.set_index("rowid")["prob"].sort_index().to_numpy()
                   - small_g.set_index("rowid")["prob"].sort_index().to_numpy()).max()
        print(json.dumps({"fused_vs_generic_max_abs_diff": float(d), "rows": a.generic_rows}), flush=True)


if __name__ == "__main__":
    main()
