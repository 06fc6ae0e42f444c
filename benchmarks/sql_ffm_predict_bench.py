"""Fused vs generic FFM scoring query (sql/fused.try_fused_ffm):

    SELECT t.rowid, sigmoid(ffm_predict(m1.Wi, m1.Vi, m2.Vi, t.Xi, t.Xj)) FROM tp t
    LEFT OUTER JOIN ffm_model m1 ON (t.i = m1.i) LEFT OUTER JOIN ffm_model m2 ON (t.j = m2.i)
    GROUP BY t.rowid

over ``--rows`` test rows of ``--fields`` fields (feature_pairs('-ffm') gives fields*(fields+1)/2
+ 1 exploded rows each).  Times the query only (the exploded table is built beforehand),
fused on the session device and, unless ``--generic 0``, the generic join + GROUP BY path.

    python benchmarks/sql_ffm_predict_bench.py --rows 100000 --fields 10 [--device cuda]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hivemall_amd.sql import Session  # noqa: E402

Q = """
SELECT t.rowid, sigmoid(ffm_predict(m1.Wi, m1.Vi, m2.Vi, t.Xi, t.Xj)) AS p FROM tp t
LEFT OUTER JOIN ffm_model m1 ON (t.i = m1.i)
LEFT OUTER JOIN ffm_model m2 ON (t.j = m2.i)
GROUP BY t.rowid"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100000)
    ap.add_argument("--fields", type=int, default=10)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--generic", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    nf = a.fields
    rows = [[f"{f}:{int(rng.integers(0, 1000))}:1" for f in range(nf)] for _ in range(a.rows)]
    y = (rng.random(a.rows) < 0.3).astype(int)
    opts = f"-c -factors 4 -num_fields {nf} -feature_hashing 16 -iters 1"
    base = Session(device="cpu")
    base.register("t", pd.DataFrame({"rowid": range(a.rows), "features": rows, "label": y}))
    t0 = time.perf_counter()
    model = base.sql(f"SELECT train_ffm(features, label, '{opts}') AS (model_id, i, Wi, Vi) FROM t")
    t1 = time.perf_counter()
    tp = base.sql(f"SELECT rowid, i, j, Xi, Xj FROM t LATERAL VIEW feature_pairs(features, "
                  f"'-ffm -feature_hashing 16 -num_fields {nf}') x AS i, j, Xi, Xj")
    t2 = time.perf_counter()
    s = Session(device=a.device)
    s.register("ffm_model", model)
    s.register("tp", tp)
    res = {"rows": a.rows, "fields": nf, "exploded_rows": len(tp), "model_rows": len(model),
           "device": a.device, "train_s": round(t1 - t0, 3), "feature_pairs_s": round(t2 - t1, 3)}
    fused = []
    for _ in range(a.reps):
        s.last_plan = None
        t0 = time.perf_counter()
        pf = s.sql(Q)
        fused.append(time.perf_counter() - t0)
        assert s.last_plan == "fused_ffm_join_predict", s.last_plan
    res["fused_s"] = round(min(fused), 4)
    res["fused_exploded_rows_per_s"] = round(len(tp) / min(fused))
    if a.generic:
        os.environ["HM_SQL_FUSED"] = "0"
        s.last_plan = None
        t0 = time.perf_counter()
        pg = s.sql(Q)
        res["generic_s"] = round(time.perf_counter() - t0, 3)
        os.environ.pop("HM_SQL_FUSED")
        res["speedup"] = round(res["generic_s"] / res["fused_s"], 1)
        m = pf.merge(pg, on="rowid")
        res["max_abs_diff"] = float(np.abs(m["p_x"] - m["p_y"]).max())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
