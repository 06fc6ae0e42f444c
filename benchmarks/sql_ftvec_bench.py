"""HiveQL feature engineering + training on Criteo-shaped string rows:

    SELECT train_classifier(add_bias(feature_hashing(features)), label, '-loss logloss -opt adagrad')

Times the feature-engineering expressions alone (SELECT add_bias(feature_hashing(features)))
and the whole training statement, on an Arrow-backed table (list<string> column, as a Parquet
or Arrow source arrives) and on a table of Python lists.

    python benchmarks/sql_ftvec_bench.py [rows] [device] [arrow|lists|both]
"""
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import pyarrow as pa

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def table(n, arrow=True):
    from hivemall_amd.io.synthetic import criteo_like
    idx, y = criteo_like(n, 20, seed=1)
    idx = idx.numpy()
    # Criteo-shaped raw feature names "<field>#<value>" (categorical, hashed by the query)
    names = np.char.add(np.char.add(np.arange(39).astype(str)[None, :].repeat(n, 0), "#"), idx.astype(str))
    flat = pa.array(names.reshape(-1).astype(object), type=pa.string())
    col = pa.ListArray.from_arrays(pa.array(np.arange(0, n * 39 + 1, 39, dtype=np.int32)), flat)
    feats = pd.Series(pd.arrays.ArrowExtensionArray(col)) if arrow else pd.Series(col.to_pylist(), dtype=object)
    return pd.DataFrame({"features": feats, "label": (y.numpy() > 0).astype(np.int32)})


def main():
    from hivemall_amd.sql import Session
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    dev = sys.argv[2] if len(sys.argv) > 2 else "cpu"
    which = sys.argv[3] if len(sys.argv) > 3 else "both"
    for arrow in {"arrow": (True,), "lists": (False,)}.get(which, (True, False)):
        t = time.perf_counter()
        df = table(n, arrow)
        gen = time.perf_counter() - t
        s = Session(device=dev)
        s.register("criteo", df)
        t = time.perf_counter()
        fe = s.sql("SELECT add_bias(feature_hashing(features)) AS f FROM criteo")
        t_fe = time.perf_counter() - t
        from hivemall_amd.io import ingest

        res = {}
        tabs = {}
        # fused: feature_hashing + add_bias evaluated on the device into CSR (sql/device_ftvec.py);
        # strings: the column of hashed strings re-parsed by the learner (HM_SQL_DEVICE_FTVEC=0)
        for mode in (("fused", "strings") if dev.startswith("cuda") else ("strings",)):
            os.environ["HM_SQL_DEVICE_FTVEC"] = "1" if mode == "fused" else "0"
            for rep in range(2):                     # the first run pays one-time setup
                prof = None
                if rep == 1 and os.environ.get("HM_SQL_PROFILE") == "1":
                    import cProfile
                    prof = cProfile.Profile()
                    prof.enable()
                t = time.perf_counter()
                m = s.sql("SELECT train_classifier(add_bias(feature_hashing(features)), label, "
                          "'-loss logloss -opt adagrad') AS (feature, weight) FROM criteo")
                if dev.startswith("cuda"):
                    import torch
                    torch.cuda.synchronize()
                t_all = time.perf_counter() - t
                if prof is not None:
                    import io
                    import pstats
                    prof.disable()
                    buf = io.StringIO()
                    pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(30)
                    print(f"== profile {mode}\n" + buf.getvalue(), file=sys.stderr, flush=True)
            res[mode] = {"train_stmt_s": round(t_all, 3), "train_stmt_rows_per_s": round(n / t_all),
                         "ingest": ingest.LAST_STATS.as_dict()}
            tabs[mode] = m.sort_values("feature").reset_index(drop=True)
        same = None
        if len(tabs) == 2:
            # the timed default engine is Hogwild (two runs of one path differ in the last bits);
            # bit-identity of the two paths is checked on the deterministic replica engine
            det = {}
            for mode in ("fused", "strings"):
                os.environ["HM_SQL_DEVICE_FTVEC"] = "1" if mode == "fused" else "0"
                det[mode] = s.sql("SELECT train_classifier(add_bias(feature_hashing(features)), label, "
                                  "'-loss logloss -opt adagrad -engine replica -replicas 8') AS (feature, weight) "
                                  "FROM criteo").sort_values("feature").reset_index(drop=True)
            a, b = det["fused"], det["strings"]
            same = bool(len(a) == len(b) and (a["feature"].to_numpy() == b["feature"].to_numpy()).all()
                        and (a["weight"].to_numpy() == b["weight"].to_numpy()).all())
            os.environ["HM_SQL_DEVICE_FTVEC"] = "1"
        print(json.dumps({"rows": n, "device": dev, "table": "arrow list<string>" if arrow else "python lists",
                          "gen_s": round(gen, 2), "feature_eng_s": round(t_fe, 3),
                          "feature_eng_rows_per_s": round(n / t_fe), **res, "model_rows": len(m),
                          "model_tables_identical": same, "first": fe["f"].iloc[0][:3]}), flush=True)


if __name__ == "__main__":
    main()
