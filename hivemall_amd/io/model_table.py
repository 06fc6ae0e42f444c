"""Model-table dump / load — the checkpoint and interchange format.

Upstream the model table *is* the checkpoint: ``close()`` forwards the rows and Hive writes
them; scoring is plain SQL over them, and ``-loadmodel`` warm-starts from a file.  Here a
model table is a pandas DataFrame with the Hivemall column layout, written as

* ``.parquet`` (default; array columns stay arrays),
* ``.tsv`` / ``.txt`` (Hive text layout: array elements joined with ``,``; ``\\N`` for NULL),
* ``.csv``.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pandas as pd


def _is_array_col(s: pd.Series) -> bool:
    for v in s:
        if v is None or (isinstance(v, float) and np.isnan(v)):
            continue
        return isinstance(v, (list, tuple, np.ndarray))
    return False


def write_table(df: pd.DataFrame, path: str) -> str:
    ext = os.path.splitext(path)[1].lower()
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    if ext in (".parquet", ".pq", ""):
        out = df.copy()
        for c in out.columns:
            if _is_array_col(out[c]):
                out[c] = [None if v is None else np.asarray(v).tolist() for v in out[c]]
        out.to_parquet(path if ext else path + ".parquet", index=False)
        return path if ext else path + ".parquet"
    sep = "\t" if ext in (".tsv", ".txt") else ","
    out = df.copy()
    for c in out.columns:
        if _is_array_col(out[c]):
            out[c] = ["\\N" if v is None else ",".join(repr(float(x)) for x in np.asarray(v).ravel())
                      for v in out[c]]
    meta = {"columns": list(df.columns),
            "arrays": [c for c in df.columns if _is_array_col(df[c])]}
    with open(path, "w") as f:
        f.write("#hivemall_amd " + json.dumps(meta) + "\n")
        out.to_csv(f, sep=sep, index=False, header=False, na_rep="\\N",
                   quoting=3 if sep == "\t" else 0, escapechar="\\" if sep == "\t" else None)
    return path


def read_table(path: str) -> pd.DataFrame:
    ext = os.path.splitext(path)[1].lower()
    if ext in (".parquet", ".pq"):
        df = pd.read_parquet(path)
        for c in df.columns:
            if _is_array_col(df[c]):
                df[c] = [None if v is None else np.asarray(v, dtype=np.float32) for v in df[c]]
        return df
    sep = "\t" if ext in (".tsv", ".txt") else ","
    with open(path) as f:
        first = f.readline()
    meta = None
    skip = 0
    if first.startswith("#hivemall_amd "):
        meta = json.loads(first[len("#hivemall_amd "):])
        skip = 1
    df = pd.read_csv(path, sep=sep, header=None, skiprows=skip, na_values=["\\N"],
                     keep_default_na=False, quoting=3 if sep == "\t" else 0)
    if meta:
        df.columns = meta["columns"]
        for c in meta["arrays"]:
            df[c] = [None if (isinstance(v, float) and np.isnan(v)) else
                     np.array([float(x) for x in str(v).split(",") if x != ""], dtype=np.float32)
                     for v in df[c]]
    else:
        df.columns = ["feature", "weight", "covar"][: df.shape[1]] if df.shape[1] <= 3 else \
            [f"c{i}" for i in range(df.shape[1])]
    return df
