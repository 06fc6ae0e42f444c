"""DataFrame DSL — the analogue of Hivemall's Spark ``HivemallOps`` (SURVEY.md §2.1:
spark/spark-common HivemallOps.scala, HivemallGroupedDataset.scala).

Every registered SQL function is available on pandas objects through the ``hivemall``
accessor, with the SQL argument order::

    import hivemall_amd.dsl  # registers the accessor
    model = train.hivemall.train_classifier("features", "label", "-loss logloss -opt adagrad")
    train["features"] = train.hivemall.add_bias("features")
    scores.groupby("rowid").hivemall.auc("prob", "label")      # UDAF per group

* UDF  -> Series (one value per row; vectorised UDFs receive whole columns)
* UDTF -> DataFrame (learners return their model table; per-row UDTFs explode)
* UDAF -> scalar on a DataFrame, Series on a GroupBy
Column arguments are column names; anything else is passed as a constant.
"""
from __future__ import annotations

import pandas as pd

from . import registry


def _resolve(df: pd.DataFrame, args):
    out = []
    for a in args:
        if isinstance(a, str) and a in df.columns:
            out.append(df[a])
        elif isinstance(a, pd.Series):
            out.append(a)
        else:
            out.append(a)
    return out


def _call(fd, df: pd.DataFrame, args, device=None):
    cols = _resolve(df, args)
    n = len(df)
    if fd.kind == registry.UDF:
        if fd.vectorized:
            res = fd.impl(*cols)
            return pd.Series(list(res) if not isinstance(res, pd.Series) else res, index=df.index)
        lists = [c.tolist() if isinstance(c, pd.Series) else None for c in cols]
        vals = [fd.impl(*[l[i] if l is not None else c for l, c in zip(lists, cols)]) for i in range(n)]
        return pd.Series(vals, index=df.index, dtype=object).infer_objects()
    if fd.kind == registry.UDAF:
        lists = [c.tolist() if isinstance(c, pd.Series) else [c] * n for c in cols]
        return fd.impl(*lists)
    # UDTF
    lists = [c.tolist() if isinstance(c, pd.Series) else [c] * n for c in cols]
    if fd.per_row:
        rows = []
        for i in range(n):
            rows.extend(tuple(t) for t in fd.impl(*[l[i] for l in lists]))
        names = list(fd.cols) if fd.cols else None
        df_out = pd.DataFrame(rows)
        if names and len(names) == df_out.shape[1]:
            df_out.columns = names
        return df_out
    kw = {}
    if getattr(fd.impl, "wants_session", False):
        kw["session"] = _DeviceSession(device)
    return fd.impl(*lists, **kw)


class _DeviceSession:
    def __init__(self, device):
        self.device = device


@pd.api.extensions.register_dataframe_accessor("hivemall")
class HivemallFrameAccessor:
    def __init__(self, df: pd.DataFrame):
        self._df = df
        self.device = None

    def on(self, device) -> "HivemallFrameAccessor":
        """Select the device learners run on (``df.hivemall.on('cuda').train_fm(...)``)."""
        self.device = device
        return self

    def __getattr__(self, name):
        fd = registry.lookup(name)
        if fd is None:
            raise AttributeError(f"no Hivemall function '{name}'")
        return lambda *args: _call(fd, self._df, args, self.device)

    def __dir__(self):
        return registry.names()


class _GroupedAccessor:
    def __init__(self, gb):
        self._gb = gb

    def __getattr__(self, name):
        fd = registry.lookup(name)
        if fd is None or fd.kind != registry.UDAF:
            raise AttributeError(f"no Hivemall aggregate '{name}'")

        def agg(*args):
            return self._gb.apply(lambda g: _call(fd, g, args), include_groups=False)
        return agg


def _grouped(self):
    return _GroupedAccessor(self)


pd.core.groupby.DataFrameGroupBy.hivemall = property(_grouped)
