"""Fused join-predict for the SQL executor (SURVEY.md §2.5 K13, §3.1 "prediction" queries).

Hivemall scores a test set by exploding it to one row per feature, joining the model table
and aggregating per test row:

    SELECT t.rowid, sigmoid(sum(m.weight * t.value)) AS prob, max(t.label) AS label
    FROM test_exploded t LEFT OUTER JOIN model m ON (t.feature = m.feature)
    GROUP BY t.rowid

    SELECT t.rowid, fm_predict(m.Wi, m.Vif, t.Xi) FROM (...) t
    LEFT OUTER JOIN fm_model m ON (t.feature = m.feature) GROUP BY t.rowid

The generic executor materialises the joined table (an object-typed row per exploded row) and
reduces it group by group.  This operator recognises the shape — a LEFT/INNER equi-join of two
sources, GROUP BY columns of the left side, aggregates that are ``sum(<model col> * <test
col>)``, ``fm_predict(<model W>, <model V>, <test x>)`` or plain aggregates of test columns —
resolves the join to a model-row index per test row with one hash lookup (model keys must be
unique) and runs the gather / multiply / per-group reduction in one pass on the session device
(``ops.join_predict``: gfx950 kernels on a GPU session).  The output — values, row order, NULL
handling — is the generic path's (tests/test_sql_fused.py compares the two); anything outside
the shape falls back to the generic path.  ``HM_SQL_FUSED=0`` disables it.
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd

from .parser import BinOp, Col, Func, Join, Lit

# agg kinds: ("dot", model_col, test_col) | ("fm", W, V, x) | ("test", None) | ("count_star",)


def enabled() -> bool:
    return os.environ.get("HM_SQL_FUSED", "1") != "0"


def _aggs_of(session, s):
    from .executor import _collect_aggs

    aggs = []
    for it in s.items:
        _collect_aggs(it.expr, session, aggs)
    for e, _ in s.order_by:
        _collect_aggs(e, session, aggs)
    return aggs


def _cols_outside_aggs(e, aggs_ids, out):
    from .executor import _children

    if id(e) in aggs_ids:
        return
    if isinstance(e, Col):
        out.append(e)
        return
    for ch in _children(e):
        _cols_outside_aggs(ch, aggs_ids, out)


def _syntactic_ok(session, s) -> bool:
    j = s.source
    if not (isinstance(j, Join) and j.kind in ("left", "inner") and isinstance(j.on, BinOp)
            and j.on.op == "=" and isinstance(j.on.left, Col) and isinstance(j.on.right, Col)):
        return False
    if isinstance(j.left, Join) or isinstance(j.right, Join):
        return False
    if s.where is not None or s.having is not None or s.distinct or not s.group_by:
        return False
    if not all(isinstance(g, Col) for g in s.group_by):
        return False
    aggs = _aggs_of(session, s)
    if not aggs:
        return False
    for a in aggs:
        n = a.name.lower()
        if a.distinct or a.window is not None:
            return False
        if n == "count" and (a.star or not a.args):
            continue
        if n == "sum" and len(a.args) == 1 and isinstance(a.args[0], BinOp) and a.args[0].op == "*" \
                and isinstance(a.args[0].left, Col) and isinstance(a.args[0].right, Col):
            continue
        if n == "fm_predict" and len(a.args) == 3 and all(isinstance(x, Col) for x in a.args):
            continue
        if n in ("sum", "max", "min", "avg", "mean", "count") and len(a.args) == 1 and isinstance(a.args[0], Col):
            continue
        return False
    return True


def _side(col: Col, L, R):
    """'L' / 'R' / None for a column reference (None: unresolvable or on both sides)."""
    from .executor import SQLError

    try:
        li = L.resolve(col.name, col.table)
    except SQLError:
        return None, None
    try:
        ri = R.resolve(col.name, col.table)
    except SQLError:
        return None, None
    if (li is None) == (ri is None):
        return None, None
    return ("L", li) if li is not None else ("R", ri)


def _key_arrays(lk: pd.Series, rk: pd.Series):
    """Join keys comparable the way the generic join compares them, or None (fall back)."""
    num_l, num_r = pd.api.types.is_numeric_dtype(lk), pd.api.types.is_numeric_dtype(rk)
    if num_l and num_r and not pd.api.types.is_bool_dtype(lk) and not pd.api.types.is_bool_dtype(rk):
        return lk.astype(np.float64), rk.astype(np.float64)
    if lk.dtype == object and rk.dtype == object:
        sl, sr = lk.dropna(), rk.dropna()
        if sl.map(type).eq(str).all() and sr.map(type).eq(str).all():
            return lk, rk
    return None


def try_fused(session, s, ctes):
    """Run ``s`` through the fused operator; returns the result Frame, or None after stashing
    the already-built join inputs for the generic path."""
    if not enabled() or not _syntactic_ok(session, s):
        return None
    from .executor import Frame, _GroupBase
    from ..ops.join_predict import join_dot, join_fm

    j = s.source
    L = session._source(j.left, ctes)
    R = session._source(j.right, ctes)

    def fallback():
        session._prebuilt[id(j)] = (L, R)
        return None

    sa, sb = _side(j.on.left, L, R), _side(j.on.right, L, R)
    if sa[0] == "L" and sb[0] == "R":
        lki, rki = sa[1], sb[1]
    elif sa[0] == "R" and sb[0] == "L":
        lki, rki = sb[1], sa[1]
    else:
        return fallback()
    gcols = []
    for gc in s.group_by:
        side = _side(gc, L, R)
        if side[0] != "L":
            return fallback()
        gcols.append(side[1])
    aggs = _aggs_of(session, s)
    ids = {id(a) for a in aggs}
    bare = []
    for it in s.items:
        _cols_outside_aggs(it.expr, ids, bare)
    gset = {(c.name.lower(), (c.table or "").lower()) for c in s.group_by}
    for c in bare:
        if (c.name.lower(), (c.table or "").lower()) not in gset and _side(c, L, R)[0] != "L":
            return fallback()
    specs = []
    for a in aggs:
        n = a.name.lower()
        if n == "count" and (a.star or not a.args):
            specs.append(("count_star",))
        elif n == "sum" and isinstance(a.args[0], BinOp):
            x, y = _side(a.args[0].left, L, R), _side(a.args[0].right, L, R)
            if x[0] == "R" and y[0] == "L":
                specs.append(("dot", x[1], y[1]))
            elif x[0] == "L" and y[0] == "R":
                specs.append(("dot", y[1], x[1]))
            else:
                return fallback()
        elif n == "fm_predict":
            w, v, xx = (_side(c, L, R) for c in a.args)
            if not (w[0] == "R" and v[0] == "R" and xx[0] == "L"):
                return fallback()
            specs.append(("fm", w[1], v[1], xx[1]))
        else:
            if _side(a.args[0], L, R)[0] != "L":
                return fallback()
            specs.append(("test",))

    # ---- resolve the join: model row per test row (model keys unique, NULL keys never match)
    keys = _key_arrays(L.series(lki), R.series(rki))
    if keys is None:
        return fallback()
    lk, rk = keys
    rnn = rk.notna().to_numpy()
    rpos = np.nonzero(rnn)[0]
    ridx = pd.Index(rk[rnn].to_numpy())
    if not ridx.is_unique:
        return fallback()
    tm = ridx.get_indexer(lk.to_numpy())
    tm = np.where(lk.notna().to_numpy() & (tm >= 0), rpos[np.maximum(tm, 0)], -1).astype(np.int32)
    # ---- numeric operands (else the generic path decides what the SQL means)
    arrays = {}
    for sp in specs:
        if sp[0] == "dot":
            mw, tv = R.series(sp[1]), L.series(sp[2])
            if not (pd.api.types.is_numeric_dtype(mw) and pd.api.types.is_numeric_dtype(tv)):
                return fallback()
        elif sp[0] == "fm":
            mw, mv, tx = R.series(sp[1]), R.series(sp[2]), L.series(sp[3])
            if not (pd.api.types.is_numeric_dtype(mw) and pd.api.types.is_numeric_dtype(tx)) or tx.isna().any():
                return fallback()
            vl = mv.tolist()
            ks = {len(v) for v in vl if v is not None and not isinstance(v, float)}
            if len(ks) != 1 or any(isinstance(v, float) and not np.isnan(v) for v in vl):
                return fallback()
            k = ks.pop()
            vmask = np.array([v is not None and not isinstance(v, float) for v in vl], dtype=bool)
            V = np.zeros((len(vl), k), dtype=np.float32)
            if vmask.any():
                V[vmask] = np.asarray([v for v, m in zip(vl, vmask) if m], dtype=np.float32)
            arrays[id(sp)] = (V, vmask)

    # ---- joined row order of the generic path: matched test rows (test order), then for a
    # LEFT join the unmatched ones; groups numbered by first appearance in that order
    matched = np.nonzero(tm >= 0)[0]
    if j.kind == "left":
        order_rows = np.concatenate([matched, np.nonzero(tm < 0)[0]])
    else:
        order_rows = matched
    Lj = L.take(order_rows)
    if len(gcols) == 1:
        codes = pd.factorize(Lj.series(gcols[0]), use_na_sentinel=False)[0]
    else:
        kdf = pd.DataFrame({f"k{i}": Lj.series(c) for i, c in enumerate(gcols)})
        codes = kdf.groupby(list(kdf.columns), sort=False, dropna=False).ngroup().to_numpy()
    codes = codes.astype(np.int64)
    n_groups = int(codes.max()) + 1 if len(codes) else 0
    order = np.argsort(codes, kind="stable")
    bounds = np.searchsorted(codes[order], np.arange(n_groups + 1))
    first_idx = order[bounds[:-1]] if len(codes) else np.zeros(0, dtype=np.int64)
    gframe = Lj.take(first_idx)
    tmj = tm[order_rows]
    g32 = codes.astype(np.int32)
    dev = session.device
    agg_values = {}
    for a, sp in zip(aggs, specs):
        if sp[0] == "count_star":
            agg_values[id(a)] = pd.Series(np.diff(bounds))
        elif sp[0] == "test":
            agg_values[id(a)] = session._agg_values(a, Lj, ctes, order, bounds, n_groups, codes)
        elif sp[0] == "dot":
            W = R.series(sp[1]).to_numpy(dtype=np.float32, na_value=np.nan)
            v = Lj.series(sp[2]).to_numpy(dtype=np.float32, na_value=np.nan)
            ssum, _ = join_dot(tmj, v, g32, W, n_groups, dev)
            agg_values[id(a)] = pd.Series(ssum)       # pandas SUM: all-NULL group -> 0.0
        else:
            V, vmask = arrays[id(sp)]
            W = R.series(sp[1]).to_numpy(dtype=np.float32, na_value=np.nan)
            x = Lj.series(sp[3]).to_numpy(dtype=np.float32)
            agg_values[id(a)] = pd.Series(join_fm(tmj, x, g32, W, V, vmask, n_groups, dev))
    session.last_plan = "fused_join_predict"
    out = session._project(s.items, gframe, ctes, agg_values)
    base = _GroupBase(gframe, agg_values, session)
    return session._finish(out, base, s, ctes)
