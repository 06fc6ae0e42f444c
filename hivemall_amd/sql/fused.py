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
        return False       # the two-join FFM shape goes through try_fused_ffm
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
    if enabled() and isinstance(s.source, Join) and isinstance(s.source.left, Join):
        return try_fused_ffm(session, s, ctes)
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


# ------------------------------------------------------------------ FFM: two model joins
#   SELECT t.rowid, ffm_predict(m1.Wi, m1.Vi, m2.Vi, t.Xi, t.Xj) FROM (... feature_pairs(
#     features, '-ffm') ...) t LEFT OUTER JOIN m m1 ON (t.i = m1.i) LEFT OUTER JOIN m m2 ON
#   (t.j = m2.i) GROUP BY t.rowid
def _eqjoin(j) -> bool:
    return (isinstance(j, Join) and j.kind in ("left", "inner") and isinstance(j.on, BinOp)
            and j.on.op == "=" and isinstance(j.on.left, Col) and isinstance(j.on.right, Col))


def _ffm_syntactic_ok(session, s) -> bool:
    j2 = s.source
    j1 = j2.left if isinstance(j2, Join) else None
    if not (_eqjoin(j2) and _eqjoin(j1)) or isinstance(j2.right, Join) \
            or isinstance(j1.left, Join) or isinstance(j1.right, Join):
        return False
    if s.where is not None or s.having is not None or s.distinct or not s.group_by:
        return False
    if not all(isinstance(g, Col) for g in s.group_by):
        return False
    aggs = _aggs_of(session, s)
    n_ffm = 0
    for a in aggs:
        n = a.name.lower()
        if a.distinct or a.window is not None:
            return False
        if n == "ffm_predict" and len(a.args) == 5 and all(isinstance(x, Col) for x in a.args):
            n_ffm += 1
            continue
        if n == "count" and (a.star or not a.args):
            continue
        if n in ("sum", "max", "min", "avg", "mean", "count") and len(a.args) == 1 and isinstance(a.args[0], Col):
            continue
        return False
    return n_ffm >= 1


def _which(col: Col, frames):
    """Index of the one frame that resolves ``col`` (None: unresolvable or ambiguous) and the
    column position in it."""
    from .executor import SQLError

    hits = []
    for fi, fr in enumerate(frames):
        try:
            ci = fr.resolve(col.name, col.table)
        except SQLError:
            return None, None
        if ci is not None:
            hits.append((fi, ci))
    return hits[0] if len(hits) == 1 else (None, None)


def _int_keys(s: pd.Series):
    """int64 keys of an all-integral, NULL-free numeric column (else None)."""
    if not pd.api.types.is_numeric_dtype(s) or pd.api.types.is_bool_dtype(s):
        return None
    a = s.to_numpy()
    if a.dtype.kind in "iu":
        return a.astype(np.int64, copy=False)
    if a.dtype.kind == "f" and not np.isnan(a).any() and np.all(a == np.round(a)) \
            and (a.size == 0 or np.abs(a).max() < 2.0 ** 53):
        return a.astype(np.int64)
    return None


def _join_index(lk: pd.Series, rk: pd.Series):
    """Model row per test row (-1: none; NULL keys never match), or None when the model keys
    are not unique or not comparable (the generic join decides then).  Integer keys (the
    feature / V(feature, field) keys of the linear, FM and FFM model tables) resolve through
    the native open-addressing table (utils.collections.Int2LongOpenHashTable); NULL test keys
    (NaN) are mapped to a key no model row holds."""
    from ..utils.collections import Int2LongOpenHashTable

    rki = _int_keys(rk)
    if rki is not None and rki.size and not (rki == np.iinfo(np.int64).min).any():
        lnull = lk.isna().to_numpy()
        lki = _int_keys(lk.fillna(0)) if pd.api.types.is_numeric_dtype(lk) else None
        if lki is not None:
            tab = Int2LongOpenHashTable(rki.size)
            if len(np.unique(rki)) != rki.size:
                return None
            tab.put_many(rki, np.arange(rki.size, dtype=np.int64))
            tm = tab.get_many(lki, default=-1)
            tm[lnull] = -1
            return tm.astype(np.int32)
    keys = _key_arrays(lk, rk)
    if keys is None:
        return None
    lk, rk = keys
    rnn = rk.notna().to_numpy()
    rpos = np.nonzero(rnn)[0]
    ridx = pd.Index(rk[rnn].to_numpy())
    if not ridx.is_unique:
        return None
    tm = ridx.get_indexer(lk.to_numpy())
    return np.where(lk.notna().to_numpy() & (tm >= 0), rpos[np.maximum(tm, 0)], -1).astype(np.int32)


def _v_matrix(col: pd.Series):
    """list column -> (V f32 [R, k], row mask) or None when the lists disagree on k."""
    vl = col.tolist()
    null = [v is None or v is pd.NA or (isinstance(v, float) and np.isnan(v)) for v in vl]
    if any(not n and not isinstance(v, (list, tuple, np.ndarray)) for v, n in zip(vl, null)):
        return None
    ks = {len(v) for v, n in zip(vl, null) if not n}
    if len(ks) > 1:
        return None
    k = ks.pop() if ks else 1
    vmask = ~np.asarray(null, dtype=bool)
    V = np.zeros((len(vl), k), dtype=np.float32)
    if vmask.any():
        V[vmask] = np.asarray([v for v, m in zip(vl, vmask) if m], dtype=np.float32)
    return V, vmask


def try_fused_ffm(session, s, ctes):
    """The FFM scoring query as one gather-reduce (``ops.join_predict.join_ffm``): both joins
    resolve to a model-row index per exploded test row; no joined table is materialised."""
    if not _ffm_syntactic_ok(session, s):
        return None
    from .executor import Frame, _GroupBase
    from ..ops.join_predict import join_ffm

    j2 = s.source
    j1 = j2.left
    T = session._source(j1.left, ctes)
    M1 = session._source(j1.right, ctes)

    def fallback():
        session._prebuilt[id(j1)] = (T, M1)
        return None

    M2 = session._source(j2.right, ctes)
    frames = (T, M1, M2)
    # join 1: T x M1; join 2: (T, M1) x M2 with the left key on T
    a, b = _which(j1.on.left, frames), _which(j1.on.right, frames)
    if {a[0], b[0]} != {0, 1}:
        return fallback()
    t1, m1k = (a[1], b[1]) if a[0] == 0 else (b[1], a[1])
    a, b = _which(j2.on.left, frames), _which(j2.on.right, frames)
    if {a[0], b[0]} != {0, 2}:
        return fallback()
    t2, m2k = (a[1], b[1]) if a[0] == 0 else (b[1], a[1])
    gcols = []
    for gc in s.group_by:
        w = _which(gc, frames)
        if w[0] != 0:
            return fallback()
        gcols.append(w[1])
    aggs = _aggs_of(session, s)
    ids = {id(x) for x in aggs}
    bare = []
    for it in s.items:
        _cols_outside_aggs(it.expr, ids, bare)
    gset = {(c.name.lower(), (c.table or "").lower()) for c in s.group_by}
    for c in bare:
        if (c.name.lower(), (c.table or "").lower()) not in gset and _which(c, frames)[0] != 0:
            return fallback()
    specs = []
    for x in aggs:
        n = x.name.lower()
        if n == "ffm_predict":
            w = [_which(c, frames) for c in x.args]
            if [f for f, _ in w] != [1, 1, 2, 0, 0]:
                return fallback()
            specs.append(("ffm",) + tuple(c for _, c in w))
        elif n == "count" and (x.star or not x.args):
            specs.append(("count_star",))
        else:
            if _which(x.args[0], frames)[0] != 0:
                return fallback()
            specs.append(("test",))

    ti = _join_index(T.series(t1), M1.series(m1k))
    tj = _join_index(T.series(t2), M2.series(m2k))
    if ti is None or tj is None:
        return fallback()
    ffm_in = {}
    for sp in specs:
        if sp[0] != "ffm":
            continue
        _, w1c, v1c, v2c, xic, xjc = sp
        W1 = M1.series(w1c)
        xi, xj = T.series(xic), T.series(xjc)
        if not all(pd.api.types.is_numeric_dtype(c) or c.isna().all() for c in (W1, xi, xj)):
            return fallback()
        A, B = _v_matrix(M1.series(v1c)), _v_matrix(M2.series(v2c))
        if A is None or B is None or A[0].shape[1] != B[0].shape[1]:
            return fallback()
        xi_a = xi.to_numpy(dtype=np.float32, na_value=np.nan)
        xj_a = xj.to_numpy(dtype=np.float32, na_value=np.nan)
        both = (ti >= 0) & (tj >= 0)
        both &= A[1][np.maximum(ti, 0)] & B[1][np.maximum(tj, 0)]
        if np.isnan(xi_a[ti >= 0]).any() or np.isnan(xj_a[both]).any():
            return fallback()          # NULL operands: the generic UDAF defines what they mean
        ffm_in[id(sp)] = (W1.to_numpy(dtype=np.float32, na_value=np.nan), A, B, xi_a, xj_a)

    # joined row order of the generic path: join 1 (matched in test order, then for LEFT the
    # unmatched), then join 2 over that order the same way
    def order_of(tm, kind, base):
        hit = tm[base] >= 0
        return np.concatenate([base[hit], base[~hit]]) if kind == "left" else base[hit]

    rows = order_of(ti, j1.kind, np.arange(T.n))
    rows = order_of(tj, j2.kind, rows)
    Lj = T.take(rows)
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
    g32 = codes.astype(np.int32)
    agg_values = {}
    for x, sp in zip(aggs, specs):
        if sp[0] == "count_star":
            agg_values[id(x)] = pd.Series(np.diff(bounds))
        elif sp[0] == "test":
            agg_values[id(x)] = session._agg_values(x, Lj, ctes, order, bounds, n_groups, codes)
        else:
            W1, (V1, vm1), (V2, vm2), xi_a, xj_a = ffm_in[id(sp)]
            agg_values[id(x)] = pd.Series(join_ffm(ti[rows], tj[rows], xi_a[rows], xj_a[rows], g32, W1,
                                                   V1, vm1, V2, vm2, n_groups, session.device))
    session.last_plan = "fused_ffm_join_predict"
    out = session._project(s.items, gframe, ctes, agg_values)
    base = _GroupBase(gframe, agg_values, session)
    return session._finish(out, base, s, ctes)
