"""Fused join-predict (sql/fused.py, ops/join_predict.py, csrc/kernels/join_predict.hip): the
fused operator must return exactly what the generic join + GROUP BY path returns."""
import os

import numpy as np
import pandas as pd
import pytest

from hivemall_amd.sql import Session


def _run(sess_factory, script, query, fused: bool):
    old = os.environ.get("HM_SQL_FUSED")
    os.environ["HM_SQL_FUSED"] = "1" if fused else "0"
    try:
        s = sess_factory()
        if script:
            s.sql(script)
        s.last_plan = None
        out = s.sql(query)
        return out, s.last_plan
    finally:
        if old is None:
            os.environ.pop("HM_SQL_FUSED", None)
        else:
            os.environ["HM_SQL_FUSED"] = old


def _assert_same(a: pd.DataFrame, b: pd.DataFrame):
    assert list(a.columns) == list(b.columns)
    assert len(a) == len(b)
    for c in a.columns:
        x, y = a[c].to_numpy(), b[c].to_numpy()
        if np.issubdtype(np.asarray(x).dtype, np.number) or np.issubdtype(np.asarray(y).dtype, np.number):
            np.testing.assert_allclose(np.asarray(x, dtype=float), np.asarray(y, dtype=float), rtol=1e-6,
                                       atol=1e-7, err_msg=c)
        else:
            assert list(x) == list(y), c


def _tables(device="cpu", seed=0, n=400, nf=60):
    rng = np.random.default_rng(seed)
    rows = []
    for r in range(n):
        k = int(rng.integers(0, 8))
        for _ in range(k):
            f = int(rng.integers(0, nf))
            rows.append((r, str(f), float(rng.uniform(0.1, 2.0)), int(r % 2)))
    test = pd.DataFrame(rows, columns=["rowid", "feature", "value", "label"])
    feats = [str(i) for i in range(0, nf, 2)]            # half the features are unknown
    w = rng.normal(size=len(feats))
    w[::7] = np.nan                                       # NULL weights
    model = pd.DataFrame({"feature": feats, "weight": w})

    def make():
        s = Session(device=device)
        s.register("test_exploded", test)
        s.register("model", model)
        return s
    return make


LINEAR_Q = """
SELECT t.rowid, sigmoid(sum(m.weight * t.value)) AS prob, max(t.label) AS label, count(*) AS n,
       avg(t.value) AS av
FROM test_exploded t LEFT OUTER JOIN model m ON (t.feature = m.feature)
GROUP BY t.rowid"""


@pytest.mark.parametrize("query", [
    LINEAR_Q,
    LINEAR_Q + " ORDER BY prob DESC",
    LINEAR_Q.replace("LEFT OUTER JOIN", "JOIN"),
    """SELECT t.rowid, sum(t.value * m.weight) AS s FROM test_exploded t
       LEFT OUTER JOIN model m ON (m.feature = t.feature) GROUP BY t.rowid ORDER BY rowid""",
    """SELECT t.label, t.rowid, sum(m.weight * t.value) AS s FROM test_exploded t
       LEFT OUTER JOIN model m ON (t.feature = m.feature) GROUP BY t.label, t.rowid""",
])
def test_fused_linear_equals_generic(query):
    make = _tables()
    a, plan_a = _run(make, None, query, fused=True)
    b, plan_b = _run(make, None, query, fused=False)
    assert plan_a == "fused_join_predict" and plan_b is None
    _assert_same(a, b)


def test_fused_falls_back_on_duplicate_model_keys():
    make0 = _tables()

    def make():
        s = make0()
        m = s.table("model")
        s.register("model", pd.concat([m, m.iloc[:3]], ignore_index=True))
        return s
    a, plan_a = _run(make, None, LINEAR_Q, fused=True)
    b, _ = _run(make, None, LINEAR_Q, fused=False)
    assert plan_a is None
    _assert_same(a, b)


def test_fused_fm_predict_equals_generic_and_trainer():
    from hivemall_amd.models.fm import FMTrainer
    rng = np.random.default_rng(0)
    rows = [[f"{int(i) + 1}:1" for i in rng.choice(100, size=5, replace=False)] for _ in range(400)]
    y = rng.random(400).astype(np.float32)
    script = "CREATE TABLE fm_model AS SELECT train_fm(features, y, '-factors 3 -iters 2') AS (feature, Wi, Vif) FROM t"
    q = """
    SELECT t.rowid, fm_predict(m.Wi, m.Vif, t.Xi) AS p FROM (
      SELECT rowid, extract_feature(fv) AS feature, extract_weight(fv) AS Xi
      FROM t LATERAL VIEW explode(add_bias(features)) e AS fv) t
    LEFT OUTER JOIN fm_model m ON (t.feature = m.feature)
    GROUP BY t.rowid ORDER BY rowid"""

    def make():
        s = Session(device="cpu")
        s.register("t", pd.DataFrame({"rowid": range(400), "features": rows, "y": y}))
        return s
    a, plan_a = _run(make, script, q, fused=True)
    b, _ = _run(make, script, q, fused=False)
    assert plan_a == "fused_join_predict"
    _assert_same(a, b)
    ref = FMTrainer("-factors 3 -iters 2", device="cpu").fit(rows, y).predict(rows)
    np.testing.assert_allclose(a["p"].to_numpy(dtype=float), ref, rtol=1e-3, atol=1e-4)


@pytest.mark.gpu
def test_fused_join_predict_gpu_equals_cpu():
    """The gfx950 kernels (GPU session) against the numpy path (CPU session)."""
    for q in (LINEAR_Q + " ORDER BY rowid",):
        a, pa_ = _run(_tables("cuda", seed=3, n=20000, nf=5000), None, q, fused=True)
        b, pb_ = _run(_tables("cpu", seed=3, n=20000, nf=5000), None, q, fused=True)
        assert pa_ == pb_ == "fused_join_predict"
        _assert_same(a, b)


FFM_Q = """
SELECT t.rowid, sigmoid(ffm_predict(m1.Wi, m1.Vi, m2.Vi, t.Xi, t.Xj)) AS p, max(t.Xi) AS mx,
       count(*) AS n
FROM tp t
LEFT OUTER JOIN ffm_model m1 ON (t.i = m1.i)
LEFT OUTER JOIN ffm_model m2 ON (t.j = m2.i)
GROUP BY t.rowid ORDER BY rowid"""


def _ffm_tables(device="cpu", n=300, nf=5, seed=1, drop_model_rows=0):
    """Trains an FFM model on ``n`` rows, explodes them with feature_pairs('-ffm'); optionally
    drops model rows so some joins miss (the LEFT JOIN NULL paths)."""
    rng = np.random.default_rng(seed)
    rows = [[f"{f}:{int(rng.integers(0, 20))}:1" for f in range(nf)] for _ in range(n)]
    y = (rng.random(n) < 0.4).astype(int)
    opts = f"-c -factors 3 -num_fields {nf} -feature_hashing 10 -iters 2 -w0"
    base = Session(device="cpu")
    base.register("t", pd.DataFrame({"rowid": range(n), "features": rows, "label": y}))
    model = base.sql(f"SELECT train_ffm(features, label, '{opts}') AS (model_id, i, Wi, Vi) FROM t")
    if drop_model_rows:
        model = model.drop(index=rng.choice(len(model), drop_model_rows, replace=False)).reset_index(drop=True)
    tp = base.sql(f"SELECT rowid, i, j, Xi, Xj FROM t LATERAL VIEW feature_pairs(features, "
                  f"'-ffm -feature_hashing 10 -num_fields {nf}') x AS i, j, Xi, Xj")

    def make():
        s = Session(device=device)
        s.register("ffm_model", model)
        s.register("tp", tp)
        return s
    return make, rows, y, opts


@pytest.mark.parametrize("drop", [0, 40])
def test_fused_ffm_predict_equals_generic(drop):
    """The two-join FFM scoring query runs as one gather-reduce and returns
    exactly the generic path's table; with every model row present it is the trainer's
    prediction."""
    from hivemall_amd.models.ffm import FFMTrainer

    make, rows, y, opts = _ffm_tables(drop_model_rows=drop)
    a, plan_a = _run(make, None, FFM_Q, fused=True)
    b, plan_b = _run(make, None, FFM_Q, fused=False)
    assert plan_a == "fused_ffm_join_predict" and plan_b is None
    _assert_same(a, b)
    if not drop:
        ref = FFMTrainer(opts, device="cpu").fit(rows, y).predict(rows)
        np.testing.assert_allclose(a["p"].to_numpy(dtype=float), ref, rtol=1e-4, atol=1e-6)


def test_fused_ffm_inner_joins_equal_generic():
    make, *_ = _ffm_tables(drop_model_rows=25, seed=4)
    q = FFM_Q.replace("LEFT OUTER JOIN", "JOIN")
    a, plan_a = _run(make, None, q, fused=True)
    b, _ = _run(make, None, q, fused=False)
    assert plan_a == "fused_ffm_join_predict"
    _assert_same(a, b)


@pytest.mark.gpu
def test_fused_ffm_predict_gpu_equals_cpu():
    """hm_join_ffm (gfx950, wave-reduced fp64 atomics) against the numpy path."""
    mk_g, *_ = _ffm_tables("cuda", n=3000, nf=8, drop_model_rows=30)
    mk_c, *_ = _ffm_tables("cpu", n=3000, nf=8, drop_model_rows=30)
    a, pa_ = _run(mk_g, None, FFM_Q, fused=True)
    b, pb_ = _run(mk_c, None, FFM_Q, fused=True)
    assert pa_ == pb_ == "fused_ffm_join_predict"
    _assert_same(a, b)
