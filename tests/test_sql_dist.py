"""Distributed HiveQL (gloo, world 2): every rank runs the same script on the same tables; the
train_* UDTFs split their input rows over the ranks and mix over the collective backend, so all
ranks materialise one model table — the one the Python-API data-parallel path trains."""
import numpy as np
import pandas as pd

from tests.test_dist import run_world


def _tables():
    from hivemall_amd.io.synthetic import a9a_like

    rows, y = a9a_like(1200, seed=3)
    train = pd.DataFrame({"rowid": range(len(rows)), "features": [[str(int(i)) for i in r] for r in rows],
                          "label": y})
    rng = np.random.default_rng(1)
    frows = [[f"{f}:{int(rng.integers(0, 20))}:1" for f in range(4)] for _ in range(400)]
    fy = (rng.random(400) < 0.4).astype(int)
    ffm = pd.DataFrame({"rowid": range(400), "features": frows, "label": fy})
    X = rng.normal(size=(600, 4)).astype(np.float32)
    rf = pd.DataFrame({"features": [list(map(float, r)) for r in X], "label": (X[:, 0] > 0).astype(int)})
    return train, ffm, rf


A9A_OPTS = "-loss logloss -opt adagrad -reg no -iters 2"
FFM_OPTS = "-c -factors 2 -num_fields 4 -feature_hashing 10 -iters 2"


def _sql_world(ctx):
    from hivemall_amd.models import linear as L
    from hivemall_amd.models.ffm import FFMTrainer
    from hivemall_amd.parallel.mix import ModelMixer
    from hivemall_amd.sql import Session

    train, ffm, rf = _tables()
    s = Session(device="cpu")
    assert s.ctx is not None and s.ctx.world_size == 2
    s.register("train", train)
    s.register("ffm_t", ffm)
    s.register("rf_t", rf)
    s.sql(f"""CREATE TABLE model AS
      SELECT feature, avg(weight) AS weight FROM (
        SELECT train_classifier(features, label, '{A9A_OPTS}') AS (feature, weight) FROM train) t
      GROUP BY feature""")
    s.sql(f"CREATE TABLE ffm_model AS SELECT train_ffm(features, label, '{FFM_OPTS}') AS (model_id, i, Wi, Vi) FROM ffm_t")
    s.sql("CREATE TABLE rf_model AS SELECT train_randomforest_classifier(features, label, '-trees 4 -seed 5') "
          "AS (model_id, model_weight, model, var_importance, oob_errors, oob_tests) FROM rf_t")
    sql = {"lin": s.table("model").sort_values("feature").reset_index(drop=True),
           "ffm": s.table("ffm_model").sort_values("i").reset_index(drop=True),
           "rf": sorted(s.table("rf_model")["model"].tolist()),
           "cnt": int(s.sql("SELECT count(*) AS n FROM train")["n"][0])}
    # the Python-API data-parallel path: rank r trains on rows r, r + 2, ... and mixes
    me = slice(ctx.rank, None, ctx.world_size)
    lin = L.LEARNERS["train_classifier"](A9A_OPTS, device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
    lin.fit(list(train["features"])[me], list(train["label"])[me])
    tab = lin.model_table().groupby("feature", as_index=False)["weight"].mean()
    f = FFMTrainer(FFM_OPTS, device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
    f.fit(list(ffm["features"])[me], list(ffm["label"])[me])
    api = {"lin": tab.sort_values("feature").reset_index(drop=True),
           "ffm": f.model_table().sort_values("i").reset_index(drop=True)}
    return {"sql": sql, "api": api}


def test_distributed_sql_matches_python_dp_path():
    out = run_world("tests.test_sql_dist:_sql_world", world=2)
    for r in (0, 1):
        sql, api = out[r]["sql"], out[r]["api"]
        assert sql["cnt"] == 1200                          # queries see the global table
        pd.testing.assert_frame_equal(sql["lin"], api["lin"], check_dtype=False)
        assert sql["ffm"]["i"].tolist() == api["ffm"]["i"].tolist()
        np.testing.assert_allclose(sql["ffm"]["Wi"].to_numpy(float), api["ffm"]["Wi"].to_numpy(float),
                                   equal_nan=True)
    # one model on every rank
    pd.testing.assert_frame_equal(out[0]["sql"]["lin"], out[1]["sql"]["lin"])
    pd.testing.assert_frame_equal(out[0]["sql"]["ffm"], out[1]["sql"]["ffm"])
    # RandomForest: the union of the ranks' trees is the single-process forest
    assert out[0]["sql"]["rf"] == out[1]["sql"]["rf"] and len(out[0]["sql"]["rf"]) == 4
    from hivemall_amd.models.trees import RandomForestClassifier

    _, _, rf = _tables()
    single = RandomForestClassifier("-trees 4 -seed 5", device="cpu").fit(list(rf["features"]), list(rf["label"]))
    assert sorted(single.model_table()["model"].tolist()) == out[0]["sql"]["rf"]
