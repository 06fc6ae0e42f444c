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


def _sql_edge_world(ctx):
    """Shards whose largest ids differ (the max user / item / feature id sits on rank 0 only),
    no explicit sizes: the replicas must still agree on one shape and the mixing collectives
    must pair up.  Also uneven batch counts with -mix_interval and an early convergence stop."""
    from hivemall_amd.sql import Session

    rng = np.random.default_rng(7)
    n = 401                                  # rank 0 gets 201 rows, rank 1 gets 200
    u = rng.integers(0, 30, n)
    i = rng.integers(0, 40, n)
    u[0], i[0] = 97, 131                     # row 0 -> rank 0 only
    mf = pd.DataFrame({"u": u, "i": i, "r": rng.random(n) * 5})
    feats = [[f"{j}:1.0" for j in rng.choice(50, 5, replace=False)] for _ in range(n)]
    feats[0] = ["499:1.0", "3:1.0"]
    fm = pd.DataFrame({"features": feats, "label": rng.integers(0, 2, n)})
    frows = [[f"{f}:{int(rng.integers(0, 20))}:1" for f in range(4)] for _ in range(n)]
    frows[0] = [f"{f}:{300 + f}:1" for f in range(6)]          # 6 fields, ids > 300: rank 0 only
    ffm = pd.DataFrame({"features": frows, "label": rng.integers(0, 2, n)})
    s = Session(device="cpu")
    s.register("mf_t", mf)
    s.register("fm_t", fm)
    s.register("ffm_t", ffm)
    a = s.sql("SELECT train_mf_sgd(u, i, r, '-factors 3 -iters 3') AS (idx, Pu, Qi, Bu, Bi, mu) FROM mf_t")
    b = s.sql("SELECT train_fm(features, label, '-c -factors 3 -iters 4 -mix_interval 1 -batch_size 64') "
              "AS (feature, Wi, Vi) FROM fm_t")
    c = s.sql("SELECT train_ffm(features, label, '-c -factors 2 -iters 5 -mix_interval 1 -batch_size 50 "
              "-cv_rate 0.5') AS (model_id, i, Wi, Vi) FROM ffm_t")
    return {"mf": (int(a["idx"].max()), len(a), float(np.nansum(a["Bu"].to_numpy(float)))),
            "fm": (len(b), float(np.nansum(b["Wi"].to_numpy(float)))),
            "ffm": (len(c), int(c["i"].max()), float(np.nansum(c["Wi"].to_numpy(float))))}


def test_distributed_sql_shards_with_different_max_ids():
    out = run_world("tests.test_sql_dist:_sql_edge_world", world=2)
    assert out[0] == out[1]
    assert out[0]["mf"][0] == 131            # one table sized by the union of the shards
    assert out[0]["fm"][0] > 0 and out[0]["ffm"][0] > 0


def _gbt_missing_class_world(ctx):
    """Row-sharded boosting where rank 1's shard lacks class 2: the class list is the union."""
    from hivemall_amd.models.trees import GradientTreeBoostingClassifier
    from hivemall_amd.models.xgboost import XGBoostTrainer
    from hivemall_amd.parallel.mix import ModelMixer

    rng = np.random.default_rng(3 + ctx.rank)
    X = rng.normal(size=(300, 4)).astype(np.float32)
    y = (X[:, 0] > 0).astype(int)
    if ctx.rank == 0:
        y[:20] = 2
    gb = GradientTreeBoostingClassifier("-trees 2 -max_depth 3 -subsample 1.0 -seed 5", device="cpu",
                                        mixer=ModelMixer(ctx), rank=ctx.rank).fit(X, y)
    xg = XGBoostTrainer("-objective multi:softprob -num_class 3 -num_round 2 -max_depth 3",
                        device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank).fit(X, y)
    return gb.classes, list(gb.model_table()["pred_models"].map(tuple)), xg.classes, \
        xg.model_table()["model"].iloc[0]


def test_boosting_data_parallel_class_union():
    out = run_world("tests.test_sql_dist:_gbt_missing_class_world", world=2)
    assert out[0][0] == out[1][0] == [0, 1, 2]
    assert out[0][2] == out[1][2] == [0, 1, 2]
    assert out[0][1] == out[1][1] and out[0][3] == out[1][3]
