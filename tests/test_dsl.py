import numpy as np
import pandas as pd

import hivemall_amd.dsl  # noqa: F401
from hivemall_amd.io.synthetic import a9a_like


def test_dataframe_dsl():
    rows, y = a9a_like(2000)
    df = pd.DataFrame({"rowid": range(2000), "features": [[str(int(i)) for i in r] for r in rows], "label": y})
    df["features"] = df.hivemall.add_bias("features")
    assert df["features"][0][-1] == "0:1.0"
    model = df.hivemall.on("cpu").train_classifier("features", "label", "-loss logloss -iters 3")
    assert list(model.columns) == ["feature", "weight"] and len(model) > 100
    ex = df.head(3).hivemall.explode("features") if False else None
    w = dict(zip(model["feature"], model["weight"]))
    df["prob"] = [1 / (1 + np.exp(-sum(w.get(f.split(":")[0] if ":" in f else f, 0.0) for f in fs))) for fs in df["features"]]
    auc = df.hivemall.auc("prob", "label")
    assert auc > 0.8
    g = df.assign(g=df["rowid"] % 2).groupby("g").hivemall.logloss("prob", "label")
    assert len(g) == 2
    pairs = df.head(2).hivemall.feature_pairs("features", "-kpa")
    assert pairs.shape[1] == 4
