import numpy as np
import pandas as pd
import pytest
import torch
from sklearn.metrics import roc_auc_score

from hivemall_amd.io.synthetic import higgs_like
from hivemall_amd.models.trees import (GradientTreeBoostingClassifier, RandomForestClassifier,
                                       RandomForestRegressor, Tree, decision_path, quantize,
                                       rf_ensemble, tree_export, tree_predict)
from hivemall_amd.sql import Session


@pytest.fixture(scope="module")
def higgs():
    X, y = higgs_like(30000)
    Xt, yt = higgs_like(6000, seed=9)
    return X, y.long(), Xt, yt.long()


def test_quantize_bins_monotone():
    X = torch.randn(5000, 3)
    q = quantize(X, 16)
    assert q.bins.dtype == torch.uint8 and int(q.bins[:, :3].max()) <= 15
    o = torch.argsort(X[:, 0])
    assert (q.bins[o, 0].diff().to(torch.int64) >= 0).all()


def test_random_forest_classifier(higgs):
    X, y, Xt, yt = higgs
    rf = RandomForestClassifier("-trees 10 -max_depth 10 -seed 3", device="cpu").fit(X, y)
    auc = roc_auc_score(yt.numpy(), rf.predict_proba(Xt)[:, 1])
    assert auc > 0.72
    tab = rf.model_table()
    assert list(tab.columns) == ["model_id", "model_weight", "model", "var_importance", "oob_errors", "oob_tests"]
    assert (tab["oob_tests"] > 0).all()
    r = tree_predict(tab.iloc[0]["model_id"], tab.iloc[0]["model"], Xt[0].tolist(), "-classification")
    assert set(r) == {"value", "posteriori"}
    assert "digraph" in tree_export(tab.iloc[0]["model"])
    assert decision_path(tab.iloc[0]["model_id"], tab.iloc[0]["model"], Xt[0].tolist())[-1].startswith("value=")


def test_gbt_matches_sklearn_quality(higgs):
    from sklearn.ensemble import HistGradientBoostingClassifier
    X, y, Xt, yt = higgs
    gb = GradientTreeBoostingClassifier("-trees 40 -eta 0.1 -max_depth 6 -seed 3", device="cpu").fit(X, y)
    auc = roc_auc_score(yt.numpy(), gb.predict_proba(Xt)[:, 1])
    ref = HistGradientBoostingClassifier(max_iter=40, learning_rate=0.1, max_depth=6).fit(X.numpy(), y.numpy())
    auc_ref = roc_auc_score(yt.numpy(), ref.predict_proba(Xt.numpy())[:, 1])
    assert auc > auc_ref - 0.015, (auc, auc_ref)
    tab = gb.model_table()
    assert list(tab.columns) == ["iteration", "pred_models", "intercept", "shrinkage", "var_importance", "oob_error_rate"]


def test_gbt_multiclass():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(6000, 5)).astype(np.float32)
    y = (X[:, 0] > 0).astype(int) + (X[:, 1] > 0.5).astype(int)
    gb = GradientTreeBoostingClassifier("-trees 20 -eta 0.2 -max_depth 4", device="cpu").fit(X, y)
    assert (gb.predict(X) == y).mean() > 0.9


def test_rf_regressor():
    rng = np.random.default_rng(1)
    X = rng.normal(size=(8000, 4)).astype(np.float32)
    y = 2 * X[:, 0] + np.sin(X[:, 1])
    rr = RandomForestRegressor("-trees 10", device="cpu").fit(X, y)
    assert np.sqrt(((rr.predict(X) - y) ** 2).mean()) < 0.5


def test_tree_serialization_roundtrip():
    t = Tree([0, -1, -1], [0.5, float("inf"), float("inf")], [1, -1, -1], [2, -1, -1],
             [None, [1.0, 0.0], [0.0, 1.0]], 2)
    t2 = Tree.deserialize(t.serialize())
    assert t2.predict_one([0.2]) == [1.0, 0.0] and t2.predict_one([0.9]) == [0.0, 1.0]


def test_rf_sql_pipeline(higgs):
    X, y, Xt, yt = higgs
    s = Session(device="cpu")
    s.register("train", pd.DataFrame({"features": [list(map(float, r)) for r in X[:5000].tolist()],
                                      "label": y[:5000].numpy()}))
    s.register("test", pd.DataFrame({"rowid": range(500), "features": [list(map(float, r)) for r in Xt[:500].tolist()],
                                     "label": yt[:500].numpy()}))
    s.sql("CREATE TABLE rf AS SELECT train_randomforest_classifier(features, label, '-trees 5 -seed 71') "
          "AS (model_id, model_weight, model, var_importance, oob_errors, oob_tests) FROM train")
    p = s.sql("""
    SELECT rowid, rf_ensemble(predicted.value, predicted.posteriori, model_weight) AS predicted FROM (
      SELECT t.rowid, m.model_weight, tree_predict(m.model_id, m.model, t.features, '-classification') AS predicted
      FROM rf m CROSS JOIN test t) x GROUP BY rowid""")
    assert len(p) == 500
    acc = np.mean([d["label"] == lab for d, lab in zip(p["predicted"], yt[:500].numpy()[p["rowid"].to_numpy()])])
    assert acc > 0.55   # 5 trees on 5,000 rows: ~0.59-0.65 across seeds (chance 0.5)


@pytest.mark.gpu
def test_hist_kernel_matches_cpu(higgs):
    X, y, _, _ = higgs
    res = {}
    for dev in ("cpu", "cuda"):
        gb = GradientTreeBoostingClassifier("-trees 3 -eta 0.1 -max_depth 5 -subsample 1.0 -seed 3", device=dev).fit(X, y)
        res[dev] = gb
    a = res["cpu"].iters[0][0]
    b = res["cuda"].iters[0][0]
    assert a.feature == b.feature
    np.testing.assert_allclose(res["cpu"].decision_function(X[:2000]), res["cuda"].decision_function(X[:2000]),
                               rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_gbt_gpu_fused_path_subsample_matches_cpu_quality(higgs):
    """Binary GBT on the GPU runs the fused statistics / leaf-update kernels (hm_gbt_stats /
    hm_gbt_apply); with row subsampling the masked rows must drop out of the histograms and
    still get their leaf update.  Quality equals the CPU engine's (same rule, its own sampling)."""
    X, y, Xt, yt = higgs
    auc = {}
    for dev in ("cpu", "cuda"):
        gb = GradientTreeBoostingClassifier("-trees 20 -eta 0.1 -max_depth 5 -subsample 0.7 -seed 3",
                                            device=dev).fit(X, y)
        auc[dev] = roc_auc_score(yt.numpy(), gb.predict_proba(Xt)[:, 1])
        assert len(gb.oob_rates) == 20 and 0.0 < gb.oob_rates[-1] < 0.5
    assert abs(auc["cpu"] - auc["cuda"]) < 0.01, auc


@pytest.mark.gpu
def test_rf_gpu_quality(higgs):
    X, y, Xt, yt = higgs
    aucs = {}
    for dev in ("cpu", "cuda"):
        rf = RandomForestClassifier("-trees 10 -max_depth 10 -seed 3", device=dev).fit(X, y)
        aucs[dev] = roc_auc_score(yt.numpy(), rf.predict_proba(Xt)[:, 1])
    # the bootstrap draws come from each device's RNG stream: 10 trees differ by up to ~0.015 AUC
    assert abs(aucs["cpu"] - aucs["cuda"]) < 0.02, aucs


def _leaf_vs_predict(dev):
    from hivemall_amd.models.trees import HistTreeBuilder, predict_forest
    g = torch.Generator().manual_seed(0)
    X = torch.randn(20000, 9, generator=g)
    X[torch.rand(20000, 9, generator=g) < 0.05] = float("nan")          # missing values go right
    y = (torch.nan_to_num(X[:, 0]) * torch.nan_to_num(X[:, 1]) > 0).float()
    X = X.to(dev)
    q = quantize(X, 64)
    st = torch.stack([y - 0.5, torch.full_like(y, 0.25), torch.ones_like(y)], 1).to(dev)
    st[::7] = 0                                                           # unsampled rows are routed too
    b = HistTreeBuilder(q, "gbt", max_depth=6, seed=1)
    tree = b.build(st)
    via_leaf = b.node_values[b.leaf_of_row.long(), 0]
    via_pred = predict_forest([tree], X)[:, 0]
    torch.testing.assert_close(via_leaf, via_pred)
    assert tree.depth() == 6


def test_builder_leaf_routing_matches_predict():
    _leaf_vs_predict("cpu")


@pytest.mark.gpu
def test_builder_leaf_routing_matches_predict_gpu():
    _leaf_vs_predict("cuda")


def _hist_case(NS=3, d=27):
    g = torch.Generator().manual_seed(1)
    n, dpad, B = 300000, 32, 256
    bins = torch.zeros(n, dpad, dtype=torch.uint8)
    bins[:, :d] = torch.randint(0, B, (n, d), generator=g, dtype=torch.uint8)
    stats = torch.randn(n, NS, generator=g)
    sizes = torch.tensor([150000, 3, 0, 70, 100000, 1, 500, 20000])
    rows = torch.randperm(n, generator=g)[: int(sizes.sum())].to(torch.int32)
    seg = torch.zeros(len(sizes) + 1, dtype=torch.int64)
    seg[1:] = torch.cumsum(sizes, 0)
    S = len(sizes)
    ref = torch.zeros(S * d * B * NS, dtype=torch.float64)
    node = torch.repeat_interleave(torch.arange(S), sizes)
    for f in range(d):
        for s in range(NS):
            idx = ((node * d + f) * B + bins[rows.long(), f].long()) * NS + s
            ref.index_add_(0, idx, stats[rows.long(), s].double())
    return (bins, rows, seg, stats), ref.view(S, d, B, NS), (d, dpad, B, NS, S)


def _run_hist(dev, FG, NS=3, d=27):
    from hivemall_amd import _native
    (bins, rows, seg, stats), ref, (d, dpad, B, NS, S) = _hist_case(NS, d)
    hb, hr, hs, hst = (t.to(dev) for t in (bins, rows, seg, stats))
    out = torch.zeros(S, d, B, NS, device=dev)
    p = _native.ptr
    smax = stats.abs().amax(0).to(dev)
    args = (p(hb), d, dpad, B, p(hr), p(hs), S, p(hst), p(smax), NS, FG, p(out))
    gargs = args + (0,)
    if dev == "cuda":
        _native.check(_native.hip().hm_hist_build(*gargs, _native.stream_of(torch.device(dev))), "hm_hist_build")
    else:
        assert _native.host().hm_hist_build_cpu(*args) == 0
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-4, atol=2e-3)


def test_hist_cpu_segments_vs_torch():
    _run_hist("cpu", 16)


@pytest.mark.gpu
def test_hist_kernel_segments_vs_torch():
    """Segmented histogram kernel (LDS path for large segments, global path for small ones)
    against a torch fp64 scatter-add reference; two feature-group widths."""
    for FG in (16, 8, 4):
        _run_hist("cuda", FG)


@pytest.mark.gpu
@pytest.mark.parametrize("NS", [5, 7, 8])
def test_hist_kernel_5_to_8_statistics_vs_torch(NS):
    """5..8 statistics (RandomForest with 5..8 classes) on 20 features: the feature-group
    kernel with 4-feature groups (the shape models/trees.py routes there) against fp64."""
    _run_hist("cuda", 4, NS=NS, d=20)


def _nominal_data(n=4000, seed=3):
    rng = np.random.default_rng(seed)
    cat = rng.integers(0, 12, n).astype(np.float32)
    x1 = rng.normal(size=n).astype(np.float32)
    y = (cat == 5).astype(int)            # one category against the rest
    return np.stack([cat, x1], 1), y


def test_rf_nominal_attrs_one_vs_rest_split():
    """-attrs C: a stump isolates one category (x == 5), which an ordinal stump cannot."""
    X, y = _nominal_data()
    nom = RandomForestClassifier("-trees 3 -max_depth 1 -mtry 2 -attrs C,Q -seed 1", device="cpu").fit(X, y)
    assert (nom.predict(X) == y).mean() == 1.0
    assert all(t.cat and t.cat[0] and t.feature[0] == 0 and t.threshold[0] == 5.0 for t in nom.trees)
    ordn = RandomForestClassifier("-trees 3 -max_depth 1 -mtry 2 -attrs Q,Q -seed 1", device="cpu").fit(X, y)
    assert (ordn.predict(X) == y).mean() < 1.0
    tab = nom.model_table()
    m = tab.iloc[0]["model"]
    assert tree_predict(tab.iloc[0]["model_id"], m, [5.0, 0.3], "-classification")["value"] == 1
    assert tree_predict(tab.iloc[0]["model_id"], m, [6.0, 0.3], "-classification")["value"] == 0
    assert "==" in tree_export(m) and "x[0] == 5" in tree_export(m, "-type js")
    assert decision_path(tab.iloc[0]["model_id"], m, [5.0, 0.0])[0].startswith("0 == 5")
    with pytest.raises(Exception):
        RandomForestClassifier("-attrs C", device="cpu").fit(X, y)     # one type per column


def test_gbt_nominal_attrs():
    X, y = _nominal_data(seed=4)
    gb = GradientTreeBoostingClassifier("-trees 5 -eta 0.5 -max_depth 1 -attrs C,Q -subsample 1.0", device="cpu").fit(X, y)
    assert (gb.predict(X) == y).mean() == 1.0


def test_stratified_bootstrap_keeps_class_shares():
    from hivemall_amd.models.trees import bootstrap_weights
    y = torch.tensor([0] * 990 + [1] * 10)
    g = torch.Generator().manual_seed(0)
    w = bootstrap_weights(1000, 0.5, g, "cpu", y)
    assert float(w[:990].sum()) == 495 and float(w[990:].sum()) == 5
    w = bootstrap_weights(1000, 1.0, g, "cpu")
    assert float(w.sum()) == 1000
    rf = RandomForestClassifier("-trees 2 -stratified -subsample 0.5 -seed 2", device="cpu").fit(
        np.random.default_rng(0).normal(size=(1000, 3)).astype(np.float32), y.numpy())
    assert len(rf.trees) == 2


@pytest.mark.gpu
def test_rf_nominal_attrs_gpu_matches_cpu():
    X, y = _nominal_data(n=20000, seed=6)
    X[:, 1] += (X[:, 0] == 3) * 2.0
    y = ((X[:, 0] == 5) | (X[:, 1] > 1.5)).astype(int)
    # bootstrap draws come from the device's RNG stream, so the forests differ in detail:
    # compare quality, the nominal nodes, and GPU traversal against the host walk of the same trees
    for dev in ("cpu", "cuda"):
        rf = RandomForestClassifier("-trees 4 -max_depth 4 -mtry 2 -attrs C,Q -seed 1", device=dev).fit(X, y)
        assert (rf.predict(X) == y).mean() > 0.99
        assert any(any(t.cat) for t in rf.trees)
    from hivemall_amd.models.trees import predict_forest
    host = np.array([[rf.trees[0].predict_one(list(map(float, r)))[1]] for r in X[:2000]])
    dev_p = predict_forest(rf.trees[:1], torch.from_numpy(X[:2000]).cuda())[:, 1:2].cpu().numpy()
    np.testing.assert_allclose(dev_p, host, atol=1e-6)


def _split_case(crit, NS, cat=False, seed=0):
    from hivemall_amd.models.trees import HistTreeBuilder, Quantized
    g = torch.Generator().manual_seed(seed)
    L, d, B = 5, 7, 64
    H = torch.rand(L, d, B, NS, generator=g)
    if crit == "gbt":
        H[..., 0] -= 0.5
        H[..., 2] = torch.randint(0, 3, (L, d, B), generator=g).float()
    if crit == "xgb":
        H[..., 0] -= 0.5
    # every feature's bins must sum to the node total (one set of rows per node)
    H = H / H.sum(2, keepdim=True) * H[:, :1].sum(2, keepdim=True)
    edges = torch.sort(torch.rand(d, B - 1, generator=g), 1).values
    cm = torch.tensor([i % 3 == 0 for i in range(d)]) if cat else None
    q = Quantized(torch.zeros(1, 16, dtype=torch.uint8), edges, d, B, cm)
    b = HistTreeBuilder(q, crit, min_samples_leaf=0.5 if crit in ("gini", "entropy", "variance") else 0.0,
                        lam=0.3 if crit in ("gbt", "xgb") else 0.0, alpha=0.05 if crit == "xgb" else 0.0)
    return b, H, cm


def _split_ref(b, H, cm):
    """The per-level split search as tensor ops (the pre-fused formulation)."""
    tot = H[:, 0].sum(1)
    cum = torch.cumsum(H, 2)
    right = tot[:, None, None] - cum
    gain = b._score(cum) + b._score(right) - b._score(tot)[:, None, None]
    ok = (b._weight(cum) >= b.min_leaf) & (b._weight(right) >= b.min_leaf)
    if cm is not None:
        rest = tot[:, None, None] - H
        ge = b._score(H) + b._score(rest) - b._score(tot)[:, None, None]
        oe = (b._weight(H) >= b.min_leaf) & (b._weight(rest) >= b.min_leaf)
        oe[:, :, b.q.edges.shape[1]:] = False
        gain = torch.where(cm[None, :, None], ge, gain)
        ok = torch.where(cm[None, :, None], oe, ok)
    gain = torch.where(ok, gain, torch.full_like(gain, -float("inf")))
    bg, bi = gain.reshape(H.shape[0], -1).max(1)
    return bg, bi, tot


@pytest.mark.parametrize("crit,NS,cat", [("gini", 3, False), ("entropy", 4, True), ("variance", 2, False),
                                         ("gbt", 3, True), ("xgb", 2, False)])
def test_split_find_matches_tensor_formulation(crit, NS, cat):
    b, H, cm = _split_case(crit, NS, cat)
    gain, feat, bins, left, tot, _ = b._split_find(H, 0)
    bg, bi, rtot = _split_ref(b, H, cm)
    torch.testing.assert_close(tot, rtot, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gain, bg, rtol=1e-4, atol=1e-5)
    assert torch.equal(feat.long() * H.shape[2] + bins.long(), bi)


def test_split_find_mtry_draw():
    b, H, _ = _split_case("gini", 3)
    b.mtry = 2
    _, feat, _, _, _, _ = b._split_find(H, 0)
    _, feat2, _, _, _, _ = b._split_find(H, 0)
    assert torch.equal(feat, feat2)           # the draw is a pure function of (seed, node)
    draws = {tuple(b._split_find(H, base)[1].tolist()) for base in range(0, 400, 40)}
    assert len(draws) > 1                     # ... and differs between nodes


@pytest.mark.gpu
@pytest.mark.parametrize("crit,NS,cat", [("gini", 3, False), ("entropy", 2, True), ("gbt", 3, True), ("xgb", 2, False)])
def test_split_find_kernel_matches_host(crit, NS, cat):
    b, H, cm = _split_case(crit, NS, cat, seed=5)
    b.mtry = 4
    host = b._split_find(H, 7)
    b._masks = None
    dev = b._split_find(H.cuda(), 7)
    torch.testing.assert_close(dev[0].cpu(), host[0], rtol=1e-4, atol=1e-5)
    assert torch.equal(dev[1].cpu(), host[1]) and torch.equal(dev[2].cpu(), host[2])
    torch.testing.assert_close(dev[3].cpu(), host[3], rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_partition_kernel_groups_rows_like_sort():
    """Counting-sort partition of a level == stable key sort, as sets per segment."""
    from hivemall_amd.models.trees import HistTreeBuilder
    g = torch.Generator().manual_seed(3)
    n, nb, n_split = 300000, 15, 40
    node = torch.randint(nb - 5, nb + 2 * n_split, (n,), generator=g, dtype=torch.int32)
    act = torch.nonzero(torch.rand(n, generator=g) < 0.7).flatten().to(torch.int32)
    lut = torch.full((2 * n_split,), 32767, dtype=torch.int16)
    pick = torch.randperm(2 * n_split, generator=g)[:n_split]
    lut[pick] = torch.arange(n_split, dtype=torch.int16)
    rows, seg = HistTreeBuilder._partition_gpu(act.cuda(), node.cuda(), nb, lut.cuda(), n_split)
    rows, seg = rows.cpu(), seg.cpu()
    nr = node[act.long()] - nb
    key = torch.where((nr >= 0) & (nr < 2 * n_split), lut[nr.clamp(0, 2 * n_split - 1).long()],
                      torch.full_like(nr, 32767, dtype=torch.int16))
    for k in range(n_split):
        want = set(act[key == k].tolist())
        got = rows[seg[k]:seg[k + 1]].tolist()
        assert len(got) == len(want) and set(got) == want, k
    assert int(seg[n_split]) == int((key < n_split).sum())


# ---------------------------------------------------------------- many classes (NS > 8)
def _int_split_case(crit, NS, cat=False, seed=0):
    """Integer class-count histograms (exact in fp32) for the class-decomposed split search."""
    b, _, cm = _split_case(crit, 2, cat, seed)
    g = torch.Generator().manual_seed(seed + 100)
    L, d, B = 5, 7, 64
    rows = torch.randint(0, NS, (L, 4000), generator=g)
    binsel = torch.randint(0, B, (L, d, 4000), generator=g)
    H = torch.zeros(L, d, B, NS)
    for l in range(L):
        for f in range(d):
            H[l, f].index_put_((binsel[l, f], rows[l]), torch.ones(4000), accumulate=True)
    return b, H, cm


@pytest.mark.parametrize("crit,cat", [("gini", False), ("entropy", True)])
def test_split_find_many_classes_matches_tensor_formulation(crit, cat):
    b, H, cm = _int_split_case(crit, 11, cat)
    gain, feat, bins, left, tot, _ = b._split_find(H, 0)
    bg, bi, rtot = _split_ref(b, H, cm)
    torch.testing.assert_close(tot, rtot)
    torch.testing.assert_close(gain, bg, rtol=1e-4, atol=1e-3)
    assert torch.equal(feat.long() * H.shape[2] + bins.long(), bi)
    # left statistics of the chosen split
    for l in range(H.shape[0]):
        f, bb = int(feat[l]), int(bins[l])
        want = H[l, f, bb] if (cm is not None and bool(cm[f])) else H[l, f, :bb + 1].sum(0)
        torch.testing.assert_close(left[l], want)


def _ten_class_data(n=6000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 6)).astype(np.float32)
    y = (np.floor((X[:, 0] + 3) * 10 / 6).clip(0, 9)).astype(int)   # 10 bands of feature 0
    return X, y


def test_rf_ten_classes_cpu():
    X, y = _ten_class_data()
    rf = RandomForestClassifier("-trees 8 -max_depth 8 -seed 3", device="cpu").fit(X, y)
    assert len(rf.classes) == 10
    assert (rf.predict(X) == y).mean() > 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("crit,cat", [("gini", False), ("entropy", True), ("gini", True)])
def test_split_find_many_classes_kernel_matches_host(crit, cat):
    b, H, cm = _int_split_case(crit, 10, cat, seed=4)
    b.mtry = 4
    host = b._split_find(H, 7)
    b._masks = None
    dev = b._split_find(H.cuda(), 7)
    # gains: hardware logf vs libm log over ~10^4-sized terms -> 1e-3 relative for entropy
    torch.testing.assert_close(dev[0].cpu(), host[0], rtol=1e-3 if crit == "entropy" else 1e-5, atol=1e-4)
    assert torch.equal(dev[1].cpu(), host[1]) and torch.equal(dev[2].cpu(), host[2])
    assert torch.equal(dev[3].cpu(), host[3]) and torch.equal(dev[4].cpu(), host[4])


@pytest.mark.gpu
def test_rf_ten_classes_gpu_matches_cpu():
    """10 classes: class-tiled LDS histograms + the class-decomposed split kernel grow the same
    tree as the host engine from the same (integer) statistics."""
    from hivemall_amd.models.trees import HistTreeBuilder, Quantized

    X, y = _ten_class_data(n=20000, seed=1)
    q = quantize(torch.from_numpy(X), 64)
    w = torch.from_numpy(np.random.default_rng(2).integers(0, 3, len(y)).astype(np.float32))
    stats = torch.nn.functional.one_hot(torch.from_numpy(y), 10).float() * w[:, None]
    trees = []
    for dev in ("cpu", "cuda"):
        qd = q if dev == "cpu" else Quantized(q.bins.to(dev), q.edges, q.d, q.B, q.cat)
        b = HistTreeBuilder(qd, "gini", 6, 2.0, 1.0, mtry=3, seed=11)
        trees.append(b.build(stats.to(dev)))
    tc, tg = trees
    assert list(tc.feature) == list(tg.feature)
    np.testing.assert_allclose(np.asarray(tc.threshold, dtype=np.float64),
                               np.asarray(tg.threshold, dtype=np.float64))
    rf = RandomForestClassifier("-trees 4 -max_depth 8 -seed 3", device="cuda").fit(X, y)
    assert (rf.predict(X) == y).mean() > 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("n_classes", [5, 7, 8])
def test_rf_5_to_8_classes_wide_rows_gpu_matches_cpu(n_classes):
    """5..8 classes on 20 features: the statistics fit one <= 160 KB all-features LDS image, but
    the one-pass histogram kernel is instantiated for <= 4 statistics only, so these take the
    feature-group kernel (this shape used to fail with hipErrorInvalidValue)."""
    from hivemall_amd.models.trees import HistTreeBuilder, Quantized

    rng = np.random.default_rng(5)
    X = rng.normal(size=(12000, 20)).astype(np.float32)
    y = (np.floor((X[:, 3] + 3) * n_classes / 6).clip(0, n_classes - 1)).astype(int)
    q = quantize(torch.from_numpy(X), 256)
    stats = torch.nn.functional.one_hot(torch.from_numpy(y), n_classes).float()
    trees = []
    for dev in ("cpu", "cuda"):
        qd = q if dev == "cpu" else Quantized(q.bins.to(dev), q.edges, q.d, q.B, q.cat)
        b = HistTreeBuilder(qd, "gini", 5, 2.0, 1.0, seed=11)
        trees.append(b.build(stats.to(dev)))
    tc, tg = trees
    assert list(tc.feature) == list(tg.feature)
    # the forest trains end to end on the GPU path; its accuracy matches the CPU engine's.  The
    # engines draw different bootstrap / feature-subset streams, so a 4-tree forest's accuracy is
    # seed noise (8 classes, seeds 1..8: CPU 0.86-0.95, GPU 0.78-0.95); at 32 trees CPU
    # 0.883-0.918 (mean 0.897), GPU 0.899-0.944 (mean 0.914) (profiles/r5/rf_multiclass_probe.jsonl)
    acc = {dev: (RandomForestClassifier("-trees 32 -max_depth 8 -seed 3", device=dev).fit(X, y).predict(X) == y).mean()
           for dev in ("cpu", "cuda")}
    assert acc["cuda"] > acc["cpu"] - 0.03, acc


def test_heap_layout_tree_compaction_matches_compact_numbering():
    """A heap-layout build (children of node k at 2k+1, 2k+2; slots of parents that did not
    split stay in the arrays) materialises to the per-level build's compact numbering: the
    reachable nodes in id order, children renumbered (models/trees.py _tree_from_arrays)."""
    from hivemall_amd.models.trees import PendingTree, _tree_from_arrays, materialize_trees

    # depth-2 heap: root 0 splits; node 1 splits, node 2 is a leaf -> slots 5, 6 unreachable
    F = np.array([3, 1, -1, -1, -1, -1, -1], dtype=np.int32)
    T = np.array([0.5, 1.5, np.inf, np.inf, np.inf, np.inf, np.inf], dtype=np.float32)
    Lc = np.array([1, 3, -1, -1, -1, -1, -1], dtype=np.int32)
    Rc = np.array([2, 4, -1, -1, -1, -1, -1], dtype=np.int32)
    V = np.arange(7, dtype=np.float64)[:, None]
    t = _tree_from_arrays(F, T, Lc, Rc, V, 1)
    assert t.feature == [3, 1, -1, -1, -1]
    assert t.left == [1, 3, -1, -1, -1] and t.right == [2, 4, -1, -1, -1]
    assert t.value == [None, None, [2.0], [3.0], [4.0]]
    # a parent that did not split at level 1 (node 1), its sibling did: slots 3, 4 dropped
    F2 = np.array([0, -1, 2, -1, -1, -1, -1], dtype=np.int32)
    Lc2 = np.array([1, -1, 5, -1, -1, -1, -1], dtype=np.int32)
    Rc2 = np.array([2, -1, 6, -1, -1, -1, -1], dtype=np.int32)
    t2 = _tree_from_arrays(F2, T, Lc2, Rc2, V, 1)
    assert t2.feature == [0, -1, 2, -1, -1]
    assert t2.left == [1, -1, 3, -1, -1] and t2.right == [2, -1, 4, -1, -1]
    assert t2.value == [None, [1.0], None, [5.0], [6.0]]
    # deferred trees: one host copy for all of them, leaf values scaled (XGBoost's eta)
    p = PendingTree(torch.from_numpy(F2), torch.from_numpy(T), torch.from_numpy(Lc2), torch.from_numpy(Rc2),
                    torch.from_numpy(V.astype(np.float32)), 1)
    p.scale = 0.5
    (t3,), = materialize_trees([[p]])
    assert t3.feature == t2.feature and t3.value == [None, [0.5], None, [2.5], [3.0]]


@pytest.mark.gpu
def test_gpu_bootstrap_weights_are_a_multinomial_draw():
    """RandomForest bagging on the GPU (csrc hm_bootstrap_counts): per-chunk draw counts from an
    exact multinomial, each chunk's draws counted in LDS.  The multiplicities sum to m, repeat
    for one seed, differ across seeds, and have the bootstrap's moments (mean rate, P(0) =
    e^-rate, variance ~ rate)."""
    from hivemall_amd.models.trees import BOOT_CHUNK, bootstrap_weights

    n = 3 * BOOT_CHUNK + 777
    for rate in (1.0, 0.5):
        m = int(round(n * rate))
        w = [bootstrap_weights(n, rate, torch.Generator(device="cuda").manual_seed(s), "cuda") for s in (5, 5, 6)]
        assert w[0].dtype == torch.float32 and w[0].shape == (n,)
        assert int(w[0].sum().item()) == m and torch.equal(w[0], w[1]) and not torch.equal(w[0], w[2])
        a = w[0].double()
        assert (a == a.round()).all() and (a >= 0).all()
        assert abs(a.mean().item() - rate) < 1e-9 + 1.0 / n
        assert abs((a == 0).double().mean().item() - np.exp(-rate)) < 0.01
        assert abs(a.var().item() - rate) < 0.05
        # no chunk boundary artefact: the last (short) chunk has the same mean
        assert abs(a[-777:].mean().item() - rate) < 0.15
