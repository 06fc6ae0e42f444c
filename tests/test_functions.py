"""Unit tests of the host-side SQL function library (ftvec / tools / evaluation / ensemble /
knn / sketch / geospatial / anomaly)."""
import math

import numpy as np
import pytest

from hivemall_amd import registry
from hivemall_amd.anomaly import changefinder, sst
from hivemall_amd.ensemble import argmin_kld, max_label, maxrow, voted_avg, weight_voted_avg
from hivemall_amd.evaluation import metrics as M
from hivemall_amd.ftvec import functions as F
from hivemall_amd.knn import (cosine_similarity, euclid_distance, hamming_distance, jaccard_similarity,
                              minhashes, topk_similar)
from hivemall_amd.misc import HyperLogLog, approx_count_distinct, bloom, bloom_contains, haversine_distance, lat2tiley, lon2tilex, tile
from hivemall_amd.tools import functions as T
from hivemall_amd.utils.hashing import mhash


def test_registry_covers_survey_inventory():
    registry.load_all()
    must = """train_perceptron train_pa train_pa1 train_pa2 train_cw train_arow train_arowh train_scw
    train_scw2 train_adagrad_rda train_classifier train_multiclass_perceptron train_multiclass_pa
    train_multiclass_pa1 train_multiclass_pa2 train_multiclass_cw train_multiclass_arow
    train_multiclass_arowh train_multiclass_scw train_multiclass_scw2 logress train_logregr
    train_pa1_regr train_pa1a_regr train_pa2_regr train_pa2a_regr train_arow_regr train_arowe_regr
    train_arowe2_regr train_adagrad_regr train_adadelta_regr train_regressor train_fm fm_predict
    train_ffm ffm_predict feature_pairs ffm_features add_field_indices
    cosine_similarity jaccard_similarity angular_similarity euclid_similarity distance2similarity
    dimsum_mapper euclid_distance cosine_distance angular_distance manhattan_distance
    minkowski_distance jaccard_distance hamming_distance popcnt kld minhash minhashes bbit_minhash
    each_top_k changefinder sst add_bias add_feature_index extract_feature extract_weight feature
    feature_index sort_by_feature feature_hashing mhash sha1 array_hash_values prefixed_hash_values
    rescale zscore l1_normalize l2_normalize normalize amplify rand_amplify conv2dense
    to_dense_features to_sparse_features quantify build_bins feature_binning polynomial_features
    powered_features bpr_sampling item_pairs_sampling populate_not_in chi2 snr tf bm25 tfidf
    vectorize_features categorical_features quantitative_features indexed_features
    quantified_features binarize_label onehot_encoding auc logloss mae mse rmse r2 f1score fmeasure
    precision_at recall_at hitrate mrr average_precision ndcg voted_avg weight_voted_avg max_label
    maxrow argmin_kld approx_count_distinct bloom bloom_and bloom_or bloom_not bloom_contains
    bloom_contains_any tile map_url lat2tiley lon2tilex tilex2lon tiley2lat haversine_distance
    lr_datagen array_concat concat_array array_avg array_sum array_remove array_intersect
    array_slice subarray sort_and_uniq_array subarray_endwith subarray_startwith to_string_array
    array_append array_union array_flatten first_element last_element element_at float_array
    select_k_best conditional_emit array_to_str map_get_sum map_tail_n to_map to_ordered_map
    map_include_keys map_exclude_keys map_key_values map_roulette merge_maps to_ordered_list to_bits
    unbits bits_or bits_collect deflate inflate base91 unbase91 tokenize split_words is_stopword
    normalize_unicode word_ngrams singularize sigmoid l2_norm infinity is_finite nan is_nan
    transpose_and_dot vector_add vector_dot rowid rownum taskid jobid jobconf_gets distcache_gets
    generate_series convert_label x_rank try_cast sessionize to_json from_json assert raise_error
    moving_avg max2 min2 rand_gid idf hivemall_version""".split()
    missing = [n for n in must if registry.lookup(n) is None]
    assert not missing, missing


def test_ftvec_basic():
    assert F.add_bias(["1:2", "x"]) == ["1:2", "x", "0:1.0"]
    assert F.add_feature_index([0.5, 2.0]) == ["1:0.5", "2:2.0"]
    assert F.extract_feature("abc:1.5") == "abc" and F.extract_weight("abc:1.5") == 1.5
    assert F.extract_weight("abc") == 1.0
    assert F.feature("a", 2) == "a:2"
    assert F.feature_index(["3:1", "7:2"]) == [3, 7]
    assert F.feature_hashing(["a:2", "b"]) == [f"{mhash('a')}:2", str(mhash("b"))]
    assert 1 <= F.sha1("hello", 100) <= 100
    assert F.rescale(5, 0, 10) == 0.5 and F.zscore(5, 3, 2) == 1.0
    n = F.l2_normalize(["a:3", "b:4"])
    assert n == ["a:0.6", "b:0.8"]
    assert F.to_sparse_features([0.0, 1.5, 0.0]) == ["1:1.5"]
    assert F.to_dense_features(["1:1.5", "3:2"], 3) == [0.0, 1.5, 0.0, 2.0]
    assert "a^b:6.0" in F.polynomial_features(["a:2", "b:3"], 2)
    assert "a^2:4.0" in F.powered_features(["a:2"], 2)
    assert F.vectorize_features(["x", "y", "z"], 1.5, "cat", 0) == ["x:1.5", "y#cat"]
    assert F.categorical_features(["x", "y"], "a", "b") == ["x#a", "y#b"]
    assert F.indexed_features(1.0, 2.0) == ["1:1.0", "2:2.0"]
    assert F.add_field_indices(["a", "b"]) == ["1:a", "2:b"]
    ff = F.ffm_features(["c1", "c2"], "x", 2.0, "-feature_hashing 10")
    assert len(ff) == 2 and ff[0].startswith("0:") and ff[1].startswith("1:")
    bins = F.build_bins(list(range(100)), 4)
    assert len(bins) == 5 and bins[0] == -math.inf
    assert F.feature_binning(30.0, bins) == 1
    rows = list(F.bpr_sampling(7, [1, 2, 3], 10))
    assert len(rows) == 3 and all(r[2] not in (1, 2, 3) for r in rows)
    assert [r[0] for r in F.populate_not_in([0, 2], 3)] == [1, 3]
    assert len(list(F.amplify(3, "a", 1))) == 3
    c = F.chi2([[10, 5], [5, 10]], [[7.5, 7.5], [7.5, 7.5]])
    assert len(c["chi2"]) == 2 and 0 <= c["pvalue"][0] <= 1
    assert F.tf(["a", "b", "a"])["a"] == pytest.approx(2 / 3)
    assert F.bm25(3, 100, 120, 1000, 10) > 0
    assert F.onehot_encoding(["a", "b", "a"], [1, 2])[0] == {"a": 1, "b": 2}


def test_evaluation_metrics():
    s = np.array([0.9, 0.8, 0.7, 0.3, 0.2])
    y = np.array([1, 1, 0, 1, 0])
    from sklearn.metrics import log_loss, roc_auc_score
    assert M.auc(s, y) == pytest.approx(roc_auc_score(y, s))
    assert M.logloss(s, y) == pytest.approx(log_loss(y, s))
    p, a = [1.0, 2.0, 3.0], [1.5, 2.0, 2.0]
    assert M.mae(p, a) == pytest.approx(0.5)
    assert M.rmse(p, a) == pytest.approx(math.sqrt(1.25 / 3))
    assert M.r2(a, a) == 1.0
    part = M.regression_partial(p, a)
    assert M.regression_merge(part)["mae"] == pytest.approx(0.5)
    assert M.f1score([[1, 2]], [[1, 3]]) == pytest.approx(0.5)
    assert M.fmeasure([1, 0, 1], [1, 1, 0], "-average binary") == pytest.approx(0.5)
    rank, truth = [[1, 2, 3, 4]], [[2, 4]]
    assert M.precision_at(rank, truth, [2]) == 0.5
    assert M.recall_at(rank, truth) == 1.0
    assert M.mrr(rank, truth) == 0.5
    assert M.hitrate(rank, truth, [1]) == 0.0
    assert M.average_precision(rank, truth) == pytest.approx((1 / 2 + 2 / 4) / 2)
    assert 0 < M.ndcg(rank, truth) < 1
    assert M.auc([[1, 2, 3]], [[1]]) == 1.0


def test_ensemble():
    assert voted_avg([1.0, 2.0, -1.0]) == 1.5
    assert weight_voted_avg([1.0, -5.0, 2.0]) == -5.0
    assert max_label([0.1, 0.9, 0.5], ["a", "b", "c"]) == "b"
    assert maxrow([0.1, 0.9], ["a", "b"]) == [0.9, "b"]
    assert argmin_kld([1.0, 3.0], [1.0, 1.0]) == 2.0
    assert argmin_kld([1.0, 3.0], [1.0, 3.0]) == pytest.approx((1 + 1) / (1 + 1 / 3))


def test_knn_and_lsh():
    assert cosine_similarity(["a:1", "b:1"], ["a:1", "b:1"]) == pytest.approx(1.0)
    assert jaccard_similarity(["a", "b"], ["b", "c"]) == pytest.approx(1 / 3)
    assert euclid_distance([0.0, 0.0], [3.0, 4.0]) == 5.0
    assert hamming_distance(0b1011, 0b0001) == 2
    a = minhashes(["a", "b", "c", "d"], False, 5, 2)
    assert a == minhashes(["d", "c", "b", "a"], False, 5, 2) and len(a) == 5
    import torch
    X = torch.randn(50, 8)
    sc, ix = topk_similar(X, k=3)
    assert ix.shape == (50, 3) and not (ix == torch.arange(50)[:, None]).any()


def test_sketch_geo():
    h = HyperLogLog(12)
    for i in range(20000):
        h.add(i)
    assert abs(h.cardinality() - 20000) / 20000 < 0.05
    assert approx_count_distinct(["a", "b", "a"]) == 2
    b = bloom(["x", "y"])
    assert bloom_contains(b, "x") and not bloom_contains(b, "zzz-not-there")
    assert lon2tilex(0, 1) == 1 and lat2tiley(0, 1) == 1
    assert tile(0.0, 0.0, 1) == 3
    assert haversine_distance(35.6, 139.7, 35.6, 139.7) == 0.0


def test_tools():
    assert T.array_concat([1], [2, 3]) == [1, 2, 3]
    assert T.array_avg([[1, 2], [3, 4]]) == [2.0, 3.0]
    assert T.array_slice([1, 2, 3, 4], 1, 2) == [2, 3]
    assert T.array_intersect([1, 2, 3], [2, 3, 4]) == [2, 3]
    assert T.sort_and_uniq_array([3, 1, 3]) == [1, 3]
    assert T.subarray_endwith([1, 2, 3, 2, 5], 2) == [1, 2, 3, 2]
    assert T.select_k_best([10, 20, 30], [0.1, 0.9, 0.5], 2) == [20, 30]
    assert T.unbits(T.to_bits([1, 3, 64])) == [1, 3, 64]
    assert T.inflate(T.deflate("hello")) == "hello"
    assert T.unbase91(T.base91("hello")) == b"hello"
    assert T.tokenize("Hello, world!") == ["Hello", "world"]
    assert T.word_ngrams(["a", "b", "c"], 1, 2) == ["a", "b", "c", "a b", "b c"]
    assert T.singularize("apples") == "apple" and T.singularize("children") == "child"
    assert T.sigmoid(0) == 0.5
    assert T.to_ordered_list([3, 1, 2]) == [1, 2, 3]
    assert T.to_ordered_list(["a", "b", "c"], [3, 1, 2], "-k 2") == ["a", "c"]
    vals, keys = ["a", "b", "c", "d", "e"], [3, 1, 2, 1, 5]
    assert T.to_ordered_list(vals, keys, "-k -2") == ["b", "d"]          # smallest, ties in order
    assert T.to_ordered_list(vals, keys, "-k 3 -reverse") == ["b", "d", "c"]
    assert T.to_ordered_list(vals, keys, "-k 0") == []
    assert T.to_ordered_list(vals, keys, "-k 9") == ["e", "a", "c", "b", "d"]
    rng = np.random.default_rng(0)
    ks = rng.integers(0, 50, 400).tolist()
    vs = list(range(400))
    full = sorted(vs, key=lambda i: ks[i], reverse=True)
    assert T.to_ordered_list(vs, ks, "-k 37") == full[:37]       # bounded heap == stable sort
    assert T.convert_label(0) == -1 and T.convert_label(-1) == 0
    assert [r[0] for r in T.generate_series(1, 3)] == [1, 2, 3]
    assert T.from_json(T.to_json({"a": [1, 2]})) == {"a": [1, 2]}
    assert T.transpose_and_dot([[1, 2]], [[3, 4]]) == [[3.0, 4.0], [6.0, 8.0]]
    assert T.map_tail_n({1: "a", 2: "b", 3: "c"}, 2) == {2: "b", 3: "c"}


def test_anomaly_detects_level_shift():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.normal(0, 1, 300), rng.normal(6, 1, 300)])
    cp = np.array([c[1] for c in changefinder(x, "-k 3")])
    assert 295 <= cp[100:].argmax() + 100 <= 330
    # SST detects a change of the series' pattern (here: its frequency)
    t = np.arange(600)
    x2 = np.where(t < 300, np.sin(t / 3.0), np.sin(t / 1.2)) + rng.normal(0, 0.1, 600)
    s = np.array([c[0] for c in sst(x2, "-w 20")])
    assert 300 <= s.argmax() <= 360 and s[:290].max() < 0.1 * s.max()


@pytest.mark.gpu
def test_mhash_kernel_bit_exact():
    import random
    from hivemall_amd.utils.hashing import mhash_batch, mhash_device, murmur3_batch
    rng = random.Random(0)
    words = ["", "a", "ab", "abc", "abcd", "feature_name_42", "日本語", "x" * 5000] + \
        ["".join(rng.choice("abcdefghij:0123456789_") for _ in range(rng.randint(1, 40))) for _ in range(20000)]
    for nf in (1 << 24, 1000, 0):
        got = mhash_device(words, nf).cpu().numpy()
        ref = murmur3_batch(words) if nf == 0 else mhash_batch(words, nf)
        assert (got == ref).all(), nf


def test_bpr_sampling_is_stable_across_hash_seeds():
    """The per-user stream must not depend on Python's salted ``hash()``: two interpreters
    with different PYTHONHASHSEED emit identical triples for string and int users."""
    import os
    import subprocess
    import sys

    code = ("import hivemall_amd.ftvec.functions as F;"
            "print([list(F.bpr_sampling(u, [1, 5, 9], 50, '-seed 7 -sampling_rate 2')) "
            "for u in ('alice', 'bob', 42)])")
    outs = []
    for hs in ("1", "12345"):
        env = dict(os.environ, PYTHONHASHSEED=hs)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout)
    assert outs[0] == outs[1] and outs[0].count("(") == 18
    a = list(F.bpr_sampling("alice", [1, 5, 9], 50, "-seed 7"))
    b = list(F.bpr_sampling("alice", [1, 5, 9], 50, "-seed 8"))
    assert a != b


def test_rand_amplify_seed_and_streaming():
    amp = F.RandAmplifier(3, 16, seed=5)
    src = ((i,) for i in range(1000))                  # a generator: never materialised
    it = amp.run(src)
    first = [next(it) for _ in range(10)]
    assert all(r[0] < 20 for r in first)               # reservoir of 16 rows, 3 copies each
    rest = list(it)
    assert sorted(r[0] for r in first + rest) == sorted(list(range(1000)) * 3)
    a = F.rand_amplify(2, 50, list(range(200)), "-seed 1")
    b = F.rand_amplify(2, 50, list(range(200)), "-seed 1")
    c = F.rand_amplify(2, 50, list(range(200)), "-seed 2")
    assert a["c0"].tolist() == b["c0"].tolist() != c["c0"].tolist()
    assert sorted(a["c0"].tolist()) == sorted(list(range(200)) * 2)


def test_add_feature_index_vectorised_matches_rowwise():
    """The column path (hm_format_feature_index: Python repr digits via std::to_chars) gives the
    per-row strings exactly, nulls skipped with their positions kept; non-finite values fall
    back to the per-row path and raise as before."""
    import numpy as np
    import pandas as pd
    import pytest

    from hivemall_amd.ftvec import functions as F

    rng = np.random.default_rng(3)
    rows = []
    for _ in range(3000):
        row = []
        for _ in range(int(rng.integers(0, 8))):
            t = int(rng.integers(0, 7))
            row.append([int(rng.integers(-10**6, 10**6)), float(rng.standard_normal()),
                        float(rng.standard_normal() * 10.0 ** rng.integers(-12, 20)), None,
                        float(10.0 ** rng.integers(14, 18)) * float(rng.choice([1, -1, 2.5])), -0.0,
                        float(np.float32(rng.random()))][t])
        rows.append(row if rng.random() > 0.05 else None)
    got = F.add_feature_index(pd.Series(rows, dtype=object)).tolist()
    norm = lambda a: None if a is None or a is pd.NA else list(a)
    assert [norm(a) for a in got] == [F._add_feature_index1(r) for r in rows]
    assert F.add_feature_index([1, 2.5, None, 1e-7]) == ["1:1.0", "2:2.5", "4:1e-07"]
    with pytest.raises((ValueError, OverflowError)):
        F.add_feature_index(pd.Series([[1.0, float("nan")]], dtype=object))


def test_normalize_vectorised_matches_rowwise():
    """l1 / l2_normalize over a column (hm_normalize_features) equal the per-row rule bit for
    bit: bare names, "name:v" and "field:index:v" forms, zero-norm rows, null rows."""
    import numpy as np
    import pandas as pd

    from hivemall_amd.ftvec import functions as F

    rng = np.random.default_rng(7)

    def val():
        return [str(int(rng.integers(-50, 50))), repr(float(rng.standard_normal())), f"{rng.random():.3e}",
                "0", repr(float(rng.standard_normal() * 1e12)), f"{rng.random():.4f}"][int(rng.integers(0, 6))]
    rows = []
    for _ in range(2000):
        row = []
        for j in range(int(rng.integers(0, 10))):
            t = int(rng.integers(0, 4))
            row.append([f"f{j}", f"f{j}:{val()}", f"{j}:{int(rng.integers(0, 99))}:{val()}", f"{j}:0"][t])
        rows.append(row if rng.random() > 0.03 else None)
    col = pd.Series(rows, dtype=object)
    norm = lambda a: None if a is None or a is pd.NA else list(a)
    for fn, p in ((F.l1_normalize, 1), (F.l2_normalize, 2)):
        assert [norm(a) for a in fn(col).tolist()] == [F._normalize(r, p) for r in rows]
    # a value the plain parser does not take (spaces) sends the column down the per-row path
    assert F.l2_normalize(pd.Series([["a: 3", "b:4"]], dtype=object)).tolist() == [["a:0.6", "b:0.8"]]


def test_vectorised_math_udfs_match_rowwise():
    """sigmoid (native, libm exp) / rescale / zscore over numeric columns equal the per-row
    Python bit for bit, with per-row semantics for constants, equal bounds, zero stddev, +-inf."""
    import numpy as np
    import pandas as pd

    from hivemall_amd.ftvec import functions as F
    from hivemall_amd.tools import functions as T

    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000) * 30, [0.0, -0.0, 700, -700, 745, -745, np.inf, -np.inf]])
    got = T.sigmoid(pd.Series(x)).to_numpy()
    want = np.array([T._sigmoid1(v) for v in x])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    lo = pd.Series(rng.standard_normal(len(x)))
    hi = lo + pd.Series(rng.random(len(x)))
    hi[:10] = lo[:10]
    xs = pd.Series(x)
    for fn, f1, args in ((F.rescale, F._rescale1, (xs, lo, hi)), (F.rescale, F._rescale1, (xs, -3.0, 5.0)),
                         (F.zscore, F._zscore1, (xs, lo, hi)), (F.zscore, F._zscore1, (xs, 0.5, 0.0))):
        g = fn(*args).to_numpy()
        cols = [a.tolist() if isinstance(a, pd.Series) else [a] * len(xs) for a in args]
        w = np.array([f1(*r) for r in zip(*cols)], dtype=float)
        assert np.array_equal(g, w, equal_nan=True), fn.__name__
    assert F.rescale(pd.Series(["a:3", "b:7"]), 0, 10).tolist() == ["a:0.3", "b:0.7"]
