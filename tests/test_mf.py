import numpy as np
import pandas as pd
import pytest
import torch

from hivemall_amd.io.synthetic import movielens_like
from hivemall_amd.models.mf import (BPRMF, MatrixFactorization, MatrixFactorizationAdaGrad,
                                    auc_implicit, bprmf_predict, mf_predict)
from hivemall_amd.sql import Session


def _ratings(n=40000, nu=500, ni=300, k=5, seed=0):
    rng = np.random.default_rng(seed)
    P = rng.normal(0, 1, (nu, k))
    Q = rng.normal(0, 1, (ni, k))
    u = rng.integers(0, nu, n)
    i = rng.integers(0, ni, n)
    r = (P[u] * Q[i]).sum(1) + 3 + rng.normal(0, 0.1, n)
    return u, i, r.astype(np.float32)


def _oracle_sgd(u, i, r, P, Q, mu, eta, lam):
    P, Q = P.astype(np.float64).copy(), Q.astype(np.float64).copy()
    Bu, Bi = np.zeros(P.shape[0]), np.zeros(Q.shape[0])
    for a, b, x in zip(u, i, r):
        e = x - (mu + Bu[a] + Bi[b] + P[a] @ Q[b])
        pa = P[a].copy()
        P[a] += eta * (e * Q[b] - lam * P[a])
        Q[b] += eta * (e * pa - lam * Q[b])
        Bu[a] += eta * (e - lam * Bu[a])
        Bi[b] += eta * (e - lam * Bi[b])
    return P, Q, Bu, Bi


def test_mf_sgd_matches_oracle():
    u, i, r = _ratings(2000)
    m = MatrixFactorization("-factors 4 -iters 1 -eta0 0.01 -mu 3", device="cpu")
    m.init_state(500, 300)
    P0, Q0 = m.state["P"].numpy().copy(), m.state["Q"].numpy().copy()
    m.fit(u, i, r)
    P, Q, Bu, Bi = _oracle_sgd(u, i, r, P0, Q0, 3.0, 0.01, 0.03)
    np.testing.assert_allclose(m.state["P"].numpy(), P, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(m.state["Bi"].numpy(), Bi, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("cls,opts", [(MatrixFactorization, "-eta0 0.01"), (MatrixFactorizationAdaGrad, "-eta0 0.1")])
def test_mf_learns(cls, opts):
    u, i, r = _ratings()
    m = cls(f"-factors 10 -iters 20 -update_mean {opts}", device="cpu").fit(u[:35000], i[:35000], r[:35000])
    pr = m.predict(u[35000:], i[35000:])
    assert np.sqrt(((pr - r[35000:]) ** 2).mean()) < 0.3 * r.std()
    tab = m.model_table()
    assert list(tab.columns) == ["idx", "Pu", "Qi", "Bu", "Bi", "mu"]
    row = tab.iloc[3]
    assert mf_predict(row.Pu, row.Qi, row.Bu, row.Bi, row.mu) == pytest.approx(
        m.predict([row.idx], [row.idx])[0], rel=1e-4, abs=1e-4)


def test_bprmf_triples_and_device_sampling_cpu():
    us, its = movielens_like(100000, 1000, 500, k=8)
    m = BPRMF("-factors 16 -iters 10 -eta0 0.05", device="cpu").fit_implicit(us[:95000], its[:95000], 1000, 500)
    assert auc_implicit(m, us[95000:].numpy(), its[95000:].numpy()) > 0.65
    rng = np.random.default_rng(0)
    u = us[:20000].numpy()
    i = its[:20000].numpy()
    j = rng.integers(0, 500, 20000)
    m2 = BPRMF("-factors 8 -iters 3", device="cpu").fit(u, i, j)
    tab = m2.model_table()
    assert list(tab.columns) == ["idx", "Pu", "Qi", "Bi"]
    s, ix = m2.recommend_topk([0, 1], k=5)
    assert ix.shape == (2, 5)
    r = tab.iloc[0]
    assert isinstance(bprmf_predict(r.Pu, r.Qi, r.Bi), float)


def test_mf_sql():
    u, i, r = _ratings(5000)
    s = Session(device="cpu")
    s.register("ratings", pd.DataFrame({"userid": u, "itemid": i, "rating": r}))
    s.sql("CREATE TABLE mf AS SELECT train_mf_sgd(userid, itemid, rating, '-factors 5 -iters 5 -eta0 0.01') "
          "AS (idx, Pu, Qi, Bu, Bi, mu) FROM ratings")
    p = s.sql("""SELECT t.rating, mf_predict(p.Pu, q.Qi, p.Bu, q.Bi, p.mu) AS pred FROM ratings t
                 JOIN mf p ON (t.userid = p.idx) JOIN mf q ON (t.itemid = q.idx)""")
    assert len(p) == 5000 and np.isfinite(p["pred"].astype(float)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("cls,opts", [(MatrixFactorization, "-eta0 0.01"), (MatrixFactorizationAdaGrad, "-eta0 0.1")])
def test_mf_gpu_matches_cpu_on_disjoint_pairs(cls, opts):
    n = 300
    u = np.arange(n)
    i = np.arange(n)
    r = np.random.default_rng(1).normal(3, 1, n).astype(np.float32)
    res = {}
    for dev in ("cpu", "cuda"):
        m = cls(f"-factors 10 -iters 1 {opts}", device=dev).fit(u, i, r)
        res[dev] = {k: v.cpu() for k, v in m.state.items()}
    for k in ("P", "Q", "Bu", "Bi"):
        np.testing.assert_allclose(res["cuda"][k].numpy(), res["cpu"][k].numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_mf_gpu_quality():
    u, i, r = _ratings()
    res = {}
    for dev in ("cpu", "cuda"):
        m = MatrixFactorization("-factors 10 -iters 20 -eta0 0.01 -update_mean", device=dev).fit(
            u[:35000], i[:35000], r[:35000])
        pr = m.predict(u[35000:], i[35000:])
        res[dev] = float(np.sqrt(((pr - r[35000:]) ** 2).mean()))
    assert res["cuda"] < res["cpu"] * 1.5 + 0.05, res


@pytest.mark.gpu
@pytest.mark.parametrize("cls,opts", [(MatrixFactorization, "-eta0 0.01"), (MatrixFactorizationAdaGrad, "-eta0 0.1")])
def test_mf_gpu_wide_grid_learns_factors(cls, opts):
    """Hogwild at -grid 9 / 36 (up to 576 ratings in flight on a 300-item catalogue): with the
    atomic delta updates the factors are learned as sequentially (plain read-modify-write
    stores lost most concurrent updates and stayed at the bias-only RMSE 2.25;
    profiles/mf_atomic_r2/)."""
    u, i, r = _ratings()
    base = cls(f"-factors 10 -iters 20 -disable_cv -update_mean {opts}", device="cpu").fit(u[:35000], i[:35000], r[:35000])
    ref = float(np.sqrt(((base.predict(u[35000:], i[35000:]) - r[35000:]) ** 2).mean()))
    for grid in (9, 36):
        m = cls(f"-factors 10 -iters 20 -disable_cv -update_mean -grid {grid} {opts}", device="cuda").fit(
            u[:35000], i[:35000], r[:35000])
        rmse = float(np.sqrt(((m.predict(u[35000:], i[35000:]) - r[35000:]) ** 2).mean()))
        assert rmse < ref * 1.1 + 0.02, (grid, rmse, ref)


@pytest.mark.gpu
def test_bpr_gpu_explicit_triples_match_cpu():
    n = 200
    u, i, j = np.arange(n), np.arange(n), np.arange(n, 2 * n)
    res = {}
    for dev in ("cpu", "cuda"):
        m = BPRMF("-factors 16 -iters 1 -eta0 0.05", device=dev).fit(u, i, j)
        res[dev] = {k: v.cpu() for k, v in m.state.items()}
    for k in ("P", "Q", "Bi"):
        np.testing.assert_allclose(res["cuda"][k].numpy(), res["cpu"][k].numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_bpr_gpu_device_sampling_quality():
    us, its = movielens_like(400000, 5000, 2000, k=8)
    res = {}
    for dev in ("cpu", "cuda"):
        m = BPRMF("-factors 32 -iters 10 -eta0 0.05", device=dev).fit_implicit(us[:380000], its[:380000], 5000, 2000)
        res[dev] = auc_implicit(m, us[380000:].numpy(), its[380000:].numpy())
    assert res["cuda"] > res["cpu"] - 0.03, res


@pytest.mark.gpu
def test_bpr_gpu_pipelined_kernel_quality_matches_pf(monkeypatch):
    """The three-stage pipelined BPR kernel (bpr_pf3_kernel, the default with device sampling)
    draws exactly bpr_pf_kernel's triples and reads a row at most one update staler: the same
    sampled AUC within 0.01 (k = 64: one triple per wave; k = 16: four)."""
    us, its = movielens_like(400000, 5000, 2000, k=8)
    for k in (64, 16):
        res = {}
        for var in ("2", "0"):
            monkeypatch.setenv("HM_BPR_VARIANT", var)
            m = BPRMF(f"-factors {k} -iters 6 -eta0 0.05 -seed 4", device="cuda").fit_implicit(
                us[:380000], its[:380000], 5000, 2000)
            res[var] = auc_implicit(m, us[380000:].numpy(), its[380000:].numpy())
        assert abs(res["0"] - res["2"]) < 0.01 and res["0"] > 0.6, (k, res)


@pytest.mark.parametrize("cls", ["bpr", "mf"])
def test_bold_driver_eta_follows_the_rule(cls):
    """-eta bolddriver (AdjustingEtaEstimator): x1.05 after a loss decrease, x0.5 after an
    increase, capped at 1.0; the kernel is fed the adjusted rate every epoch."""
    from hivemall_amd.models.mf import BPRMF, MatrixFactorization

    rng = np.random.default_rng(0)
    u, i, j = rng.integers(0, 40, 600), rng.integers(0, 60, 600), rng.integers(0, 60, 600)
    if cls == "bpr":
        m = BPRMF("-factors 4 -iters 6 -disable_cv -eta bolddriver -eta0 0.3", device="cpu")
        m.fit(u, i, j)
    else:
        m = MatrixFactorization("-factors 4 -iters 6 -disable_cv -eta bold_driver -eta0 0.9",
                                device="cpu")
        m.fit(u, i, rng.random(600) * 5)
    losses = m.cv.history
    etas = m.bold.history
    assert len(etas) == len(losses) + 1 and len(losses) == 6
    for k in range(1, len(losses)):
        mult = 0.5 if losses[k] > losses[k - 1] else 1.05
        assert etas[k + 1] == pytest.approx(min(1.0, etas[k] * mult), rel=1e-12)
    assert etas[1] == etas[0]             # no previous loss after the first epoch
    assert max(etas) <= 1.0


def test_inert_option_warns(caplog):
    import logging

    from hivemall_amd.models.mf import MatrixFactorization
    from hivemall_amd.utils import options as O

    O._warned.clear()
    with caplog.at_level(logging.WARNING, logger="hivemall_amd"):
        MatrixFactorization("-factors 4 -scale 10", device="cpu")
    assert any("-scale" in r.getMessage() and "no effect" in r.getMessage() for r in caplog.records)


def test_bpr_grid_rule_rounds_up_to_a_power_of_two():
    """BPRMF._grid: 1 block per 32 items / users (the contention rule), rounded up to a power of
    two once it reaches 256 blocks (ML-20M: 852 -> 1,024, profiles/r6/bpr_grid/); an explicit
    -grid is kept as given."""
    m = BPRMF("-factors 8")
    m.n_users, m.n_items = 138493, 27278
    assert m._grid() == 1024
    m.n_users, m.n_items = 5000, 4000          # 125 blocks: below the rounding threshold
    assert m._grid() == 125
    m.n_users, m.n_items = 10 ** 7, 10 ** 7    # capped
    assert m._grid() == 4096
    m2 = BPRMF("-factors 8 -grid 852")
    m2.n_users, m2.n_items = 138493, 27278
    assert m2._grid() == 852
