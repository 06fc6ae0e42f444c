import numpy as np
import pandas as pd
import pytest

from hivemall_amd.models.recommend import KPA, SLIM
from hivemall_amd.models.topicmodel import LDA, PLSA, lda_predict, plsa_predict
from hivemall_amd.sql import Session


def _docs(n=300, seed=0):
    rng = np.random.default_rng(seed)
    A = [f"a{i}" for i in range(20)]
    B = [f"b{i}" for i in range(20)]
    return [list(rng.choice(A if d % 2 == 0 else B, 30)) for d in range(n)]


def test_lda_separates_topics():
    docs = _docs()
    m = LDA("-topics 2 -iters 5", device="cpu").fit(docs)
    th = m.transform(docs[:10])
    lab = th.argmax(1)
    assert (lab[0::2] == lab[0]).all() and (lab[1::2] != lab[0]).all() and th.max(1).min() > 0.8
    tab = m.model_table()
    assert list(tab.columns) == ["label", "word", "lambda"]
    sub = tab[tab.word.isin(docs[0])]
    pred = lda_predict(sub.word.tolist(), [1] * len(sub), sub.label.tolist(), sub["lambda"].tolist(), "-topics 2")
    assert pred[0][0] == lab[0] and pred[0][1] > 0.8


def test_plsa_separates_topics():
    docs = _docs()
    m = PLSA("-topics 2 -iters 5", device="cpu").fit(docs)
    th = m.transform(docs[:10])
    assert (th.argmax(1)[0::2] == th.argmax(1)[0]).all() and (th.argmax(1)[1::2] != th.argmax(1)[0]).all()
    tab = m.model_table()
    sub = tab[tab.word.isin(docs[1])]
    p = plsa_predict(sub.word.tolist(), [1] * len(sub), sub.label.tolist(), sub["prob"].tolist())
    assert p[0][0] == th.argmax(1)[1]


def test_lda_sql():
    s = Session(device="cpu")
    s.register("docs", pd.DataFrame({"docid": range(100), "words": _docs(100)}))
    t = s.sql("SELECT train_lda(words, '-topics 2 -iters 3') AS (label, word, lambda) FROM docs")
    assert set(t.columns) == {"label", "word", "lambda"} and len(t) == 80


def test_slim_recovers_item_relation():
    rng = np.random.default_rng(0)
    users = range(50)
    r0 = {u: float(rng.integers(1, 5)) for u in users}
    r1 = {u: 2 * v for u, v in r0.items()}            # item 1 = 2 x item 0
    r2 = {u: float(rng.integers(1, 5)) for u in users}  # unrelated
    m = SLIM("-l1 0.0 -l2 0.0 -iters 100", device="cpu").fit([0, 0], [r0, r0], [None, None], [1, 2], [r1, r2])
    tab = m.model_table()
    w = {(int(a), int(b)): v for a, b, v in tab.itertuples(index=False)}
    assert w[(0, 1)] == pytest.approx(0.5, rel=0.05) and w.get((0, 2), 0.0) < 0.05


def test_kpa_learns_xor():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(2000, 2))
    y = (X[:, 0] * X[:, 1] > 0).astype(int)
    feats = [[f"a:{a}", f"b:{b}"] for a, b in X]
    m = KPA("-iters 3", device="cpu").fit(feats, y)
    acc = ((m.decision_function(feats) > 0) == (y > 0)).mean()
    assert acc > 0.9
    assert list(m.model_table().columns) == ["h", "hk", "w0", "w1", "w2", "w3"]


def _slim_scalar(G, b, l1, l2, iters, eps):
    """Per-item scalar coordinate descent (the residual-form loop of upstream SlimUDTF)."""
    w = np.zeros(len(b))
    for _ in range(iters):
        dmax = 0.0
        for k in range(len(b)):
            if G[k, k] == 0:
                continue
            rho = b[k] - G[k] @ w + G[k, k] * w[k]
            nw = max(0.0, rho - l1) / (G[k, k] + l2)
            dmax = max(dmax, abs(nw - w[k]))
            w[k] = nw
        if dmax < eps:
            break
    return w


def test_slim_batched_cd_matches_scalar_loop():
    from hivemall_amd.models.recommend import slim_cd_batched

    rng = np.random.default_rng(3)
    Gs, bs = [], []
    for m in (3, 7, 5, 1, 6):
        X = rng.random((20, m)) * (rng.random((20, m)) < 0.4)
        y = rng.random(20) * (rng.random(20) < 0.5)
        Gs.append(X.T @ X)
        bs.append(X.T @ y)
    W = slim_cd_batched(Gs, bs, 0.01, 0.05, 50, 1e-6)
    for t, (G, b) in enumerate(zip(Gs, bs)):
        np.testing.assert_allclose(W[t, :len(b)], _slim_scalar(G, b, 0.01, 0.05, 50, 1e-6),
                                   rtol=1e-9, atol=1e-12)
        assert (W[t, len(b):] == 0).all()


def test_slim_batched_cd_chunks_by_neighbourhood_size(monkeypatch):
    """Items are solved in size-sorted chunks of bounded Gram bytes; the result is the one-shot
    padded solve's (one large kNN union must not size every item's Gram matrix)."""
    from hivemall_amd.models import recommend as R

    rng = np.random.default_rng(5)
    Gs, bs = [], []
    for m in list(rng.integers(1, 6, size=40)) + [30]:
        X = rng.random((50, m)) * (rng.random((50, m)) < 0.4)
        Gs.append(X.T @ X)
        bs.append(X.T @ rng.random(50))
    full = R.slim_cd_batched(Gs, bs, 0.01, 0.05, 40, 1e-8)
    monkeypatch.setattr(R, "_SLIM_CHUNK_BYTES", 4 * 6 * 6 * 8)      # <= 4 small items per chunk
    chunked = R.slim_cd_batched(Gs, bs, 0.01, 0.05, 40, 1e-8)
    np.testing.assert_allclose(chunked, full, rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
def test_slim_batched_cd_gpu_matches_cpu():
    import torch

    from hivemall_amd.models.recommend import slim_cd_batched

    rng = np.random.default_rng(4)
    Gs, bs = [], []
    for _ in range(300):
        m = int(rng.integers(1, 20))
        X = rng.random((40, m)) * (rng.random((40, m)) < 0.3)
        Gs.append(X.T @ X)
        bs.append(X.T @ rng.random(40))
    a = slim_cd_batched(Gs, bs, 0.001, 0.0005, 30, 1e-4, torch.device("cuda"))
    b = slim_cd_batched(Gs, bs, 0.001, 0.0005, 30, 1e-4)
    np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [10, 100])
def test_lda_estep_kernel_matches_torch(K):
    """The fused gfx950 E-step (csrc/kernels/lda.hip) against the torch formulation on the CPU:
    same documents, same initial gamma, a fixed number of inner iterations."""
    import torch
    from hivemall_amd.models.topicmodel import LDA, _flatten

    rng = np.random.default_rng(0)
    V, B = 500, 64
    rows = [[(int(w), float(rng.integers(1, 4))) for w in rng.choice(V, size=int(rng.integers(5, 120)), replace=False)]
            for _ in range(B)]
    res = {}
    for dev in ("cpu", "cuda"):
        m = LDA(f"-topics {K} -delta 1e-12 -max_inner_iters 30", device=dev)
        torch.manual_seed(1)
        m._grow(V)
        doc, w, c = _flatten(rows, dev)
        Eb = torch.exp(m._elog(m.lam, 1))
        torch.manual_seed(2)
        g, contrib = m.e_step(doc, w, c, B, Eb)
        res[dev] = (g.cpu(), contrib.cpu())
    np.testing.assert_allclose(res["cuda"][0].numpy(), res["cpu"][0].numpy(), rtol=2e-3, atol=1e-4)
    np.testing.assert_allclose(res["cuda"][1].numpy(), res["cpu"][1].numpy(), rtol=2e-3, atol=1e-5)


@pytest.mark.gpu
def test_lda_gpu_learns_topics():
    from hivemall_amd.models.topicmodel import LDA
    rng = np.random.default_rng(1)
    topics = [[f"a{i}" for i in range(20)], [f"b{i}" for i in range(20)]]
    docs = [list(rng.choice(topics[d % 2], size=15)) for d in range(400)]
    m = LDA("-topics 2 -iters 5", device="cuda").fit(docs)
    th = m.transform(docs[:40])
    assert (th.argmax(1)[::2] != th.argmax(1)[1::2]).mean() > 0.9
