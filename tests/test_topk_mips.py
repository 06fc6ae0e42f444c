"""Fused MFMA top-k inner-product search (ops/topk_mips.py, csrc/kernels/topk_mips.hip).

CPU tests pin the contract on the torch path (score desc, then item index asc; exclusions;
row/item bias; split merge).  GPU tests compare the gfx950 kernel against a plain fp32/fp64
PyTorch reference of the same op on the same bf16-rounded operands:
  * integer-valued operands (exact in bf16 and in fp32 sums) -> indices must match exactly,
    including the tie order, for every Kd / k / split / exclusion combination;
  * random operands -> the returned score lists match the reference's sorted top-k values
    and every returned index scores what the kernel says it does.
"""
import numpy as np
import pytest
import torch

from hivemall_amd.ops.topk_mips import _merge, exclusion_csr, mips_topk


def _ref(Q, I, k, bias=None, ex=None, self_off=None):
    S = Q.double() @ I.double().T
    if bias is not None:
        S += bias.double()[None, :]
    M, N = S.shape
    if self_off is not None:
        for q in range(M):
            if 0 <= q + self_off < N:
                S[q, q + self_off] = -float("inf")
    if ex is not None:
        ptr, it = ex
        for q in range(M):
            S[q, it[ptr[q]:ptr[q + 1]].long()] = -float("inf")
    return S


def _check_exact(ix, sc, S, k):
    """Exact comparison with the (score desc, index asc) order of the reference matrix."""
    M, N = S.shape
    ar = torch.arange(N, dtype=torch.float64)
    for q in range(M):
        row = S[q]
        order = sorted(range(N), key=lambda n: (-row[n].item(), n))
        want = [n for n in order if row[n] != -float("inf")][:k]
        got = [int(v) for v in ix[q].tolist() if v >= 0]
        assert got == want, (q, got[:8], want[:8])
        np.testing.assert_allclose(sc[q, : len(want)].double().cpu().numpy(), row[want].numpy(), rtol=0, atol=0)
    del ar


def _int_data(M, N, d, seed):
    g = torch.Generator().manual_seed(seed)
    Q = torch.randint(-3, 4, (M, d), generator=g).float()
    I = torch.randint(-3, 4, (N, d), generator=g).float()
    return Q, I


def test_cpu_path_exact_order_and_exclusion():
    Q, I = _int_data(37, 301, 10, 0)
    bias = torch.randint(-2, 3, (301,)).float()
    rows = torch.randint(0, 37, (400,))
    items = torch.randint(0, 301, (400,))
    ex = exclusion_csr(rows, items, 37)
    ix, sc = mips_topk(Q, I, 12, item_bias=bias, exclude=ex)
    _check_exact(ix, sc, _ref(Q, I, 12, bias, ex), 12)


def test_cpu_self_exclusion_and_row_bias():
    Q, _ = _int_data(50, 50, 8, 1)
    rb = torch.arange(50).float()
    ix, sc = mips_topk(Q, Q, 5, row_bias=rb, exclude_self_offset=0)
    assert not (ix == torch.arange(50)[:, None]).any()
    ix0, sc0 = mips_topk(Q, Q, 5, exclude_self_offset=0)
    assert torch.equal(ix, ix0)
    assert torch.allclose(sc - rb[:, None], sc0)


def test_cpu_fewer_items_than_k():
    Q, I = _int_data(4, 3, 4, 2)
    ix, sc = mips_topk(Q, I, 8)
    assert (ix[:, 3:] == -1).all() and torch.isinf(sc[:, 3:]).all()
    assert sorted(ix[0, :3].tolist()) == [0, 1, 2]


def test_merge_of_splits_keeps_lexicographic_order():
    idx = torch.tensor([[[5, 9, -1]], [[2, 7, 8]]], dtype=torch.int32)
    sc = torch.tensor([[[3.0, 1.0, -float("inf")]], [[3.0, 2.0, 1.0]]])
    mi, ms = _merge(idx, sc, 3)
    assert mi.tolist() == [[2, 5, 7]] and ms.tolist() == [[3.0, 3.0, 2.0]]


def test_recommend_topk_uses_fused_contract_cpu():
    from hivemall_amd.models.mf import BPRMF
    from hivemall_amd.io.synthetic import movielens_like

    us, its = movielens_like(20000, 200, 300, k=8)
    m = BPRMF("-factors 8 -iters 2", device="cpu").fit_implicit(us, its, 200, 300)
    sc, ix = m.recommend_topk([0, 1, 2], k=7, exclude=([0, 0], [int(ix0) for ix0 in (3, 4)]))
    S = m.scores([0, 1, 2]).double()
    S[0, 3] = S[0, 4] = -float("inf")
    want = torch.topk(S, 7, dim=1)
    np.testing.assert_allclose(sc.numpy(), want.values.numpy(), rtol=1e-5, atol=1e-5)
    assert 3 not in ix[0].tolist() and 4 not in ix[0].tolist()


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("d", [10, 64, 100, 256])
@pytest.mark.parametrize("k", [1, 10, 64])
def test_gpu_exact_integer_operands(d, k):
    Q, I = _int_data(150, 1000, d, d * 100 + k)
    bias = torch.randint(-2, 3, (1000,)).float()
    dev = torch.device("cuda")
    for splits in (1, 4):
        ix, sc = mips_topk(Q.to(dev), I.to(dev), k, item_bias=bias.to(dev), splits=splits)
        torch.cuda.synchronize()
        _check_exact(ix.cpu(), sc.cpu(), _ref(Q, I, k, bias), k)


@pytest.mark.gpu
def test_gpu_exclusions_self_and_ragged_shapes():
    dev = torch.device("cuda")
    Q, I = _int_data(131, 517, 40, 7)
    rows = torch.randint(0, 131, (3000,))
    items = torch.randint(0, 517, (3000,))
    ex = exclusion_csr(rows, items, 131)
    ix, sc = mips_topk(Q.to(dev), I.to(dev), 33, exclude=tuple(t.to(dev) for t in ex), exclude_self_offset=2)
    _check_exact(ix.cpu(), sc.cpu(), _ref(Q, I, 33, None, ex, 2), 33)
    # fewer admissible items than k
    ix, sc = mips_topk(Q[:5].to(dev), I[:20].to(dev), 40)
    assert (ix[:, 20:] == -1).all().item() and (ix[:, :20] >= 0).all().item()


@pytest.mark.gpu
def test_gpu_random_operands_match_fp64_reference():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    Q = torch.randn(700, 64, generator=g).bfloat16().float()
    I = torch.randn(5000, 64, generator=g).bfloat16().float()
    bias = torch.randn(5000, generator=g) * 0.1
    ix, sc = mips_topk(Q.to(dev), I.to(dev), 20, item_bias=bias.to(dev))
    S = _ref(Q, I, 20, bias)
    want = torch.topk(S, 20, dim=1).values
    np.testing.assert_allclose(sc.cpu().double().numpy(), want.numpy(), rtol=0, atol=2e-4)
    got = S.gather(1, ix.cpu())
    np.testing.assert_allclose(got.numpy(), sc.cpu().double().numpy(), rtol=0, atol=2e-4)
    for q in range(0, 700, 37):
        assert len(set(ix[q].tolist())) == 20


@pytest.mark.gpu
def test_gpu_recommend_topk_and_topk_similar():
    from hivemall_amd.knn import topk_similar
    from hivemall_amd.models.mf import BPRMF
    from hivemall_amd.io.synthetic import movielens_like

    dev = torch.device("cuda")
    X = torch.randn(300, 24, device=dev)
    sc, ix = topk_similar(X, k=5)
    Xn = torch.nn.functional.normalize(X.double(), dim=1)
    S = Xn @ Xn.T
    S.fill_diagonal_(-float("inf"))
    np.testing.assert_allclose(sc.double().cpu().numpy(), torch.topk(S, 5, dim=1).values.cpu().numpy(), atol=2e-2)
    assert not (ix == torch.arange(300, device=dev)[:, None]).any().item()
    us, its = movielens_like(50000, 500, 800, k=8)
    m = BPRMF("-factors 16 -iters 2", device=dev).fit_implicit(us.to(dev), its.to(dev), 500, 800)
    sc, ix = m.recommend_topk(None, k=10)
    S = m.scores().double()
    np.testing.assert_allclose(sc.double().cpu().numpy(), torch.topk(S, 10, dim=1).values.cpu().numpy(),
                               atol=5e-2)
