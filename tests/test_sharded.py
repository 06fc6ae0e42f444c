"""Row-sharded model tables (parallel/sharded.py, SURVEY.md §2.4 sharded parameter server):
pull/push against a dense reference, and model-parallel BPR-MF (-shard_model) on gloo world 2/3
against the single-process learner."""
import numpy as np
import pytest
import torch

from tests.test_dist import run_world


def _table_ops(ctx):
    from hivemall_amd.parallel.sharded import ShardedTable

    n, dim = 1001, 3
    ref = torch.arange(n * dim, dtype=torch.float32).reshape(n, dim)
    t = ShardedTable(n, dim, ctx, init=lambda gid: ref[gid])
    assert t.local.shape[0] == len(range(ctx.rank, n, ctx.world_size))        # 1/world of the rows
    g = torch.Generator().manual_seed(ctx.rank)
    ids = torch.unique(torch.randint(0, n, (200,), generator=g))
    ok_pull = bool(torch.equal(t.pull(ids), ref[ids]))
    # every rank adds +1 to rows [0, 50) and (rank+1) to its random ids: the owner sees all adds
    t.push_add(torch.arange(50), torch.ones(50, dim))
    t.push_add(ids, torch.full((ids.numel(), dim), float(ctx.rank + 1)))
    t.push_add(torch.zeros(0, dtype=torch.int64), torch.zeros(0, dim))            # empty batches are fine
    full = t.full()
    return ok_pull, full.numpy().tolist(), ids.tolist()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_table_pull_push_matches_dense(world):
    out = run_world("tests.test_sharded:_table_ops", world)
    n, dim = 1001, 3
    exp = torch.arange(n * dim, dtype=torch.float32).reshape(n, dim)
    exp[:50] += world
    for r in range(world):
        exp[torch.tensor(out[r][2])] += r + 1
    for r in range(world):
        assert out[r][0]
        np.testing.assert_array_equal(np.array(out[r][1]), exp.numpy())


def _triples(seed=0, n=60000, users=400, items=300):
    pref = np.random.default_rng(123).integers(0, 3, size=users)    # 3 taste groups (fixed)
    rng = np.random.default_rng(seed)
    u = rng.integers(0, users, size=n)
    i = (pref[u] * 100 + rng.integers(0, 100, size=n)) % items
    j = rng.integers(0, items, size=n)
    keep = (j // 100) != pref[u]
    return u[keep], i[keep], j[keep]


def _auc(P, Q, Bi, seed=1):
    u, i, j = _triples(seed, 20000)
    s = lambda a, b: (P[a] * Q[b]).sum(1) + Bi[b]
    return float((s(u, i) > s(u, j)).mean())


def _bpr_sharded(ctx):
    from hivemall_amd.models.mf import BPRMF
    from hivemall_amd.parallel.mix import ModelMixer

    u, i, j = _triples()
    sl = slice(ctx.rank, None, ctx.world_size)
    m = BPRMF("-factors 8 -iters 8 -eta0 0.05 -disable_cv -seed 3 -shard_model -shard_batch 4096",
              device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
    m.fit(u[sl], i[sl], j[sl])
    rows_local = m.sharded["Q"].local.shape[0]
    st = m.state
    return rows_local, _auc(st["P"].numpy(), st["Q"].numpy(), st["Bi"].numpy()), st["Q"].numpy()[:5].tolist()


def test_bpr_shard_model_world2_matches_single_process_quality():
    from hivemall_amd.models.mf import BPRMF

    out = run_world("tests.test_sharded:_bpr_sharded", 2)
    u, i, j = _triples()
    ref = BPRMF("-factors 8 -iters 8 -eta0 0.05 -disable_cv -seed 3", device="cpu").fit(u, i, j)
    auc_ref = _auc(ref.state["P"].numpy(), ref.state["Q"].numpy(), ref.state["Bi"].numpy())
    assert out[0][0] + out[1][0] == 300 and max(out[0][0], out[1][0]) == 150      # each rank holds half of Q
    assert out[0][2] == out[1][2]                                                  # one model on both ranks
    assert out[0][1] > 0.85 and abs(out[0][1] - auc_ref) < 0.03, (out[0][1], auc_ref)


def test_bpr_shard_model_single_process_equals_unsharded():
    """World 1: pull/compute/push over the whole batch is the plain kernel on the full tables."""
    from hivemall_amd.models.mf import BPRMF

    u, i, j = _triples(n=20000)
    a = BPRMF("-factors 8 -iters 3 -disable_cv -seed 5 -shard_model -shard_batch 100000", device="cpu").fit(u, i, j)
    b = BPRMF("-factors 8 -iters 3 -disable_cv -seed 5", device="cpu").fit(u, i, j)
    np.testing.assert_allclose(a.state["P"].numpy(), b.state["P"].numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(a.state["Q"].numpy(), b.state["Q"].numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_bpr_shard_model_gpu_single_process():
    """Device tables through pull/compute/push.  -grid 1: on this 300-item catalogue wider
    Hogwild grids stall the factors on the near-zero init whether sharded or not (AUC 0.50 at
    the default grid 9 vs 1.00 at grid 1 for the plain learner too: benchmarks/probes/
    bpr_shard_probe.py, profiles/bpr_shard_probe_r2.log; docs/perf_notes.md MF staleness)."""
    from hivemall_amd.models.mf import BPRMF

    u, i, j = _triples(n=40000)
    a = BPRMF("-factors 8 -iters 5 -eta0 0.05 -disable_cv -seed 5 -shard_model -shard_batch 8192 -grid 1",
              device="cuda").fit(u, i, j)
    st = a.state
    assert _auc(st["P"].cpu().numpy(), st["Q"].cpu().numpy(), st["Bi"].cpu().numpy()) > 0.85
