"""SparseDeltaMixer: touched-row (index, Δ) all-gather equals the dense replica average."""
import torch

from tests.test_dist import run_world


def _sparse(ctx):
    from hivemall_amd.parallel.mix import ModelMixer, SparseDeltaMixer

    g = torch.Generator().manual_seed(100 + ctx.rank)
    w = torch.randn(4096, generator=g)                     # replicas differ at start
    V = torch.randn(4096, 3, 4, generator=g)
    sm = SparseDeltaMixer(ModelMixer(ctx))
    sm.mix([w, V])                                         # first mix: dense average
    out = {"first": [float(w.sum()), float(V.sum())], "dense_mixes": sm.dense_mixes}
    steps = []
    for s in range(3):
        gs = torch.Generator().manual_seed(1000 * s + ctx.rank)
        rows = torch.randint(0, 4096, (50,), generator=gs)  # overlapping touched sets
        before_w, before_V = w.clone(), V.clone()
        w[rows] += torch.randn(50, generator=gs)
        V[rows[:20]] += torch.randn(20, 3, 4, generator=gs)
        # what the dense average would be (computed with a plain all-reduce of copies)
        dw, dV = w.clone(), V.clone()
        ModelMixer(ctx).average([dw, dV])
        sm.mix([w, V])
        steps.append([float((w - dw).abs().max()), float((V - dV).abs().max()),
                      float((w - before_w).abs().max() > 0)])
    out["steps"] = steps
    out["sparse_rows"] = sm.sparse_rows
    out["dense_after"] = sm.dense_mixes
    # touching everything falls back to the dense path on every rank
    w += 1.0 + ctx.rank
    dw = w.clone()
    ModelMixer(ctx).average([dw])
    sm.mix([w, V])
    out["fallback"] = [sm.dense_mixes, float((w - dw).abs().max())]
    return out


def test_sparse_delta_mixer_equals_dense_average():
    for world in (2, 3):
        out = run_world("tests.test_mix_sparse:_sparse", world=world)
        for r in range(world):
            o = out[r]
            assert o["dense_mixes"] == 1
            for ew, eV, _ in o["steps"]:
                assert ew < 1e-5 and eV < 1e-5
            assert o["sparse_rows"] > 0 and o["dense_after"] == 1
            assert o["fallback"][0] == 2 and o["fallback"][1] < 1e-5
        # every rank holds the same mixed model
        assert all(out[r]["first"] == out[0]["first"] for r in range(world))


def test_sparse_delta_mixer_noop_without_world():
    from hivemall_amd.parallel.dist import DistContext
    from hivemall_amd.parallel.mix import ModelMixer, SparseDeltaMixer

    w = torch.arange(5.0)
    m = SparseDeltaMixer(ModelMixer(DistContext()))
    m.mix([w])
    assert torch.equal(w, torch.arange(5.0))
