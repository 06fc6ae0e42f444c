"""Low-precision replicas: the shard-mean collective sums bf16 replicas in fp32 (one rounding),
and touched-row mixing of a bf16 replica stays sparse (base tracks the stored value)."""
import pytest
import torch

from tests.test_dist import run_world


def _bf16_mean(ctx):
    from hivemall_amd.parallel.mix import ModelMixer, OverlappedMixer

    g = torch.Generator().manual_seed(7 + ctx.rank)
    x = (1.0 + torch.rand(4099, generator=g) * 1e-2).to(torch.bfloat16)   # odd length: padding
    w = torch.randn(37, generator=g)
    VG = torch.randn(33, 5, 2, 4, generator=g).to(torch.bfloat16)          # packed V|G view
    before = [x.float().clone(), w.clone(), VG[:, :, 0].float().clone(), VG[:, :, 1].clone()]
    m = ModelMixer(ctx)
    m.average([x, w, VG[:, :, 0, :]])
    # overlapped: local progress is kept, the consensus correction is applied
    y = torch.full((64,), float(ctx.rank), dtype=torch.bfloat16)
    ov = OverlappedMixer(m)
    ov.start([y])
    y += 4.0
    ov.finish()
    return {"before": before, "x": x.float(), "w": w, "V": VG[:, :, 0].float(),
            "G": VG[:, :, 1].clone(), "y": y.float(), "wire": m.wire_bytes}


def test_shard_mean_bf16_is_fp32_accumulated():
    world = 3
    out = run_world("tests.test_mix_lowp:_bf16_mean", world=world)
    for key, k in (("x", 0), ("w", 1), ("V", 2)):
        ref = sum(out[r]["before"][k].double() for r in range(world)) / world
        dt = torch.float32 if key == "w" else torch.bfloat16
        expect = ref.to(torch.float32).to(dt).float()
        for r in range(world):
            got = out[r][key]
            # fp32 sum rounded once: within one bf16 rounding of the exact mean, identical ranks
            assert torch.equal(got, out[0][key])
            if dt == torch.bfloat16:
                assert (got - expect).abs().max() <= 2 ** -7 * expect.abs().max()
            else:
                torch.testing.assert_close(got, expect, rtol=1e-6, atol=1e-6)
    for r in range(world):
        assert torch.equal(out[r]["G"], out[r]["before"][3])        # optimizer state stays local
        # y_r = r + 4 + (mean(0,1,2) - r) = 5
        assert torch.equal(out[r]["y"], torch.full((64,), 5.0))
        assert out[r]["wire"] > 0


def _sparse_bf16(ctx):
    from hivemall_amd.parallel.mix import ModelMixer, SparseDeltaMixer

    g = torch.Generator().manual_seed(3 + ctx.rank)
    V = torch.randn(2048, 4, generator=g).to(torch.bfloat16)
    sm = SparseDeltaMixer(ModelMixer(ctx))
    sm.mix([V])
    rows = []
    for s in range(4):
        gs = torch.Generator().manual_seed(100 * s + ctx.rank)
        r = torch.randint(0, 2048, (16,), generator=gs)
        V[r] += torch.randn(16, 4, generator=gs).to(torch.bfloat16)
        before = sm.sparse_rows
        sm.mix([V])
        rows.append(sm.sparse_rows - before)
    return {"rows": rows, "dense": sm.dense_mixes, "V": V.float()}


def test_sparse_mixer_bf16_touched_rows_stay_bounded():
    out = run_world("tests.test_mix_lowp:_sparse_bf16", world=2)
    for r in (0, 1):
        # each rank touches <= 16 rows per step: the per-mix count must not grow with history
        assert all(n <= 32 for n in out[r]["rows"]), out[r]["rows"]
        assert out[r]["dense"] == 1
    assert torch.equal(out[0]["V"], out[1]["V"])


@pytest.mark.gpu
def test_mix_kernels_match_torch():
    from hivemall_amd import _native
    from hivemall_amd.parallel.mix import _row_view

    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    for dt, code in ((torch.float32, 0), (torch.bfloat16, 1)):
        world, n = 5, 4096 + 12
        recv = torch.randn(world * n, generator=g).to(dt).to(dev)
        mean = torch.empty(n, dtype=dt, device=dev)
        rc = _native.hip().hm_mix_shard_mean(recv.data_ptr(), world, n, code, mean.data_ptr(),
                                             _native.stream_of(dev))
        assert rc == 0
        acc = torch.zeros(n, dtype=torch.float32, device=dev)
        for r in range(world):            # the kernel's order: rank 0..N-1, fp32, one rounding
            acc += recv.view(world, n)[r].float()
        ref = (acc * torch.tensor(1.0 / world, dtype=torch.float32)).to(dt)
        assert torch.equal(mean, ref)
        VG = torch.randn(300, 7, 2, 4, generator=g).to(dt).to(dev)
        V = VG[:, :, 0, :]
        m = torch.randn(V.shape, generator=g).to(dt).to(dev)
        s = torch.randn(V.shape, generator=g).to(dt).to(dev)
        G0 = VG[:, :, 1].clone()
        ref = (V.float() + (m.float() - s.float())).to(dt)
        rows, inner, rs = _row_view(V)
        rc = _native.hip().hm_mix_merge(V.data_ptr(), m.data_ptr(), s.data_ptr(), rows, inner, rs,
                                        code, _native.stream_of(dev))
        assert rc == 0
        torch.cuda.synchronize()
        assert torch.equal(V, ref)
        assert torch.equal(VG[:, :, 1], G0)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["slot12_bf16", "block_fp32", "contiguous_bf16"])
def test_mix_view3_pack_merge_match_torch(layout):
    """hm_mix_pack3 / hm_mix_merge3 over the V part of the per-slot FFM feature blocks (12-B
    bf16 slots: 4-B aligned quads; fp32 896-B blocks) against torch; the fused merge+pack
    leaves the snapshot bit-identical to the merged replica, and the G words are untouched."""
    from hivemall_amd import _native
    from hivemall_amd.parallel.mix import _FlatGroup, _view3

    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1)
    nf, S = 1000, 40
    if layout == "slot12_bf16":
        dt, code = torch.bfloat16, 1
        blk = torch.randn(nf, 256, generator=g).to(dt).to(dev)          # 512-B blocks
        V = blk[:, :S * 6].view(nf, S, 6)[:, :, :4]                      # 12-B slots, V = 8 B
        other = lambda: blk[:, :S * 6].view(nf, S, 6)[:, :, 4:].clone()  # noqa: E731  (G words)
    elif layout == "block_fp32":
        dt, code = torch.float32, 0
        blk = torch.randn(nf, 224, generator=g).to(dev)                 # 896-B blocks
        V = blk[:, :S * 4].view(nf, S, 4)
        other = lambda: blk[:, S * 4:].clone()                           # noqa: E731
    else:
        dt, code = torch.bfloat16, 1
        V = torch.randn(nf, S, 4, generator=g).to(dt).to(dev)
        other = lambda: torch.zeros(1)                                   # noqa: E731
    v3 = _view3(V)
    assert v3 is not None
    st = _native.stream_of(dev)
    out = torch.empty(V.numel(), dtype=dt, device=dev)
    assert _native.hip().hm_mix_pack3(V.data_ptr(), out.data_ptr(), *v3, code, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(out.view(V.shape), V.contiguous())
    keep = other()
    m = torch.randn(V.shape, generator=g).to(dt).to(dev)
    snap = V.contiguous().clone()
    snap.view(-1)[::3] += 0.5
    ref = (V.float() + (m.float() - snap.float())).to(dt)
    assert _native.hip().hm_mix_merge3(V.data_ptr(), m.data_ptr(), snap.data_ptr(), snap.data_ptr(),
                                       *v3, code, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(V, ref)
    assert torch.equal(snap.view(V.shape), V)                            # fused next snapshot
    assert torch.equal(other(), keep)
    # the _FlatGroup path (pack -> merge(repack) -> pack is skipped)
    fg = _FlatGroup([V], 8)
    fg.pack()
    assert torch.equal(fg.seg(fg.send, 0), V)
    fg.out.copy_(fg.send)
    fg.seg(fg.out, 0).add_(1.0)
    before = V.float().clone()
    fg.merge(repack=True)
    assert fg.prepacked and torch.equal(V, (before + 1.0).to(dt))
    fg.pack()
    assert not fg.prepacked and torch.equal(fg.seg(fg.send, 0), V)
