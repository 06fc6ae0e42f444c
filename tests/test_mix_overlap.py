"""OverlappedMixer: stale-by-one mixing merges the consensus correction with local progress."""
import torch

from tests.test_dist import run_world


def _overlap(ctx):
    from hivemall_amd.parallel.mix import ModelMixer, OverlappedMixer

    x = torch.full((1000,), float(ctx.rank + 1))           # ranks: 1, 2 -> mean 1.5
    xb = torch.full((10,), float(ctx.rank + 1)).to(torch.bfloat16)
    ov = OverlappedMixer(ModelMixer(ctx, bucket_mb=0.001))
    ov.start([x, xb])
    x += 10.0                                               # local progress while mixing
    xb += 10.0
    ov.finish()
    return [float(x[0]), float(x[-1]), float(xb[0])]


def test_overlapped_mixer_semantics():
    out = run_world("tests.test_mix_overlap:_overlap")
    # rank r: (r+1) + 10 + (1.5 - (r+1)) = 11.5 on every rank
    for r in (0, 1):
        assert out[r] == [11.5, 11.5, 11.5]


def _overlap_entry(ctx):
    return _overlap(ctx)
