"""The mixing collectives through RCCL itself.  The pool gives one GPU per box and RCCL refuses
two ranks on one card, so this drives the real RCCL calls (all_to_all_single,
all_gather_into_tensor, all_reduce) in a ONE-rank nccl process group, on the FFM bench's own
state layout (bf16 V in 12-B slots + fp32 FTRL state): a one-replica mean is the identity, so
every mix must leave the model bit-exact, and the overlapped mix must keep the progress made
while its collectives were in flight."""
import os
import socket

import pytest
import torch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_shard_mean_collectives_through_rccl_one_rank():
    import torch.distributed as dist

    from hivemall_amd.models.ffm import FFMTrainer
    from hivemall_amd.ops.ffm import linear_mix_tensors
    from hivemall_amd.parallel.dist import DistContext
    from hivemall_amd.parallel.mix import ModelMixer, OverlappedMixer

    assert not dist.is_initialized()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        ctx = DistContext(0, 1, 0, dev, "nccl")
        tr = FFMTrainer("-classification -factors 4 -num_fields 39 -feature_hashing 14 -bf16_state -seed 3",
                        device=dev)
        tr.init_state(1 << 14, 39)
        st = tr.state
        g = torch.Generator(device="cuda").manual_seed(0)
        st["V"].copy_(torch.randn(st["V"].shape, generator=g, device=dev).to(torch.bfloat16))
        for k in ("wz", "wn", "w"):
            st[k].copy_(torch.randn(st[k].shape, generator=g, device=dev))
        tensors = [st["V"], *linear_mix_tensors(st), st["bias"]]
        if "wz" in st and st["w"].stride(0) > 1:             # the {w, z, n} records: one row view
            assert len(tensors) == 3 and tensors[1].shape == (1 << 14, 4)
        ref = [t.clone() for t in tensors]
        ref_w = st["w"].clone()
        m = ModelMixer(ctx, min_world=1)
        m.average(tensors)                                   # all_to_all + shard mean + all_gather
        torch.cuda.synchronize()
        for t, r in zip(tensors, ref):
            assert torch.equal(t, r)
        ov = OverlappedMixer(m)
        ov.start(tensors)                                    # collectives on the side stream
        st["w"].add_(1.0)                                    # progress while they are in flight
        st["V"].add_(torch.ones_like(st["V"]))
        ov.start(tensors)                                    # finishes mix 1 (fused merge + repack)
        ov.finish()
        torch.cuda.synchronize()
        assert torch.equal(st["w"], ref_w + 1.0)
        assert torch.equal(st["V"], (ref[0].float() + 1.0).to(torch.bfloat16))
        x = torch.arange(10, dtype=torch.float32, device=dev)
        m.all_reduce_sum([x])
        assert torch.equal(x, torch.arange(10, dtype=torch.float32, device=dev))
        assert m.all_reduce_scalar(2.5, "max") == 2.5
        pr = m.probe(tensors, reps=2)
        assert pr["mix_ms"] > 0 and pr["mix_payload_bytes"] > 0
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_fused_delta_mixing_bit_identical_to_torch_path():
    """average_delta (bf16 wire, fp32 replicas) and the overlapped delta-sum merge run as fused
    HIP passes over the strided V view of the fp32 FFM feature blocks (hm_mix_delta3); through a
    one-rank nccl group they must produce exactly the torch formulation's bits."""
    import torch.distributed as dist

    from hivemall_amd.models.ffm import FFMTrainer
    from hivemall_amd.ops.ffm import linear_mix_tensors
    from hivemall_amd.parallel import mix as M
    from hivemall_amd.parallel.dist import DistContext

    assert not dist.is_initialized()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    old = M._FUSED_DELTA
    try:
        ctx = DistContext(0, 1, 0, dev, "nccl")
        res = {}
        for fused in (False, True):
            M._FUSED_DELTA = fused
            tr = FFMTrainer("-classification -factors 4 -num_fields 39 -feature_hashing 14 -seed 3", device=dev)
            tr.init_state(1 << 14, 39)
            st = tr.state
            assert M._view3(st["V"]) is not None and not st["V"].is_contiguous()
            g = torch.Generator(device="cuda").manual_seed(1)
            for k in ("wz", "wn", "w"):
                st[k].copy_(torch.randn(st[k].shape, generator=g, device=dev))
            tensors = [st["V"], *linear_mix_tensors(st), st["bias"]]
            assert all(M._view3(t) is not None for t in tensors[:2])   # both on the fused path
            m = M.ModelMixer(ctx, min_world=1)
            for step in range(3):                      # seed the consensus, then two delta mixes
                for t in tensors:
                    t.add_(torch.randn(t.shape, generator=g, device=dev) * 1e-3)
                m.average_delta(tensors)
            ov = M.OverlappedMixer(m, mode="sum")
            for step in range(3):                      # first mix seeds base, then delta-sum mixes
                ov.start(tensors)
                for t in tensors:
                    t.add_(torch.randn(t.shape, generator=g, device=dev) * 1e-3)
            ov.finish()
            torch.cuda.synchronize()
            res[fused] = [t.clone() for t in tensors]
            del tr, st, tensors, m, ov
        for a, b in zip(res[False], res[True]):
            assert torch.equal(a, b)
    finally:
        M._FUSED_DELTA = old
        dist.destroy_process_group()


@pytest.mark.gpu
def test_pipelined_buckets_bit_identical_through_rccl_one_rank():
    """The bucketed, pipelined shard mean (ModelMixer._pipelined: per-bucket fused pack of the
    tensor row ranges, all_to_all on the RCCL stream, shard mean, all_gather, fused merge of the
    rows whose means have all arrived) leaves exactly the bits of the monolithic path, for
    average_delta on fp32 replicas and average on bf16 ones, on the FFM feature-block views."""
    import torch.distributed as dist

    from hivemall_amd.models.ffm import FFMTrainer
    from hivemall_amd.ops.ffm import linear_mix_tensors
    from hivemall_amd.parallel import mix as M
    from hivemall_amd.parallel.dist import DistContext

    assert not dist.is_initialized()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        ctx = DistContext(0, 1, 0, dev, "nccl")
        for bf16 in (False, True):
            res = {}
            for mb in (0.0, 0.37):
                tr = FFMTrainer("-classification -factors 4 -num_fields 39 -feature_hashing 14 -seed 3"
                                + (" -bf16_state" if bf16 else ""), device=dev)
                tr.init_state(1 << 14, 39)
                st = tr.state
                g = torch.Generator(device="cuda").manual_seed(5)
                tensors = [st["V"], *linear_mix_tensors(st), st["bias"]]
                m = M.ModelMixer(ctx, min_world=1)
                m.PIPE_BUCKET_MB = mb
                fn = m.average if bf16 else m.average_delta
                for step in range(3):
                    for t in tensors:
                        t.add_((torch.randn(t.shape, generator=g, device=dev) * 1e-3).to(t.dtype))
                    fn(tensors)
                if mb:
                    grp = next(iter(m._plans.values()))[0]
                    assert len(grp.buckets(int(mb * (1 << 20)) // grp.send.element_size())) >= 4
                torch.cuda.synchronize()
                res[mb] = [t.clone() for t in tensors]
                del tr, st, tensors, m
            for a, b in zip(res[0.0], res[0.37]):
                assert torch.equal(a, b)
    finally:
        dist.destroy_process_group()
