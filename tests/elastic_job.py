"""Job used by tests/test_elastic.py: 2-rank FFM data parallel training with per-step
checkpoints, RCCL/gloo mixing, fault injection (HM_FAULT) and resume."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMBatch, FFMTrainer  # noqa: E402
from hivemall_amd.parallel.dist import init_distributed, shutdown  # noqa: E402
from hivemall_amd.parallel.elastic import ResumableLoop  # noqa: E402
from hivemall_amd.parallel.mix import ModelMixer  # noqa: E402

ctx = init_distributed(backend="gloo", device="cpu", timeout_s=20)
ckpt = os.environ["HM_CKPT"]
steps = int(os.environ.get("HM_STEPS", "6"))
mixer = ModelMixer(ctx)
idx, y = criteo_like(steps * 400, 10, seed=50 + ctx.rank)
tr = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 10 -seed 3", device="cpu", mixer=mixer,
                rank=ctx.rank)
tr.init_state(1 << 10, 39)


def step(learner, s):
    b = FFMBatch(idx[s * 400:(s + 1) * 400], None, None, y[s * 400:(s + 1) * 400])
    learner.train_batch(b)
    learner.mix()


loop = ResumableLoop(tr, ckpt, every=1, ctx=ctx)
tr = loop.run(steps, step)
torch.save(tr.state["V"].clone(), os.path.join(ckpt, f"final_rank{ctx.rank}.pt"))
shutdown()
