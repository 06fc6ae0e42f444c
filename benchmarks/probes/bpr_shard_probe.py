"""Probe: BPR on small explicit triples, unsharded vs -shard_model, CPU vs GPU (AUC)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_sharded import _auc, _triples  # noqa: E402
from hivemall_amd.models.mf import BPRMF  # noqa: E402

u, i, j = _triples(n=40000)
for dev in ("cpu", "cuda"):
    for extra in ("", " -shard_model -shard_batch 8192", " -shard_model -shard_batch 100000", " -grid 1"):
        m = BPRMF("-factors 8 -iters 5 -eta0 0.05 -disable_cv -seed 5" + extra, device=dev).fit(u, i, j)
        st = m.state
        print(dev, extra, round(_auc(st["P"].cpu().numpy(), st["Q"].cpu().numpy(), st["Bi"].cpu().numpy()), 4),
              "grid", m._grid(), flush=True)
