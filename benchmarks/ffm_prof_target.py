"""Small fixed FFM workload for rocprofv3 counter runs: 6 train steps of 262144 Criteo-shaped
rows (bf16 state unless FP32=1)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

dev = torch.device("cuda")
B = 262144
idx, y = criteo_like(B * 2, 20, seed=3, device=dev)
t = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 20" +
               ("" if os.environ.get("FP32") == "1" else " -bf16_state"), device=dev)
t.init_state(1 << 20, 39)
for i in range(6):
    s = (i % 2) * B
    ffm_step(t.state, idx[s:s + B], None, None, y[s:s + B], t.hyper)
torch.cuda.synchronize()
print("done")
