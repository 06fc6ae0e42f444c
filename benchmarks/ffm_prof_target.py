"""Small fixed FFM workload for rocprofv3 counter runs: 6 train steps of 262,144 rows at the
driver's headline config by default — ``criteo_ffm`` rows (explicit fields and values: the fld /
val DMAs), fp32 V + per-slot fp32 G (``ffm_pipe_sg32_kernel``).  BF16=1 selects bf16 state
(``ffm_pipe_sg12_kernel``), DATA=criteo_like the round-1..3 implicit-field rows, HM_FFM_VARIANT a
kernel variant (csrc/kernels/ffm.hip hm_ffm_step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_ffm, criteo_like  # noqa: E402
from hivemall_amd.models.ffm import FFMTrainer  # noqa: E402
from hivemall_amd.ops.ffm import ffm_step  # noqa: E402

dev = torch.device("cuda")
B = 262144
if os.environ.get("DATA", "criteo_ffm") == "criteo_ffm":
    idx, fld, val, y = criteo_ffm(B * 2, 20, seed=3, device=dev)
else:
    idx, y = criteo_like(B * 2, 20, seed=3, device=dev)
    fld = val = None
t = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 20" +
               (" -bf16_state" if os.environ.get("BF16") == "1" else ""), device=dev)
t.init_state(1 << 20, 39)
for i in range(6):
    s = (i % 2) * B
    ffm_step(t.state, idx[s:s + B], None if fld is None else fld[s:s + B],
             None if val is None else val[s:s + B], y[s:s + B], t.hyper,
             variant=int(os.environ.get("HM_FFM_VARIANT", "0")))
torch.cuda.synchronize()
print("done")
