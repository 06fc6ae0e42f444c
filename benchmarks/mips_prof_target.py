"""Profiling target: the fused MIPS top-k kernel alone on the ML-20M all-users shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.ops.topk_mips import mips_topk  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
U = (torch.randn(138493, 64, device=dev, generator=g) * 0.3).bfloat16()
V = (torch.randn(27278, 64, device=dev, generator=g) * 0.3).bfloat16()
b = torch.randn(27278, device=dev, generator=g) * 0.05
k = int(os.environ.get("MIPS_K", "10"))
for _ in range(3):
    mips_topk(U, V, k, item_bias=b)
torch.cuda.synchronize()
a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(5):
    mips_topk(U, V, k, item_bias=b)
e.record()
torch.cuda.synchronize()
print("k", k, "ms", round(a.elapsed_time(e) / 5, 3), flush=True)
