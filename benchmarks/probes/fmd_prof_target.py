"""rocprofv3 --pmc target: one epoch of train_fm -engine minibatch on 2M HIGGS-shaped rows at
B = 65536 with the f32-MFMA gradient kernel (variant 0), then with the VALU kernel (variant 1),
so one counter pass covers fmd_mfma_kernel and fmd_grad_kernel (filter by kernel name).
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES ... -- python3 benchmarks/probes/fmd_prof_target.py
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
from hivemall_amd.io.synthetic import higgs_like  # noqa: E402
from hivemall_amd.models.fm_dense import DenseMinibatchFM  # noqa: E402

X, y = higgs_like(2_000_000, seed=5, device="cuda")
yy = torch.where(y > 0, 1.0, -1.0)
V0 = torch.randn(28, 8, generator=torch.Generator().manual_seed(3)) * 0.01
for variant in (0, 1):
    eng = DenseMinibatchFM(28, 8, V0, "cuda", 65536, 0.05, 0.01, 0.01, 0.01, True, -3.4e38, 3.4e38, variant=variant)
    for b in range(0, 2_000_000 - 65535, 65536):
        eng.step(X[b:b + 65536].contiguous(), yy[b:b + 65536].contiguous())
    torch.cuda.synchronize()
print("ok", flush=True)
