import time, torch, sys
sys.path.insert(0, "/root/repo")
from hivemall_amd.io.synthetic import higgs_like
from hivemall_amd.models import trees as T
X, y = higgs_like(11_000_000, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter(); q = T.quantize(X, 256); torch.cuda.synchronize(); print("quantize", time.perf_counter() - t0)
t0 = time.perf_counter(); c, yi = T._encode_classes(y.long()); torch.cuda.synchronize(); print("encode", time.perf_counter() - t0)
st = torch.stack([y - 0.5, torch.full_like(y, 0.25), torch.ones_like(y)], 1).contiguous()
for i in range(3):
    t0 = time.perf_counter(); b = T.HistTreeBuilder(q, "gbt", 8, 5, 1, seed=i); tr = b.build(st); torch.cuda.synchronize(); print("tree", time.perf_counter() - t0, len(tr.feature))
