"""Shared-table linear engine sweep: XCD-local replicas x waves x reload
on Criteo-shaped rows hashed into 2^24 dims, train_classifier -loss logloss -opt adagrad, one
epoch; rows/s and held-out logloss against the sequential CPU engine on the same rows."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.io.synthetic import criteo_like  # noqa: E402
from hivemall_amd.models import linear as L  # noqa: E402
from hivemall_amd.ops import linear as LO  # noqa: E402

N, BITS, NT = int(os.environ.get("N", 2 * 1024 * 1024)), 24, 200000


def rows(n, seed, dev):
    idx, y = criteo_like(n, BITS, seed=seed, device=dev)
    return L.SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64, device=dev),
                        idx.reshape(-1).contiguous(), None, y)


def heldout(m, te):
    s = m.decision_function(rows=te).float()
    return torch.nn.functional.binary_cross_entropy_with_logits(s, (te.y > 0).float()).item()


def main():
    tr_c, te_c = rows(N, 5, "cpu"), rows(NT, 77, "cpu")
    if "--cpu" in sys.argv:
        m = L.TrainClassifier(f"-loss logloss -opt adagrad -dims {1 << BITS}", device="cpu")
        t0 = time.perf_counter()
        m.fit(rows=tr_c)
        dt = time.perf_counter() - t0
        print(json.dumps({"engine": "cpu sequential", "rows": N, "rows_per_s": round(N / dt),
                          "heldout_logloss": round(heldout(m, te_c), 5)}), flush=True)
    tr, te = tr_c.to("cuda"), te_c.to("cuda")
    grid = [(R, W, rl, nt) for nt in (True, False) for R in (1, 8, 32) for W in (8192, 2048, 512)
            for rl in (False, True) if (W + 3) // 4 >= R and not (not nt and W == 512)]
    for R, W, reload, nt in grid:
        m = L.TrainClassifier(f"-loss logloss -opt adagrad -dims {1 << BITS} -engine shared", device="cuda")
        m._ensure_state(tr)
        m.state = LO.new_shared_state(1 << BITS, "cuda", N, waves=W, replicas=R, reload=reload, nt=nt)
        LO.train_pass_shared(m.state, m.P, tr.indptr, tr.idx, tr.val, tr.y, 0)     # warm (code load)
        m.state = LO.new_shared_state(1 << BITS, "cuda", N, waves=W, replicas=R, reload=reload, nt=nt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.fit(rows=tr)                      # one pass + the replica mix
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"engine": "shared", "replicas": R, "waves": W, "reload": reload, "nt": nt, "rows": N,
                          "rows_per_s": round(N / dt), "heldout_logloss": round(heldout(m, te), 5)}),
              flush=True)
        del m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
