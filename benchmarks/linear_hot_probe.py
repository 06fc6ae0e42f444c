"""Shared-table linear engine with hot-feature pre-aggregation (csrc/kernels/linear.hip HOT):
held-out logloss vs the sequential CPU engine and rows/s, over chunk sizes CH and wave counts.
Criteo-shaped rows hashed into 2^24 dims, train_classifier -loss logloss -opt adagrad."""
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
EPOCHS = int(os.environ.get("EPOCHS", 1))


def rows(n, seed, dev):
    idx, y = criteo_like(n, BITS, seed=seed, device=dev)
    return L.SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64, device=dev),
                        idx.reshape(-1).contiguous(), None, y)


def heldout(m, te):
    s = m.decision_function(rows=te).float()
    return torch.nn.functional.binary_cross_entropy_with_logits(s, (te.y > 0).float()).item()


def main():
    tr_c, te_c = rows(N, 5, "cpu"), rows(NT, 77, "cpu")
    opts = f"-loss logloss -opt adagrad -dims {1 << BITS} -iters {EPOCHS}"
    m = L.TrainClassifier(opts, device="cpu")
    t0 = time.perf_counter()
    m.fit(rows=tr_c)
    seq = heldout(m, te_c)
    print(json.dumps({"engine": "cpu sequential", "rows": N, "epochs": EPOCHS,
                      "rows_per_s": round(N * EPOCHS / (time.perf_counter() - t0)),
                      "heldout_logloss": round(seq, 5)}), flush=True)
    tr, te = tr_c.to("cuda"), te_c.to("cuda")
    grid = [(0, 512, 16, 16, 4), (0, 512, 16, 16, 4)] + [(1, W, ch, mn, ev) for W, ch, mn, ev in ((1024, 16, 16, 4), (1024, 16, 16, 8), (1024, 16, 32, 8), (1024, 32, 32, 4), (1024, 32, 32, 8), (2048, 16, 16, 8), (2048, 16, 32, 16))]
    for hot, W, ch, mn, ev in grid:
        os.environ["HM_LINEAR_HOT"] = str(hot)
        os.environ["HM_LINEAR_HOT_CH"] = str(ch)
        os.environ["HM_LINEAR_HOT_MIN"] = str(mn)
        os.environ["HM_LINEAR_HOT_EVERY"] = str(ev)
        m = L.TrainClassifier(opts + " -engine shared", device="cuda")
        m._ensure_state(tr)
        m.state = LO.new_shared_state(1 << BITS, "cuda", N, waves=W)
        LO.train_pass_shared(m.state, m.P, tr.indptr, tr.idx, tr.val, tr.y, 0)     # warm (code load)
        m.state = LO.new_shared_state(1 << BITS, "cuda", N, waves=W)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hs = LO.hot_features(m.state, m.P, tr.idx, N)
        torch.cuda.synchronize()
        t_hot = time.perf_counter() - t0
        t0 = time.perf_counter()
        m.fit(rows=tr)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ll = heldout(m, te)
        print(json.dumps({"hot": hot, "waves": W, "chunk_rows_per_wave": ch, "min_rows": mn, "every": ev,
                          "hot_features": 0 if hs is None else int(hs[1].numel()),
                          "hot_select_ms": round(1e3 * t_hot, 2), "rows_per_s": round(N * EPOCHS / dt),
                          "heldout_logloss": round(ll, 5), "delta_vs_seq": round(ll - seq, 5)}), flush=True)


if __name__ == "__main__":
    main()
