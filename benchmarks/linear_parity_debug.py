"""Debug: the 2^24 parity test's setup next to linear_rules_parity.py's, same process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models import linear as L

    def rows(n, seed):
        idx, y = criteo_like(n, hash_bits=24, seed=seed)
        return L.SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64), idx.reshape(-1).contiguous(),
                            None, y.contiguous())

    tr = rows(200000, 5)
    tests = {"t50k": rows(50000, 99), "t100k": rows(100000, 99)}
    for opts in sys.argv[1:] or ["-opt sgd -eta0 0.05", "-opt adagrad -reg no"]:
        res = {}
        for dev in ("cpu", "cuda"):
            for rep in range(2 if dev == "cuda" else 1):
                m = L.TrainClassifier(f"-loss logloss {opts} -dims 16777216", device=dev)
                m.fit(rows=tr.to(dev))
                for k, t in tests.items():
                    s = m.decision_function(rows=t.to(dev)).cpu()
                    res[f"{dev}{rep}_{k}"] = round(torch.nn.functional.binary_cross_entropy_with_logits(
                        s, (t.y > 0).float()).item(), 5)
                if dev == "cuda":
                    res[f"waves{rep}"] = int(m.state.RS.shape[0])
        print(json.dumps({"opts": opts, **res}), flush=True)


if __name__ == "__main__":
    main()
