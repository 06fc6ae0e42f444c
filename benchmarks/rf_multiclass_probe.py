"""GPU vs CPU RandomForest accuracy on the 5..8-class wide-row shape of
tests/test_trees.py::test_rf_5_to_8_classes_wide_rows_gpu_matches_cpu, over seeds and forest sizes:
is a GPU/CPU accuracy difference of a 4-tree forest seed noise or an engine difference?

    python benchmarks/rf_multiclass_probe.py [n_classes] [trees...]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.models.trees import RandomForestClassifier  # noqa: E402


def main():
    nc = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    sizes = [int(t) for t in sys.argv[2:]] or [4, 32]
    rng = np.random.default_rng(5)
    X = rng.normal(size=(12000, 20)).astype(np.float32)
    y = (np.floor((X[:, 3] + 3) * nc / 6).clip(0, nc - 1)).astype(int)
    Xt = rng.normal(size=(4000, 20)).astype(np.float32)
    yt = (np.floor((Xt[:, 3] + 3) * nc / 6).clip(0, nc - 1)).astype(int)
    for T in sizes:
        for dev in ("cpu", "cuda"):
            accs, held = [], []
            for seed in range(1, 9):
                rf = RandomForestClassifier(f"-trees {T} -max_depth 8 -seed {seed}", device=dev).fit(X, y)
                accs.append(float((rf.predict(X) == y).mean()))
                held.append(float((rf.predict(Xt) == yt).mean()))
            print(json.dumps({"classes": nc, "trees": T, "device": dev, "train_acc_mean": round(np.mean(accs), 4),
                              "train_acc_min": round(min(accs), 4), "heldout_acc_mean": round(np.mean(held), 4),
                              "train_acc": [round(a, 4) for a in accs]}), flush=True)


if __name__ == "__main__":
    main()
