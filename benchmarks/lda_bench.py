"""train_lda epoch time: fused E-step kernel (csrc/kernels/lda.hip) vs the torch formulation on
the same GPU (HM_LDA_TORCH=1).  Synthetic corpus: D docs of ~L words drawn from K planted topics
over a V-word vocabulary (20-Newsgroups-like scale)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hivemall_amd.models.topicmodel import LDA  # noqa: E402


def corpus(D=20000, V=20000, K=100, L=150, seed=0):
    rng = np.random.default_rng(seed)
    beta = rng.dirichlet(np.full(V, 0.05), size=K)
    words = [f"w{i}" for i in range(V)]
    docs = []
    for _ in range(D):
        th = rng.dirichlet(np.full(K, 0.1))
        z = rng.choice(K, size=L, p=th)
        cnt = np.bincount(z, minlength=K)
        toks = []
        for k in np.nonzero(cnt)[0]:
            toks += [words[i] for i in rng.choice(V, size=cnt[k], p=beta[k])]
        docs.append(toks)
    return docs


def main():
    D = int(os.environ.get("D", 4000))
    K = int(os.environ.get("K", 100))
    docs = corpus(D=D, K=K)
    for torch_path in (False, True):
        os.environ["HM_LDA_TORCH"] = "1" if torch_path else "0"
        m = LDA(f"-topics {K} -iters 1 -mini_batch_size 256", device="cuda")
        m.fit(docs[:256])                                      # warm-up (code load)
        m = LDA(f"-topics {K} -iters 5 -eps 0 -mini_batch_size 256", device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.fit(docs)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"estep": "torch" if torch_path else "kernel", "docs": D, "topics": K,
                          "fit_5_epochs_s": round(dt, 3), "docs_epochs_per_s": round(5 * D / dt),
                          "perplexity": round(float(m.perplexity or 0), 3)}), flush=True)


if __name__ == "__main__":
    main()
