"""Data-parallel quality of BPR-MF (BASELINE config 5) and train_fm (config 2) at N = 2/4/8 on ONE
device: N model replicas in HBM, each stepped by the real kernels on the
shard rank r of ``bench_configs.py --gpus N`` would train (every N-th interaction / row), the
replicas averaged at every mix point as ``ModelMixer.average`` does (plain mean of the mixed
tables, optimizer state local), with each replica's step size scaled by N^p.  The reference is
ONE replica over the same total rows.

    python benchmarks/dp_sim_mf_fm.py --worlds 2 4 8 --powers 0 0.5 0.75 [--what bpr fm]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _mean_into(models, keys):
    for k in keys:
        ts = [m.state[k] for m in models if k in m.state]
        if not ts:
            continue
        avg = torch.stack([t.float() for t in ts]).mean(0)
        for t in ts:
            t.copy_(avg.to(t.dtype))


def bpr(worlds, powers, epochs=3, k=64, eta0=0.05):
    from hivemall_amd.io.synthetic import movielens_like
    from hivemall_amd.models.mf import BPRMF, auc_implicit

    dev = torch.device("cuda")
    nu, ni = 138493, 27278
    us, its = movielens_like(device=dev, k=16)
    ntest = 200000
    tu, ti = us[:-ntest], its[:-ntest]
    eu, ei = us[-ntest:].cpu().numpy(), its[-ntest:].cpu().numpy()
    out = []
    for N in [1] + list(worlds):
        for p in ([0.0] if N == 1 else powers):
            eta = eta0 * N ** p
            models, csrs = [], []
            for r in range(N):
                m = BPRMF(f"-factors {k} -iters 1 -eta0 {eta} -disable_cv -seed 7", device=dev)
                m.init_state(nu, ni)
                su, si = tu[r::N].contiguous(), ti[r::N].contiguous()
                csrs.append(m.build_csr(su, si, nu))
                m.seen_u[su.long()] = True
                m.seen_i.fill_(True)
                models.append(m)
            for ep in range(epochs):
                for m, c in zip(models, csrs):
                    m.step(n=c[1].numel(), csr=c)
                if N > 1:
                    _mean_into(models, ("P", "Q", "Bu", "Bi"))
            auc = auc_implicit(models[0], eu, ei)
            rec = {"what": "bpr", "N": N, "power": p, "eta0": round(eta, 5), "epochs": epochs,
                   "sampled_auc": round(auc, 5)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
            del models, csrs
            torch.cuda.empty_cache()
    return out


def fm(worlds, powers, n_rows=8 * 262144, bits=24, epochs=2, eta0=0.01):
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.models.linear import SparseRows

    dev = torch.device("cuda")
    idx, y = criteo_like(n_rows, bits, seed=5, device=dev)
    eidx, ey = criteo_like(200000, bits, seed=77, device=dev)
    er = SparseRows(torch.arange(0, 200000 * 39 + 1, 39, dtype=torch.int64, device=dev),
                    eidx.reshape(-1).contiguous(), None, None)
    yy = (ey > 0).float()
    out = []
    for N in [1] + list(worlds):
        for p in ([0.0] if N == 1 else powers):
            eta = eta0 * N ** p
            models, shards = [], []
            for r in range(N):
                m = FMTrainer(f"-c -factors 8 -num_features {1 << bits} -eta0 {eta} -sigma 0.01 -seed 11",
                              device=dev)
                sidx = idx[r::N].contiguous()
                n = sidx.shape[0]
                shards.append(SparseRows(torch.arange(0, n * 39 + 1, 39, dtype=torch.int64, device=dev),
                                         sidx.reshape(-1).contiguous(), None, y[r::N].contiguous()))
                m._ensure(shards[-1])
                models.append(m)
            for ep in range(epochs):
                # every replica trains one epoch of its shard, then the replicas are averaged (the
                # learners' per-epoch mix; -mix_interval 0 averages once after the last epoch)
                for m, s in zip(models, shards):
                    m.train_rows(s)
                if N > 1:
                    _mean_into(models, ("w", "V", "w0"))
            ll = torch.nn.functional.binary_cross_entropy_with_logits(models[0].predict_raw(rows=er), yy).item()
            rec = {"what": "fm", "N": N, "power": p, "eta0": round(eta, 5), "rows": n_rows, "epochs": epochs,
                   "logloss_heldout": round(ll, 5)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
            del models, shards
            torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--powers", type=float, nargs="+", default=[0.0, 0.5, 0.75])
    ap.add_argument("--what", nargs="+", default=["bpr", "fm"])
    a = ap.parse_args()
    if "bpr" in a.what:
        bpr(a.worlds, a.powers)
    if "fm" in a.what:
        fm(a.worlds, a.powers)


if __name__ == "__main__":
    main()
