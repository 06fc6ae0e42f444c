"""Throughput + quality for the BASELINE.json configs other than the headline FFM bench:

  classifier : train_classifier (AdaGrad logistic) on a9a-shaped libsvm rows (CPU engine, ws=1)
  linear_gpu : the same learner on 8M a9a-shaped rows on the GPU (replica-per-wave kernel)
  fm         : train_fm on Criteo-1TB-shaped rows (2^24 hashed features, bf16 V), 1 GPU
  gbdt       : GBT classifier on HIGGS-shaped dense rows (11M x 28, histogram kernel), 1 GPU
  rf         : random forest on the same data
  bprmf      : BPR-MF on MovieLens-20M-shaped implicit feedback (device negative sampling)

    python benchmarks/bench_configs.py [names...]      # one JSON line per config
    python benchmarks/bench_configs.py --gpus N [gbdt|xgboost|rf|bprmf|bprmf_shard ...]
                                                       # N ranks (one per GPU), rank 0 prints
Synthetic data of the named shapes (no datasets offline), random-init weights.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize()


def bench_classifier(dev="cpu"):
    from sklearn.metrics import roc_auc_score
    from hivemall_amd.io.synthetic import a9a_like
    from hivemall_amd.models.linear import TrainClassifier
    rows, y = a9a_like(32561)
    trows, ty = a9a_like(16281, seed=4)
    m = TrainClassifier("-loss logloss -opt adagrad -reg no -iters 10 -disable_cv", device=dev)
    r = m.prepare(rows, y)
    t0 = time.perf_counter()
    m.fit(rows=r)
    _sync(dev)
    dt = time.perf_counter() - t0
    p = 1 / (1 + np.exp(-m.decision_function(trows).cpu().numpy()))
    from sklearn.metrics import log_loss
    return {"config": "train_classifier adagrad logistic, a9a-shaped (32561 x 123, ~14 nnz), 10 epochs",
            "device": dev, "rows_per_s": round(32561 * 10 / dt), "seconds": round(dt, 3),
            "test_auc": round(roc_auc_score(ty, p), 4), "test_logloss": round(log_loss(ty, p), 4)}


def bench_linear_gpu(dev="cuda", n=8_000_000):
    from hivemall_amd.models.linear import SparseRows, TrainClassifier
    g = torch.Generator(device=dev).manual_seed(0)
    nnz = 14
    idx = torch.randint(1, 124, (n, nnz), generator=g, device=dev, dtype=torch.int32)
    wtrue = torch.randn(124, generator=g, device=dev)
    logit = wtrue[idx.long()].sum(1) * 0.5
    y = torch.where(torch.rand(n, generator=g, device=dev) < torch.sigmoid(logit), 1.0, -1.0)
    rows = SparseRows(torch.arange(0, n * nnz + 1, nnz, dtype=torch.int64, device=dev),
                      idx.reshape(-1).contiguous(), None, y)
    m = TrainClassifier("-loss logloss -opt adagrad -reg no -iters 1 -dims 124", device=dev)
    m.fit(rows=rows)  # warm (allocations, replicas)
    _sync(dev)
    t0 = time.perf_counter()
    m.fit(rows=rows)
    _sync(dev)
    dt = time.perf_counter() - t0
    s = m.decision_function(rows=rows).float()
    acc = float(((s > 0) == (y > 0)).float().mean().item())
    return {"config": f"train_classifier adagrad logistic, {n} a9a-shaped rows, GPU replica-per-wave",
            "device": dev, "replicas": m.state.R, "rows_per_s": round(n / dt), "train_acc": round(acc, 4)}


def bench_linear_hashed(dev="cuda", n_rows=8 * 262144, bits=24, epochs=2):
    """train_classifier -loss logloss -opt adagrad at Hivemall's default -dims 2^24 on
    Criteo-shaped hashed rows (39 nnz): the shared-table Hogwild engine on the GPU, the
    sequential engine on the CPU."""
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.linear import SparseRows, TrainClassifier
    idx, y = criteo_like(n_rows, bits, seed=5, device=dev)
    rows = SparseRows(torch.arange(0, n_rows * 39 + 1, 39, dtype=torch.int64, device=dev),
                      idx.reshape(-1).contiguous(), None, y)
    m = TrainClassifier(f"-loss logloss -opt adagrad -dims {1 << bits} -iters 1", device=dev)
    m.fit(rows=rows)                                   # epoch 1 (state allocation, code load)
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(epochs - 1):
        m.fit(rows=rows)
    _sync(dev)
    dt = time.perf_counter() - t0
    eidx, ey = criteo_like(200000, bits, seed=77, device=dev)
    er = SparseRows(torch.arange(0, 200000 * 39 + 1, 39, dtype=torch.int64, device=dev),
                    eidx.reshape(-1).contiguous(), None, None)
    ll = torch.nn.functional.binary_cross_entropy_with_logits(m.decision_function(rows=er),
                                                              (ey > 0).float()).item()
    eng = "shared-table Hogwild" if m.state.meta.get("shared") else f"{m.state.R} replicas"
    return {"config": f"train_classifier adagrad logistic, Criteo-shaped {n_rows} x 39 nnz, -dims 2^{bits}",
            "device": dev, "engine": eng, "rows_per_s": round(n_rows * (epochs - 1) / dt),
            "heldout_logloss_after_epochs": round(ll, 5), "epochs": epochs}


def bench_fm(dev="cuda", n_rows=8 * 262144, bits=24):
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.models.linear import SparseRows
    idx, y = criteo_like(n_rows, bits, seed=5, device=dev)
    rows = SparseRows(torch.arange(0, n_rows * 39 + 1, 39, dtype=torch.int64, device=dev),
                      idx.reshape(-1).contiguous(), None, y)
    extra = os.environ.get("HM_BENCH_FM_OPTS", "")         # A/B knobs, e.g. "-grid 512"
    t = FMTrainer(f"-c -factors 8 -num_features {1 << bits} -eta0 0.01 -sigma 0.01 {extra}", device=dev)
    t.fit(rows=rows)
    _sync(dev)
    t0 = time.perf_counter()
    t.train_rows(rows)
    _sync(dev)
    dt = time.perf_counter() - t0
    eidx, ey = criteo_like(200000, bits, seed=77, device=dev)
    er = SparseRows(torch.arange(0, 200000 * 39 + 1, 39, dtype=torch.int64, device=dev),
                    eidx.reshape(-1).contiguous(), None, None)
    ll = torch.nn.functional.binary_cross_entropy_with_logits(t.predict_raw(rows=er), (ey > 0).float()).item()
    return {"config": f"train_fm k=8, Criteo-1TB-shaped (39 fields, 2^{bits} hashed features), " + ("bf16 V" if dev == "cuda" else "fp32 V"),
            "device": dev, "rows_per_s": round(n_rows / dt), "heldout_logloss_after_2_epochs": round(ll, 5)}


def bench_gbdt(dev="cuda", n=11_000_000, trees=100):
    from sklearn.metrics import roc_auc_score
    from hivemall_amd.io.synthetic import higgs_like
    from hivemall_amd.models.trees import GradientTreeBoostingClassifier
    X, y = higgs_like(n, device=dev)
    Xt, yt = higgs_like(500000, seed=9, device=dev)
    # warm-up (kernel code objects load lazily on first launch), then the timed fit
    GradientTreeBoostingClassifier("-trees 2 -max_depth 8", device=dev).fit(X[:100000], y[:100000].long())
    gb = GradientTreeBoostingClassifier(f"-trees {trees} -eta 0.1 -max_depth 8 -subsample 1.0", device=dev)
    _sync(dev)
    t0 = time.perf_counter()
    gb.fit(X, y.long())
    _sync(dev)
    dt = time.perf_counter() - t0
    auc = roc_auc_score(yt.cpu().numpy(), gb.predict_proba(Xt)[:, 1])
    return {"config": f"GBT classifier, HIGGS-shaped {n} x 28, depth 8, {trees} trees, 256-bin histograms",
            "device": dev, "seconds": round(dt, 3), "ms_per_tree": round(dt * 1e3 / trees, 2),
            "row_trees_per_s": round(n * trees / dt), "test_auc": round(float(auc), 4)}


def bench_rf(dev="cuda", n=11_000_000, trees=50):
    from sklearn.metrics import roc_auc_score
    from hivemall_amd.io.synthetic import higgs_like
    from hivemall_amd.models.trees import RandomForestClassifier
    X, y = higgs_like(n, device=dev)
    Xt, yt = higgs_like(500000, seed=9, device=dev)
    RandomForestClassifier("-trees 2 -max_depth 12", device=dev).fit(X[:100000], y[:100000].long())
    rf = RandomForestClassifier(f"-trees {trees} -max_depth 12", device=dev)
    _sync(dev)
    t0 = time.perf_counter()
    rf.fit(X, y.long())
    _sync(dev)
    dt = time.perf_counter() - t0
    auc = roc_auc_score(yt.cpu().numpy(), rf.predict_proba(Xt)[:, 1])
    return {"config": f"RandomForest classifier, HIGGS-shaped {n} x 28, depth 12, {trees} trees",
            "device": dev, "seconds": round(dt, 3), "ms_per_tree": round(dt * 1e3 / trees, 2),
            "row_trees_per_s": round(n * trees / dt), "test_auc": round(float(auc), 4)}


def bench_bprmf(dev="cuda", k=64, epochs=3, opts=""):
    from hivemall_amd.io.synthetic import movielens_like
    from hivemall_amd.models.mf import BPRMF, auc_implicit
    us, its = movielens_like(device=dev, k=16)
    n = us.numel()
    ntest = 200000
    m = BPRMF(f"-factors {k} -iters 1 -eta0 0.05 {opts}", device=dev)
    m.fit_implicit(us[:-ntest], its[:-ntest], 138493, 27278, epochs=1)
    _sync(dev)
    t0 = time.perf_counter()
    m.fit_implicit(us[:-ntest], its[:-ntest], 138493, 27278, epochs=epochs)
    _sync(dev)
    dt = time.perf_counter() - t0
    auc = auc_implicit(m, us[-ntest:].cpu().numpy(), its[-ntest:].cpu().numpy())
    return {"config": f"BPR-MF k={k}, MovieLens-20M-shaped ({n} interactions, 138493 users, 27278 items), "
                      f"device negative sampling", "device": dev,
            "triples_per_s": round((n - ntest) * epochs / dt), "sampled_auc": round(auc, 4),
            "opts": opts, "grid": m._grid()}


def bench_xgboost(dev="cuda", n=11_000_000, rounds=100):
    """train_xgboost binary:logistic on HIGGS-shaped rows (second-order stats, learned NaN
    directions), the xgboost4j replacement; quality against scikit-learn in test_xgboost."""
    from sklearn.metrics import roc_auc_score
    from hivemall_amd.io.synthetic import higgs_like
    from hivemall_amd.models.xgboost import XGBoostClassifier
    X, y = higgs_like(n, device=dev)
    Xt, yt = higgs_like(500000, seed=9, device=dev)
    XGBoostClassifier("-num_round 2 -max_depth 6", device=dev).fit(X[:100000], y[:100000])
    xg = XGBoostClassifier(f"-num_round {rounds} -max_depth 6 -eta 0.1", device=dev)
    _sync(dev)
    t0 = time.perf_counter()
    xg.fit(X, y)
    _sync(dev)
    dt = time.perf_counter() - t0
    auc = roc_auc_score(yt.cpu().numpy(), xg.predict_proba(Xt)[:, -1])
    return {"config": f"train_xgboost binary:logistic, HIGGS-shaped {n} x 28, depth 6, {rounds} rounds",
            "device": dev, "seconds": round(dt, 3), "ms_per_round": round(dt * 1e3 / rounds, 2),
            "row_rounds_per_s": round(n * rounds / dt), "test_auc": round(float(auc), 4)}


# ------------------------------------------------------------------ N-GPU (one process per GPU)
# BASELINE.json:10-11: RF / GBDT on HIGGS-shaped dense rows and BPR-MF on MovieLens-20M-shaped
# implicit feedback on 8 x MI355X.  ``--gpus N`` starts N ranks (bench.py's self-launch); the
# dataset is fixed (strong scaling): boosting shards the 11 M rows (rows r, r + N, ...) and
# all-reduces the per-level histograms; RF keeps all rows on every rank and splits the trees;
# BPR shards the interactions and mixes the factor tables every epoch (-mix_interval 1), or
# row-shards the tables over the ranks (-shard_model, explicit triples).  Rank 0 prints the
# JSON; time = max over ranks.

def _ctx():
    from hivemall_amd.parallel.dist import init_distributed
    from hivemall_amd.parallel.mix import ModelMixer
    ctx = init_distributed()
    return ctx, ModelMixer(ctx)


def _timed(ctx, mixer, fn):
    dev = ctx.device
    _sync(dev)
    ctx.barrier()
    t0 = time.perf_counter()
    out = fn()
    _sync(dev)
    ctx.barrier()
    return out, mixer.all_reduce_scalar(time.perf_counter() - t0, "max")


def _dist_fields(ctx):
    return {"world": ctx.world_size, "rccl_world": ctx.world_size if ctx.backend == "nccl" else None,
            "dist_backend": ctx.backend, "scaling": "strong"}


def bench_gbdt_dp(n=11_000_000, trees=100, depth=8, xgb=False):
    """Row-sharded boosting: rank r holds rows r, r + N, ... of the 11 M; histograms all-reduced."""
    from sklearn.metrics import roc_auc_score
    from hivemall_amd.io.synthetic import higgs_like
    from hivemall_amd.models.trees import GradientTreeBoostingClassifier
    from hivemall_amd.models.xgboost import XGBoostClassifier
    ctx, mixer = _ctx()
    dev = ctx.device
    X, y = higgs_like(n, device=dev)
    me = slice(ctx.rank, None, ctx.world_size)
    X, y = X[me].contiguous(), y[me].contiguous()
    kw = dict(device=dev, mixer=mixer, rank=ctx.rank)
    if xgb:
        XGBoostClassifier("-num_round 2 -max_depth 6", **kw).fit(X[:100000], y[:100000])
    else:
        GradientTreeBoostingClassifier("-trees 2 -max_depth 8", **kw).fit(X[:100000], y[:100000].long())
    # the per-level histogram all-reduces, timed on the compute stream
    mixer.time_collectives(True)
    hist_bytes = mixer.bytes_reduced
    if xgb:
        m, dt = _timed(ctx, mixer, lambda: XGBoostClassifier(
            f"-num_round {trees} -max_depth {depth} -eta 0.1", **kw).fit(X, y))
    else:
        m, dt = _timed(ctx, mixer, lambda: GradientTreeBoostingClassifier(
            f"-trees {trees} -eta 0.1 -max_depth {depth} -subsample 1.0", **kw).fit(X, y.long()))
    ar_ms = mixer.all_reduce_scalar(mixer.collective_ms(), "max")
    hist_bytes = mixer.bytes_reduced - hist_bytes
    mixer.time_collectives(False)
    Xt, yt = higgs_like(500000, seed=9, device=dev)
    auc = roc_auc_score(yt.cpu().numpy(), m.predict_proba(Xt)[:, -1])
    name = "train_xgboost binary:logistic" if xgb else "GBT classifier"
    return {"config": f"{name}, HIGGS-shaped {n} x 28 rows sharded over {ctx.world_size} ranks, depth {depth}, "
                      f"{trees} trees, per-level histogram all-reduce", "device": str(dev), "seconds": round(dt, 3),
            "ms_per_tree": round(dt * 1e3 / trees, 2), "row_trees_per_s": round(n * trees / dt),
            "test_auc": round(float(auc), 4),
            "hist_allreduce_ms_per_tree": round(ar_ms / trees, 3) if ctx.world_size > 1 else 0.0,
            "hist_allreduce_mb_per_tree": round(hist_bytes / trees / 2**20, 2),
            **_dist_fields(ctx)}


def bench_rf_dp(n=11_000_000, trees=48, depth=12):
    """RandomForest: every rank all rows, trees t with t % N == rank; the union is the forest."""
    from sklearn.metrics import roc_auc_score
    from hivemall_amd.io.synthetic import higgs_like
    from hivemall_amd.models.trees import RandomForestClassifier
    ctx, mixer = _ctx()
    dev = ctx.device
    X, y = higgs_like(n, device=dev)
    kw = dict(device=dev, mixer=mixer, rank=ctx.rank)
    RandomForestClassifier("-trees 2 -max_depth 12", device=dev).fit(X[:100000], y[:100000].long())
    m, dt = _timed(ctx, mixer, lambda: RandomForestClassifier(f"-trees {trees} -max_depth {depth}", **kw).fit(X, y.long()))
    # the forest is the union of the ranks' trees (SQL: the UDTF tables are concatenated)
    import torch.distributed as tdist
    if ctx.world_size > 1:
        parts = [None] * ctx.world_size
        tdist.all_gather_object(parts, [t.to_json() for t in m.trees])
        from hivemall_amd.models.trees import Tree
        m.trees = [Tree.from_json(j) for part in parts for j in part]
    Xt, yt = higgs_like(500000, seed=9, device=dev)
    auc = roc_auc_score(yt.cpu().numpy(), m.predict_proba(Xt)[:, 1])
    return {"config": f"RandomForest classifier, HIGGS-shaped {n} x 28, depth {depth}, {trees} trees split over "
                      f"{ctx.world_size} ranks", "device": str(dev), "seconds": round(dt, 3),
            "ms_per_tree": round(dt * 1e3 / trees, 2), "row_trees_per_s": round(n * trees / dt),
            "test_auc": round(float(auc), 4), "trees_in_forest": len(m.trees), **_dist_fields(ctx)}


def bench_bprmf_dp(k=64, epochs=3, shard_model=False, n_ratings=20000263, n_users=138493, n_items=27278):
    """BPR-MF: interactions sharded over the ranks; factor tables mixed every epoch, or
    row-sharded over the ranks (-shard_model: explicit triples, uniform negatives)."""
    from hivemall_amd.io.synthetic import movielens_like
    from hivemall_amd.models.mf import BPRMF, auc_implicit
    ctx, mixer = _ctx()
    dev = ctx.device
    us, its = movielens_like(n_ratings, n_users, n_items, device=dev, k=16)
    n = us.numel()
    ntest = min(200000, n // 10)
    tu, ti = us[:-ntest], its[:-ntest]
    me = slice(ctx.rank, None, ctx.world_size)
    tu, ti = tu[me].contiguous(), ti[me].contiguous()
    kw = dict(device=dev, mixer=mixer, rank=ctx.rank)
    if shard_model:
        g = torch.Generator(device=dev).manual_seed(100 + ctx.rank)
        tj = torch.randint(0, n_items, (tu.numel(),), generator=g, device=dev, dtype=torch.int32)
        opts = f"-factors {k} -iters {epochs} -eta0 0.05 -shard_model -disable_cv"
        m, dt = _timed(ctx, mixer, lambda: BPRMF(opts, **kw).fit(tu, ti, tj))
    else:
        opts = f"-factors {k} -iters 1 -eta0 0.05 -mix_interval 1 -disable_cv"
        BPRMF(opts, **kw).fit_implicit(tu[:100000], ti[:100000], n_users, n_items, epochs=1)
        m, dt = _timed(ctx, mixer, lambda: BPRMF(opts, **kw).fit_implicit(tu, ti, n_users, n_items, epochs=epochs))
    auc = auc_implicit(m, us[-ntest:].cpu().numpy(), its[-ntest:].cpu().numpy())
    return {"config": f"BPR-MF k={k}, MovieLens-20M-shaped ({n} interactions, {n_users} users, {n_items} items) "
                      f"sharded over {ctx.world_size} ranks, "
                      + ("row-sharded tables (-shard_model), explicit triples" if shard_model else
                         "device negative sampling, tables mixed every epoch"),
            "device": str(dev), "triples_per_s": round((n - ntest) * epochs / dt), "seconds": round(dt, 3),
            "sampled_auc": round(auc, 4), **_dist_fields(ctx)}


DIST = {"gbdt": bench_gbdt_dp, "xgboost": lambda **kw: bench_gbdt_dp(xgb=True, **{"depth": 6, **kw}),
        "rf": bench_rf_dp, "bprmf": bench_bprmf_dp,
        "bprmf_shard": lambda **kw: bench_bprmf_dp(shard_model=True, **kw)}
_BPR_SMALL = dict(k=8, epochs=2, n_ratings=60000, n_users=3000, n_items=1500)
DIST_SMALL = {"gbdt": dict(n=20000, trees=3, depth=4), "xgboost": dict(n=20000, trees=3, depth=4),
              "rf": dict(n=20000, trees=4, depth=6), "bprmf": _BPR_SMALL, "bprmf_shard": _BPR_SMALL}


def main_dist(names, gpus, small):
    """--gpus N: the N-rank entry point (BASELINE configs 4 and 5)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if gpus > 1 and "WORLD_SIZE" not in os.environ:
        # start the ranks as a child process, before this process touches the GPU
        import subprocess
        from bench import _free_port
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.run(cmd, env=env).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        print(f"[bench_configs] --gpus {gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    from hivemall_amd.parallel.dist import shutdown
    for name in names or ["gbdt", "rf", "bprmf"]:
        kw = dict(DIST_SMALL.get(name, {})) if small else {}
        res = DIST[name](**kw)
        res["bench"] = name
        res["n_gpus"] = gpus
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps(res), flush=True)
    shutdown()


ALL = {"classifier": bench_classifier, "linear_gpu": bench_linear_gpu, "linear_hashed": bench_linear_hashed,
       "fm": bench_fm,
       "gbdt": bench_gbdt, "rf": bench_rf, "bprmf": bench_bprmf, "xgboost": bench_xgboost}

SMALL = {"linear_gpu": dict(n=20000), "linear_hashed": dict(n_rows=20000, bits=16), "fm": dict(n_rows=20000, bits=16),
         "gbdt": dict(n=20000, trees=4), "rf": dict(n=20000, trees=2), "bprmf": dict(k=16, epochs=1),
         "xgboost": dict(n=20000, rounds=3)}

# CPU reference-class points (8-core host): same code paths on the C++/OpenMP engines
CPU = {"linear_gpu": dict(n=1_000_000), "linear_hashed": dict(n_rows=8 * 262144, bits=24),"fm": dict(n_rows=262144, bits=20),
       "gbdt": dict(n=1_000_000, trees=10), "rf": dict(n=1_000_000, trees=4), "bprmf": dict(k=64, epochs=1),
       "xgboost": dict(n=1_000_000, rounds=10)}

if __name__ == "__main__":
    if "--gpus" in sys.argv:
        i = sys.argv.index("--gpus")
        main_dist([a for a in sys.argv[1:] if not a.startswith("--") and a != sys.argv[i + 1]],
                  int(sys.argv[i + 1]), "--small" in sys.argv)
        sys.exit(0)
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    small = "--small" in sys.argv  # CPU smoke of the harness itself (tiny shapes)
    cpu = "--cpu" in sys.argv      # reference-class CPU measurement
    prof = "--profile" in sys.argv  # per-kernel device-time table via torch.profiler
    names = args or list(ALL)
    for name in names:
        kw = dict(SMALL.get(name, {})) if small else dict(CPU.get(name, {})) if cpu else {}
        if small or cpu:
            kw["dev"] = "cpu"
        if prof:
            from torch.profiler import ProfilerActivity, profile
            with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as pr:
                res = ALL[name](**kw)
            os.makedirs("gpurun_out", exist_ok=True)
            with open(f"gpurun_out/torchprof_{name}.txt", "w") as f:
                f.write(pr.key_averages().table(sort_by="self_cuda_time_total", row_limit=40))
                f.write("\n\n")
                f.write(pr.key_averages().table(sort_by="self_cpu_time_total", row_limit=30))
        else:
            res = ALL[name](**kw)
        for r in (res if isinstance(res, list) else [res]):
            r["bench"] = name
            print(json.dumps(r), flush=True)
