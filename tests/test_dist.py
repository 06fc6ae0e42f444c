"""Multi-process (gloo, world_size=2) tests of the RCCL mixing layer — the MixServerTest
analogue: N learners, one mixed model."""
import io
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _TensorBytes(bytes):
    """A tensor serialised by value (torch.save) inside a queued result."""


def _pack(x):
    if torch.is_tensor(x):
        buf = io.BytesIO()
        torch.save(x.detach().cpu().clone(), buf)
        return _TensorBytes(buf.getvalue())
    if isinstance(x, dict):
        return {k: _pack(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_pack(v) for v in x)
    return x


def _unpack(x):
    if isinstance(x, _TensorBytes):
        return torch.load(io.BytesIO(bytes(x)), weights_only=True)
    if isinstance(x, dict):
        return {k: _unpack(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_unpack(v) for v in x)
    return x


def _worker(rank, world, port, fn_name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import tests.test_dist as T
    from hivemall_amd.parallel import dist as D

    D._CTX = None
    ctx = D.init_distributed(backend="gloo", device="cpu")
    try:
        if ":" in fn_name:
            import importlib
            mod, fn = fn_name.split(":")
            f = getattr(importlib.import_module(mod), fn)
        else:
            f = getattr(T, fn_name)
        # results travel by value: a tensor put on an mp queue is shared through a file
        # descriptor that dies with this process, racing the parent's get (FileNotFoundError)
        q.put((rank, _pack(f(ctx))))
    finally:
        D.shutdown()


def run_world(fn_name, world=2):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {r: _unpack(b) for r, b in (q.get(timeout=120) for _ in ps)}
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return out


def _avg(ctx):
    from hivemall_amd.parallel.mix import ModelMixer

    m = ModelMixer(ctx, bucket_mb=0.001, small_bytes=64)
    big = torch.full((10000,), float(ctx.rank + 1))
    small = torch.tensor([ctx.rank * 2.0, 1.0])
    m.average([big, small])
    return big.tolist()[:3] + small.tolist()


def _avg_strided(ctx):
    """A non-contiguous view (the V half of the packed FFM table) mixes like a plain tensor."""
    from hivemall_amd.parallel.mix import ModelMixer

    m = ModelMixer(ctx, bucket_mb=0.001, small_bytes=64)
    VG = torch.zeros(50, 3, 2, 4)
    VG[:, :, 0] = float(ctx.rank + 1)
    VG[:, :, 1] = 7.0 * (ctx.rank + 1)       # G: optimizer state, stays local
    m.average([VG[:, :, 0, :]])
    return [float(VG[:, :, 0].mean()), float(VG[:, :, 1].mean())]


def _kld(ctx):
    from hivemall_amd.parallel.mix import ModelMixer

    m = ModelMixer(ctx)
    w = torch.tensor([1.0, 2.0]) * (ctx.rank + 1)
    cov = torch.tensor([0.5, 1.0]) * (ctx.rank + 1)
    m.argmin_kld(w, cov)
    return w.tolist() + cov.tolist()


def _ffm_dp(ctx):
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.ffm import FFMBatch, FFMTrainer
    from hivemall_amd.parallel.mix import ModelMixer

    idx, y = criteo_like(2000, hash_bits=10, seed=100 + ctx.rank)
    t = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 10 -mix_interval 1 -batch_size 500",
                   device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
    t.fit(batch=FFMBatch(idx, None, None, y))
    return float(t.state["V"].sum()), float(t.state["w"].sum())


def _gbt_dp(ctx):
    """Data-parallel boosting: each rank holds half the rows; histograms are all-reduced per
    level, so both ranks must grow the same trees."""
    from hivemall_amd.io.synthetic import higgs_like
    from hivemall_amd.models.trees import GradientTreeBoostingClassifier
    from hivemall_amd.models.xgboost import XGBoostTrainer
    from hivemall_amd.parallel.mix import ModelMixer

    X, y = higgs_like(8000, seed=40 + ctx.rank)
    gb = GradientTreeBoostingClassifier("-trees 3 -max_depth 4 -subsample 1.0 -seed 5", device="cpu",
                                        mixer=ModelMixer(ctx), rank=ctx.rank).fit(X, y.long())
    xg = XGBoostTrainer("-num_round 3 -max_depth 4", device="cpu", mixer=ModelMixer(ctx),
                        rank=ctx.rank).fit(X, y)
    return (list(gb.model_table()["pred_models"].map(tuple)), gb.intercepts,
            xg.model_table()["model"].iloc[0])


def test_boosting_data_parallel_identical_trees():
    out = run_world("_gbt_dp")
    assert out[0][0] == out[1][0] and out[0][1] == out[1][1]
    assert out[0][2] == out[1][2]


def test_mix_average_bucketed():
    out = run_world("_avg")
    for r in (0, 1):
        assert out[r] == [1.5, 1.5, 1.5, 1.0, 1.0]


def test_mix_average_strided_view():
    out = run_world("_avg_strided")
    assert out[0][0] == 1.5 and out[1][0] == 1.5
    assert out[0][1] == 7.0 and out[1][1] == 14.0


def test_mix_argmin_kld():
    out = run_world("_kld")
    # w_r = (r+1)*w, cov_r = (r+1)*c  ->  sum(w/c) / sum(1/c)
    import numpy as np

    w = np.array([1.0, 2.0]); c = np.array([0.5, 1.0])
    num = w / c + 2 * w / (2 * c)
    inv = 1 / c + 1 / (2 * c)
    np.testing.assert_allclose(out[0], list(num / inv) + list(1 / inv), rtol=1e-6)
    assert out[0] == out[1]


def test_ffm_data_parallel_replicas_identical():
    out = run_world("_ffm_dp")
    assert out[0] == pytest.approx(out[1], rel=1e-6)


def _ffm_dp_step_rule(ctx):
    """The N^p step rule applies only with periodic mixing; an absurd power trips the guard."""
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.ffm import DP_GUARD_POWER, FFMBatch, FFMTrainer
    from hivemall_amd.parallel.mix import ModelMixer

    base = "-c -factors 4 -num_fields 39 -feature_hashing 10 -batch_size 250"
    end_only = FFMTrainer(base, device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
    periodic = FFMTrainer(base + " -mix_interval 1", device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
    idx, y = criteo_like(3000, hash_bits=10, seed=300 + ctx.rank)
    wild = FFMTrainer(base + " -mix_interval 1 -dp_lr_power 9 -eta0 1.0", device="cpu",
                      mixer=ModelMixer(ctx), rank=ctx.rank)
    eta_before = wild.hyper.eta0
    wild.fit(batch=FFMBatch(idx, None, None, y))
    return (end_only.hyper.eta0, periodic.hyper.eta0, eta_before, wild.hyper.eta0,
            wild.dp_guard_tripped, wild._dp_power == DP_GUARD_POWER)


def test_ffm_dp_step_rule_gated_and_guarded():
    """-mix_interval 0 (one average at the end, Hivemall's mappers) keeps eta0; the
    N^0.75 rule needs periodic mixes.  VERDICT r4 weak 4: a mixed-loss rise between mixes drops
    the power to 0.5 (here p = 9 at N = 2: a step size x512 must trip it)."""
    out = run_world("_ffm_dp_step_rule")
    for r in (0, 1):
        e0, e1, wild0, wild1, tripped, at_half = out[r]
        assert e0 == pytest.approx(0.2)
        assert e1 == pytest.approx(0.2 * 2 ** 0.75)
        assert wild0 == pytest.approx(2 ** 9)
        assert tripped and at_half and wild1 == pytest.approx(2 ** 0.5)
    assert out[0] == out[1]


def _ffm_dp_sparse(ctx):
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.ffm import FFMBatch, FFMTrainer
    from hivemall_amd.parallel.mix import ModelMixer

    res = []
    for extra in ("", " -mix_sparse"):
        idx, y = criteo_like(1200, hash_bits=16, seed=100 + ctx.rank)
        t = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 16 -mix_interval 1 "
                       "-batch_size 200 -seed 7" + extra,
                       device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
        t.fit(batch=FFMBatch(idx, None, None, y))
        res.append([float(t.state["V"].double().sum()), float(t.state["w"].double().sum())])
    sm = t._sparse_mixer
    res.append([sm.sparse_rows, sm.dense_mixes])
    return res


def test_ffm_sparse_mixing_matches_dense_mixing():
    """-mix_sparse (touched-row all-gather) trains the same replicas as the dense all-reduce."""
    out = run_world("_ffm_dp_sparse")
    for r in (0, 1):
        dense, sparse, (rows, dense_mixes) = out[r]
        assert sparse == pytest.approx(dense, rel=1e-4, abs=1e-3)
        assert rows > 0 and dense_mixes >= 1
    assert out[0][1] == pytest.approx(out[1][1], rel=1e-6)


def test_bench_torchrun_cpu_world2():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "512", "--hash-bits", "10",
           "--mix-every", "1", "--eval-rows", "512", "--device", "cpu", "--resident-batches", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["value"] > 0


def test_bench_self_launch_cpu_world2():
    """`python bench.py --gpus 2` with no launcher starts 2 ranks itself (the driver contract:
    the JSON's value is the whole-job rate of N ranks), and reports the mix cost."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--batch", "512", "--hash-bits", "10", "--mix-every", "1",
           "--eval-rows", "512", "--device", "cpu", "--resident-batches", "2", "--mix-probe", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["dist_backend"] == "gloo" and d["rccl_world"] is None
    assert d["config"]["mixes_in_timed_region"] == 2
    assert d["config"]["linear_steps"] == "plain-stores"   # replicas that mix (dp_lin_mode)
    assert d["mix_ms"] > 0 and d["mix_wire_bytes_per_rank"] > 0 and d["mix_bus_gbps"] > 0


def test_bench_refuses_world_mismatch():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "3", "--steps", "1", "--warmup", "0", "--batch", "256", "--hash-bits", "10",
           "--eval-rows", "256", "--device", "cpu", "--resident-batches", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode != 0
    assert "--gpus 3 but" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def _fm_mf_bpr_dp(ctx):
    import numpy as np

    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.models.mf import BPRMF, MatrixFactorization
    from hivemall_amd.parallel.mix import ModelMixer

    rng = np.random.default_rng(50 + ctx.rank)
    out = {}
    for extra in ("", " -mix_sparse"):
        feats = [[f"{j}:1.0" for j in rng.choice(3000, 8, replace=False)] for _ in range(300)]
        y = rng.integers(0, 2, 300)
        fm = FMTrainer("-c -factors 4 -iters 2 -num_features 3001 -seed 3 -mix_interval 1"
                       " -batch_size 100" + extra, device="cpu", mixer=ModelMixer(ctx),
                       rank=ctx.rank).fit(feats, y)
        u, i = rng.integers(0, 50, 400), rng.integers(0, 80, 400)
        mf = MatrixFactorization("-factors 4 -iters 3 -seed 3 -mix_interval 1" + extra,
                                 device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
        mf.fit(u, i, rng.random(400) * 5)
        bp = BPRMF("-factors 4 -iters 3 -seed 3" + extra, device="cpu", mixer=ModelMixer(ctx),
                   rank=ctx.rank).fit(u, i, rng.integers(0, 80, 400))
        out[extra or "dense"] = [float(fm.state["V"].double().sum()), float(fm.state["w"].sum()),
                                 int(fm.touched.sum()), float(mf.state["P"].double().sum()),
                                 float(mf.state["Q"].double().sum()),
                                 float(bp.state["Q"].double().sum()), int(mf.seen_u.sum())]
    return out


def test_fm_mf_bpr_data_parallel_replicas_identical():
    """FM / MF / BPR replicas agree after mixing (dense and touched-row modes), and the "seen"
    masks are the union over ranks (one model table per job)."""
    out = run_world("_fm_mf_bpr_dp")
    for mode in ("dense", " -mix_sparse"):
        assert out[0][mode] == pytest.approx(out[1][mode], rel=1e-5, abs=1e-5)


def _gbt_union_equal(ctx):
    """World-2 row-sharded boosting with fixed bin edges vs ONE process on the union of the
    shards: histograms are additive, so the trees must be the same up to float summation order."""
    import numpy as np

    from hivemall_amd.io.synthetic import higgs_like
    from hivemall_amd.models.trees import GradientTreeBoostingClassifier, quantize
    from hivemall_amd.models.xgboost import XGBoostTrainer
    from hivemall_amd.parallel.mix import ModelMixer

    X, y = higgs_like(6000, seed=40)
    edges = quantize(X, 64).edges
    mine = slice(ctx.rank, None, ctx.world_size)
    opts = "-trees 4 -max_depth 4 -subsample 1.0 -seed 5 -num_bins 64"
    xopts = "-num_round 4 -max_depth 4 -num_bins 64"
    dp = GradientTreeBoostingClassifier(opts, device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank,
                                        edges=edges).fit(X[mine], y[mine].long())
    xdp = XGBoostTrainer(xopts, device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank, edges=edges).fit(X[mine], y[mine])
    one = GradientTreeBoostingClassifier(opts, device="cpu", edges=edges).fit(X, y.long())
    xone = XGBoostTrainer(xopts, device="cpu", edges=edges).fit(X, y)
    Xt, _ = higgs_like(2000, seed=41)
    feats = lambda m: [t.feature for it in m.iters for t in it]
    xfeats = lambda m: [t.feature for rt in m.trees for t in rt]
    return {"feat_dp": feats(dp), "feat_one": feats(one), "p_dp": dp.predict_proba(Xt), "p_one": one.predict_proba(Xt),
            "xfeat_dp": xfeats(xdp), "xfeat_one": xfeats(xone),
            "xp_dp": xdp.margin(Xt).cpu().numpy(), "xp_one": xone.margin(Xt).cpu().numpy()}


def test_boosting_data_parallel_equals_single_process_on_union():
    import numpy as np

    out = run_world("_gbt_union_equal")
    for r in (0, 1):
        o = out[r]
        assert o["feat_dp"] == o["feat_one"] and o["xfeat_dp"] == o["xfeat_one"]
        np.testing.assert_allclose(o["p_dp"], o["p_one"], atol=1e-5)
        np.testing.assert_allclose(o["xp_dp"], o["xp_one"], atol=1e-4)


def test_bench_configs_n_gpu_entry_point_cpu_world2():
    """benchmarks/bench_configs.py --gpus 2 (BASELINE configs 4 and 5): self-launches 2 ranks
    (gloo here) and rank 0 prints one JSON line per config with the world fields."""
    cmd = [sys.executable, os.path.join(ROOT, "benchmarks", "bench_configs.py"), "--gpus", "2", "--small",
           "gbdt", "rf", "bprmf"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [d["bench"] for d in recs] == ["gbdt", "rf", "bprmf"]
    for d in recs:
        assert d["world"] == 2 and d["n_gpus"] == 2 and d["dist_backend"] == "gloo"
    assert recs[1]["trees_in_forest"] == 4
    assert 0.6 < recs[0]["test_auc"] and 0.6 < recs[2]["sampled_auc"]
    # the per-level histogram all-reduce of data-parallel boosting, broken out per tree
    assert recs[0]["hist_allreduce_ms_per_tree"] > 0 and recs[0]["hist_allreduce_mb_per_tree"] > 0


def _metrics_dp(ctx):
    import tempfile

    import numpy as np

    from hivemall_amd.models.mf import MatrixFactorization
    from hivemall_amd.parallel.mix import ModelMixer

    path = os.path.join(tempfile.gettempdir(), f"hm_metrics_{os.environ['MASTER_PORT']}.jsonl")
    os.environ["HM_METRICS"] = path
    rng = np.random.default_rng(5 + ctx.rank)
    u, i = rng.integers(0, 50, 400), rng.integers(0, 80, 400)
    MatrixFactorization("-factors 4 -iters 3 -seed 3 -mix_interval 1", device="cpu",
                        mixer=ModelMixer(ctx), rank=ctx.rank).fit(u, i, rng.random(400) * 5)
    return path


def test_learner_metrics_stream_world2():
    """``HM_METRICS=<path>``: every learner epoch appends a rank-tagged record with the job-wide
    loss, rows/s and the mixes' time and wire bytes."""
    out = run_world("_metrics_dp")
    path = out[0]
    try:
        recs = [json.loads(l) for l in open(path)]
    finally:
        os.remove(path)
    assert sorted({r["rank"] for r in recs}) == [0, 1]
    r0 = [r for r in recs if r["rank"] == 0]
    assert [r["epoch"] for r in r0] == [1, 2, 3]
    for r in r0:
        assert r["learner"] == "train_mf_sgd" and r["rows"] == 400 and r["rows_per_s"] > 0
        assert r["mixes"] == 1 and r["mixed_bytes"] > 50 * 4 * 4 and r["mix_ms"] > 0
    # the loss is the job-wide sum: both ranks log the same value
    r1 = [r for r in recs if r["rank"] == 1]
    assert [r["loss"] for r in r0] == [r["loss"] for r in r1]


def test_ffm_logloss_parity_world4_gloo():
    """The headline's "logloss parity" at N ranks (BASELINE.json:2): bench.py's exact schedule
    (synchronous shard mean every 10 steps, replicas stepping with eta0 / alpha x N^0.75) at
    world 4 on gloo, 2^16 hashed features (most slots are touched by one rank between mixes),
    against one rank over the same total rows: |delta| <= 1e-3 (SURVEY.md:766, fp32).
    benchmarks/dp_sim.py at this shape: +1.9e-4 (plain mean +1.27e-2); at the bench's shape,
    N = 8: +2.8e-4 (plain mean +5.3e-3), profiles/r4/."""
    sys.path.insert(0, ROOT)
    from benchmarks.dp_parity import main as dp_parity

    common = ["--worlds", "4", "--steps", "20", "--batch", "2048", "--hash-bits", "16",
              "--eval-rows", "32768", "--timeout", "900"]
    rec = dp_parity(common)[0]
    assert rec["mixes_timed"] == 2 and rec["backend"] == "gloo" and rec["dp_lr_scale"] > 2.8
    assert abs(rec["delta"]) <= 1e-3, rec
    # N replicas mixed never do worse than one rank trained on its own share
    assert rec["logloss_N"] <= rec["logloss_1_same_steps"], rec


def _bpr_dp4(ctx):
    from hivemall_amd.io.synthetic import movielens_like
    from hivemall_amd.models.mf import BPRMF, auc_implicit
    from hivemall_amd.parallel.mix import ModelMixer

    us, its = movielens_like(n_ratings=120000, n_users=3000, n_items=1500, seed=11)
    tu, ti, eu, ei = us[:-10000], its[:-10000], us[-10000:], its[-10000:]
    opts = "-factors 16 -iters 10 -eta0 0.05 -disable_cv -seed 7"
    one = BPRMF(opts, device="cpu")
    one.fit_implicit(tu, ti, n_users=3000, n_items=1500)
    W = ctx.world_size
    dp = BPRMF(opts + " -mix_interval 1", device="cpu", mixer=ModelMixer(ctx), rank=ctx.rank)
    dp.fit_implicit(tu[ctx.rank::W], ti[ctx.rank::W], n_users=3000, n_items=1500)
    return (auc_implicit(one, eu.numpy(), ei.numpy()), auc_implicit(dp, eu.numpy(), ei.numpy()),
            float(dp.state["P"].double().sum()))


def test_bpr_sampled_auc_world4_gloo():
    """VERDICT r4 item 8 (BASELINE config 5, BPR on 8 GPUs): 4 gloo ranks, each on every 4th
    positive pair, replicas averaged every epoch (plain mean, the factor tables), against one
    rank over all pairs: sampled AUC within 0.01 (measured here 0.711 vs 0.711; on MI355X at the
    ML-20M shape, N = 2/4/8 plain mean: 0.7116 / 0.7117 / 0.7118 vs 0.7095 for one replica,
    profiles/r5/dp_sim_bpr.jsonl).  Every rank ends with the same model."""
    out = run_world("_bpr_dp4", world=4)
    for r in range(4):
        auc1, aucn, _ = out[r]
        assert aucn >= auc1 - 0.01, (auc1, aucn)
    assert len({out[r][2] for r in range(4)}) == 1


def _fm_dp_rule(ctx):
    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.parallel.mix import ModelMixer

    mk = lambda extra: FMTrainer("-c -factors 4 -eta0 0.01" + extra, device="cpu",  # noqa: E731
                                 mixer=ModelMixer(ctx), rank=ctx.rank)
    return mk("").h.eta0, mk(" -mix_interval 4").h.eta0, mk(" -mix_interval 4 -dp_lr_power 0").h.eta0


def test_fm_dp_step_rule_gated():
    """train_fm's data-parallel step rule (eta0 x N^0.5, profiles/r5/dp_sim_fm.jsonl) applies only
    to replicas mixed during training; -mix_interval 0 (Hivemall's one average at the end) keeps
    eta0."""
    out = run_world("_fm_dp_rule")
    for r in (0, 1):
        end_only, periodic, off = out[r]
        assert end_only == pytest.approx(0.01) and off == pytest.approx(0.01)
        assert periodic == pytest.approx(0.01 * 2 ** 0.5)


def _avg_delta(ctx):
    """average_delta: bf16 deltas on the wire, fp32 consensus; every rank ends bit-identical,
    within a bf16 rounding of the step of the exact fp32 mean."""
    from hivemall_amd.parallel.mix import ModelMixer

    m = ModelMixer(ctx)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(50, 7, 4, generator=g)             # identical start on both ranks
    v = x[:, :5]                                       # a strided view, as the FFM V blocks
    m.average_delta([v])                               # first call: full precision + consensus
    exact = v.clone()
    res = []
    for it in range(3):
        step = torch.randn(50, 5, 4, generator=torch.Generator().manual_seed(10 * it + ctx.rank)) * 1e-2
        v += step
        ref = exact + (step + torch.randn(50, 5, 4, generator=torch.Generator().manual_seed(10 * it + 1 - ctx.rank)) * 1e-2) / 2
        m.average_delta([v])
        res.append(float((v - ref).abs().max()))
        exact = ref
    return res, float(v.double().sum()), float(x[:, 5:].abs().sum())


def test_mix_average_delta_bf16_wire():
    out = run_world("_avg_delta")
    for r in (0, 1):
        errs, _, _ = out[r]
        assert max(errs) < 2e-4, errs            # bf16 rounding of a ~1e-2 step (2^-9 relative)
    assert out[0][1] == out[1][1]                  # bit-identical replicas
    assert out[0][2] == out[1][2]                  # elements outside the view untouched


def _pipe_bitident(ctx):
    """The bucketed, pipelined shard mean (ModelMixer._pipelined) against the monolithic one
    (PIPE_BUCKET_MB = 0) on the FFM-shaped tensor list: the strided V view of the feature blocks,
    a strided [NF, 4] record view, an odd-length contiguous tensor and a 4-element bias; plain
    average and the bf16-wire average_delta, several mixes each."""
    from hivemall_amd.parallel.mix import ModelMixer

    def model(seed):
        g = torch.Generator().manual_seed(seed)
        blk = torch.randn(331, 7, 6, 4, generator=g)            # [NF][FS][slots..] blocks
        V = blk[:, :5, 1, :]                                     # strided [331, 5, 4]
        rec = torch.randn(331, 12, generator=g)[:, 4:8]          # strided [331, 4]
        odd = torch.randn(1001, generator=g)
        bias = torch.randn(4, generator=g)
        return [V, rec, odd, bias]

    out = {}
    for mb in (0.0, 0.002, 0.0007):
        for delta in (False, True):
            ts = model(7 + ctx.rank)
            m = ModelMixer(ctx)
            m.PIPE_BUCKET_MB = mb
            fn = m.average_delta if delta else m.average
            for it in range(3):
                g = torch.Generator().manual_seed(100 * it + ctx.rank)
                for t in ts:
                    t += torch.randn(t.shape, generator=g) * 1e-2
                fn(ts)
            out[(mb, delta)] = [t.clone() for t in ts]
    res = []
    for delta in (False, True):
        ref = out[(0.0, delta)]
        for mb in (0.002, 0.0007):
            res.append(all(torch.equal(a, b) for a, b in zip(ref, out[(mb, delta)])))
    return res, float(sum(float(t.double().sum()) for t in out[(0.0007, True)]))


@pytest.mark.parametrize("world", [2, 4])
def test_mix_pipelined_buckets_bit_identical_to_monolithic(world):
    out = run_world("_pipe_bitident", world=world)
    for r in range(world):
        assert out[r][0] == [True] * 4, out[r][0]
        assert out[r][1] == out[0][1]                  # every rank bit-identical


def test_bench_seq_reference_is_the_cpu_learner_on_the_same_stream():
    """bench.py's default stream (rows drawn on the CPU) is exactly the one
    benchmarks/ffm_seq_ref.py replays through the sequential engine: on the CPU, where bench.py's
    learner IS that engine, its held-out logloss equals the reference (so a GPU run's
    logloss_gap is the Hogwild / mixing gap alone); and the pinned table answers the driver's
    configuration."""
    sys.path.insert(0, ROOT)
    import bench
    from benchmarks.ffm_seq_ref import load_refs, ref_key, run

    ref = run(gpus=1, steps=2, warmup=1, batch=512, hash_bits=10, factors=4, resident=2, eval_rows=512)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "512",
           "--hash-bits", "10", "--eval-rows", "512", "--device", "cpu", "--resident-batches", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["logloss_heldout"] == pytest.approx(ref["logloss_seq"], abs=2e-5), (d["logloss_heldout"], ref)
    refs = load_refs()
    for n in (1, 2, 4, 8):
        assert ref_key(n, 20, 5, 262144, 20, 4, 8, 262144) in refs
    args = bench.parse_args(["--steps", "20", "--warmup", "5"])
    assert bench.seq_reference(args, 1) == pytest.approx(0.446395, abs=1e-5)
    assert bench.seq_reference(bench.parse_args(["--steps", "20", "--warmup", "5", "--gen-device", "auto"]), 1) is None
