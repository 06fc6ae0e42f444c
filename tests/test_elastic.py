"""Checkpoint/resume round trips and fault injection + resume."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from hivemall_amd.io import checkpoint
from hivemall_amd.io.synthetic import a9a_like, criteo_like

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_checkpoint_roundtrip_linear(tmp_path):
    from hivemall_amd.models.linear import TrainAROW
    rows, y = a9a_like(2000)
    srows = [[f"f{int(i)}" for i in r] for r in rows]
    a = TrainAROW("-replicas 2 -iters 1", device="cpu").fit(srows, y)
    checkpoint.save(a, str(tmp_path / "ck"))
    b = checkpoint.load(str(tmp_path / "ck"), device="cpu")
    assert torch.equal(a.state.S, b.state.S)
    a.fit(srows, y)
    b.fit(srows, y)
    assert torch.equal(a.weights()[0], b.weights()[0])
    assert a.model_table().equals(b.model_table())
    assert os.path.exists(tmp_path / "ck" / "model.parquet")


def test_checkpoint_roundtrip_ffm_and_fm(tmp_path):
    from hivemall_amd.models.ffm import FFMBatch, FFMTrainer
    from hivemall_amd.models.fm import FMTrainer
    idx, y = criteo_like(3000, 12, seed=1)
    a = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 12", device="cpu")
    a.fit(batch=FFMBatch(idx, None, None, y))
    checkpoint.save(a, str(tmp_path / "ffm"))
    b = checkpoint.load(str(tmp_path / "ffm"), device="cpu")
    for k in a.state:
        assert torch.equal(a.state[k], b.state[k]), k
    rows = [[f"{int(i) + 1}:1" for i in r[:5]] for r in idx[:500].numpy()]
    f = FMTrainer("-factors 3 -iters 2", device="cpu").fit(rows, y[:500].numpy())
    checkpoint.save(f, str(tmp_path / "fm"))
    g = checkpoint.load(str(tmp_path / "fm"), device="cpu")
    np.testing.assert_array_equal(f.predict(rows[:20]), g.predict(rows[:20]))


@pytest.mark.gpu
def test_checkpoint_roundtrip_gpu_record_layouts(tmp_path):
    """GPU state in the record layouts (FFM: {w, z, n} inside each fp32 feature block; FM with
    HM_FM_W_RECORD: w inside each V row) saves and loads as the same views of one table, predicts
    identically, and keeps training (the kernels take whatever strides the loaded tensors have)."""
    from hivemall_amd.io.synthetic import criteo_ffm
    from hivemall_amd.models.ffm import FFMBatch, FFMTrainer
    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.models.linear import SparseRows
    from hivemall_amd.ops import fm as fm_ops

    idx, fld, val, y = criteo_ffm(20000, 14, seed=1)
    b = FFMBatch(idx, fld, val, y).to("cuda")
    ev = FFMBatch(idx[:2000], fld[:2000], val[:2000], None).to("cuda")
    a = FFMTrainer("-classification -factors 4 -num_fields 39 -feature_hashing 14 -seed 3", device="cuda")
    a.fit(batch=b)
    assert a.state["w"].stride(0) > 1                        # the records are in use
    checkpoint.save(a, str(tmp_path / "ffm"))
    c = checkpoint.load(str(tmp_path / "ffm"), device="cuda")
    # back in the pipelined kernels' layout: feature blocks with the linear records inside
    assert c.state["w"].stride(0) == a.state["w"].stride(0) and c.state["V"].stride() == a.state["V"].stride()
    for k in ("V", "G", "w", "wz", "wn", "bias"):
        assert torch.equal(a.state[k], c.state[k]), k
    assert torch.equal(a.predict_raw(batch=ev), c.predict_raw(batch=ev))
    c.fit(batch=b)                                          # trains on the loaded views
    assert torch.isfinite(c.predict_raw(batch=ev)).all()

    old = fm_ops.W_RECORD
    fm_ops.W_RECORD = True
    try:
        cidx, cy = criteo_like(20000, 14, seed=2)
        rows = SparseRows(torch.arange(0, 20000 * 39 + 1, 39, dtype=torch.int64), cidx.reshape(-1).contiguous(),
                          None, cy).to("cuda")
        f = FMTrainer("-c -factors 8 -num_features 16384 -seed 3", device="cuda").fit(rows=rows)
        assert f.state["w"].stride(0) > 1
        checkpoint.save(f, str(tmp_path / "fm"))
        g = checkpoint.load(str(tmp_path / "fm"), device="cuda")
        assert g.state["w"].stride(0) == f.state["w"].stride(0) > 1
        assert torch.equal(f.state["w"], g.state["w"]) and torch.equal(f.state["V"], g.state["V"])
        assert torch.equal(f.predict_raw(rows=rows), g.predict_raw(rows=rows))
        g.fit(rows=rows)
        assert torch.isfinite(g.predict_raw(rows=rows)).all()
    finally:
        fm_ops.W_RECORD = old


def _run_job(ckpt, fault=None, world=2, steps=6):
    env = dict(os.environ, PYTHONPATH=ROOT, HM_CKPT=str(ckpt), HM_STEPS=str(steps),
               MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("HM_FAULT", None)
    if fault:
        env["HM_FAULT"] = fault
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000 + (7 if fault else 0)),
           os.path.join(ROOT, "tests", "elastic_job.py")]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)


def test_fault_injection_and_resume(tmp_path):
    ref = _run_job(tmp_path / "ref")
    assert ref.returncode == 0, ref.stderr[-2000:]
    crashed = _run_job(tmp_path / "job", fault="1:3")
    assert crashed.returncode != 0
    resumed = _run_job(tmp_path / "job")
    assert resumed.returncode == 0, resumed.stderr[-2000:]
    a = torch.load(tmp_path / "ref" / "final_rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "job" / "final_rank0.pt", weights_only=True)
    assert torch.equal(a, b)


def test_checkpoint_save_replaces_atomically_and_keeps_rng(tmp_path):
    import torch

    from hivemall_amd.io import checkpoint
    from hivemall_amd.models.linear import TrainClassifier
    from hivemall_amd.io.synthetic import a9a_like
    rows, y = a9a_like(500)
    m = TrainClassifier("-loss logloss", device="cpu").fit(rows, y)
    p = str(tmp_path / "ck")
    checkpoint.save(m, p)
    checkpoint.save(m, p)                       # overwrite: old renamed aside, then removed
    assert sorted(os.listdir(tmp_path)) == ["ck"]
    torch.manual_seed(123)
    before = torch.get_rng_state()
    checkpoint.load(p, device="cpu")
    assert torch.equal(torch.get_rng_state(), before)   # load does not reseed the caller
    # a crash between the renames leaves only <path>.old-*: load() falls back to it
    os.replace(p, p + ".old-x1")
    b = checkpoint.load(p, device="cpu")
    assert torch.equal(b.weights()[0], m.weights()[0])


def test_checkpoint_old_fallback_takes_newest_and_save_cleans_stale(tmp_path):
    """The .old-* fallback is ordered by the save time in meta.json, not by the random mkdtemp
    suffix, and a successful save() removes .old-* directories left by earlier crashes."""
    import json

    import torch

    from hivemall_amd.io import checkpoint
    from hivemall_amd.models.linear import TrainClassifier
    from hivemall_amd.io.synthetic import a9a_like
    rows, y = a9a_like(300)
    m1 = TrainClassifier("-loss logloss -iters 1", device="cpu").fit(rows, y)
    m2 = TrainClassifier("-loss logloss -iters 3", device="cpu").fit(rows, y)
    p = str(tmp_path / "ck")
    checkpoint.save(m1, str(tmp_path / "a"))
    checkpoint.save(m2, str(tmp_path / "b"))
    os.replace(tmp_path / "b", p + ".old-aaaa")   # newer save, lexically FIRST suffix
    os.replace(tmp_path / "a", p + ".old-zzzz")   # older save, lexically last suffix
    # make the older one really older by its recorded time
    meta = json.load(open(p + ".old-zzzz/meta.json"))
    meta["saved_ns"] = 1
    json.dump(meta, open(p + ".old-zzzz/meta.json", "w"))
    b = checkpoint.load(p, device="cpu")
    assert torch.equal(b.weights()[0], m2.weights()[0])
    checkpoint.save(m1, p)
    assert sorted(os.listdir(tmp_path)) == ["ck"]


@pytest.mark.parametrize("kind", ["ffm", "linear", "mf", "fm"])
def test_learner_checkpoint_option_resumes_bit_identically(kind, tmp_path, monkeypatch):
    """``-checkpoint <dir>``: a learner's epoch loop saves after every epoch; a run killed
    before epoch 2 (HM_FAULT=0:2:raise) and rerun with the same query resumes after epoch 1 and
    ends bit-identical to an uninterrupted run."""
    import numpy as np

    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models import linear as L
    from hivemall_amd.models.ffm import FFMBatch, FFMTrainer
    from hivemall_amd.models.fm import FMTrainer
    from hivemall_amd.models.mf import MatrixFactorization
    from hivemall_amd.parallel.elastic import InjectedFault

    rng = np.random.default_rng(0)
    idx, y = criteo_like(600, 10, seed=4)
    u, it, r = rng.integers(0, 40, 500), rng.integers(0, 60, 500), rng.random(500) * 5
    feats = [[f"{j}:1.0" for j in rng.choice(300, 6, replace=False)] for _ in range(300)]
    fy = rng.integers(0, 2, 300)

    def run(opts):
        if kind == "ffm":
            t = FFMTrainer("-c -factors 4 -num_fields 39 -feature_hashing 10 -iters 4 -disable_cv "
                           "-seed 3" + opts, device="cpu")
            t.fit(batch=FFMBatch(idx, None, None, y))
            return t.state["V"].clone()
        if kind == "linear":
            t = L.TrainClassifier("-loss logloss -opt adagrad -dims 1024 -iters 4 -disable_cv" + opts,
                                  device="cpu")
            t.fit(rows=L.SparseRows(torch.arange(0, 600 * 39 + 1, 39, dtype=torch.int64),
                                    idx.reshape(-1).contiguous(), None, y))
            return t.state.S.clone()
        if kind == "mf":
            t = MatrixFactorization("-factors 4 -iters 4 -disable_cv -seed 3" + opts, device="cpu")
            t.fit(u, it, r)
            return t.state["P"].clone()
        t = FMTrainer("-c -factors 4 -iters 4 -disable_cv -num_features 301 -seed 3" + opts, device="cpu")
        t.fit(feats, fy)
        return t.state["V"].clone()

    ref = run("")
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("HM_FAULT", "0:2:raise")
    with pytest.raises(InjectedFault):
        run(f" -checkpoint {ck}")
    assert (tmp_path / "ck" / "rank0" / "latest.json").exists()
    # a fault armed at epoch 0 cannot fire on the rerun: it starts after the saved epoch 1
    monkeypatch.setenv("HM_FAULT", "0:0:raise")
    got = run(f" -checkpoint {ck}")
    assert torch.equal(got, ref)


def test_checkpoint_of_another_run_is_not_resumed(tmp_path, monkeypatch):
    """A -checkpoint directory written by a different run (other rows, other options) is never
    resumed: the learner starts fresh (a finished run's checkpoint used to be returned
    as the new query's model)."""
    from hivemall_amd.io.synthetic import criteo_like
    from hivemall_amd.models.ffm import FFMBatch, FFMTrainer

    ck = str(tmp_path / "ck")
    base = "-c -factors 4 -num_fields 39 -feature_hashing 10 -iters 3 -disable_cv -seed 3"

    def run(seed, opts=""):
        idx, y = criteo_like(400, 10, seed=seed)
        t = FFMTrainer(base + opts + f" -checkpoint {ck}", device="cpu")
        t.fit(batch=FFMBatch(idx, None, None, y))
        return t

    first = run(4)
    assert first.cv.epoch == 3
    # same options, different rows: trains all 3 epochs from scratch, equal to a clean run
    other = run(5)
    idx, y = criteo_like(400, 10, seed=5)
    clean = FFMTrainer(base, device="cpu")
    clean.fit(batch=FFMBatch(idx, None, None, y))
    assert other.cv.epoch == 3 and torch.equal(other.state["V"], clean.state["V"])
    # same rows, different options (-iters 5): not resumed either
    again = run(5, " -eta0 0.1")
    assert again.cv.epoch == 3 and not torch.equal(again.state["V"], clean.state["V"])
