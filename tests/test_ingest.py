"""Device-side ingest (io/ingest.py, csrc/kernels/ingest.hip): Arrow list<string> feature columns
-> pinned double-buffered H2D -> parse/mhash kernels.  The host parser (csrc/host/hashing.cpp)
is the oracle: the device output must be bit-identical, chunk boundaries included, and strings
the device refuses must fall back to the host (which raises its usual error)."""
import random

import numpy as np
import pyarrow as pa
import pytest
import torch

from hivemall_amd.io import ingest
from hivemall_amd.utils.features import FeatureEncoder, parse_ffm_rows
from hivemall_amd.utils.options import UDFArgumentException


def _ffm_rows(n, seed=0, odd=True):
    rnd = random.Random(seed)
    vals = ["1", "0.5", "0.25", "3.0e-2", "-7", "1E3", ".5", "12345.678", "0.1", "2.5e+1"]
    if odd:   # values outside the device's exact decimal fast path -> host fallback
        vals += ["1e-300", "0.1234567890123456789012"]
    rows = []
    for _ in range(n):
        k = rnd.randint(0, 12)
        r = []
        for _ in range(k):
            f = rnd.choice([str(rnd.randint(0, 38)), "cat%d" % rnd.randint(0, 9)])
            i = rnd.choice([str(rnd.randint(0, 1 << 20)), "tok_%x" % rnd.getrandbits(24)])
            r.append(f"{f}:{i}" if rnd.random() < 0.3 else f"{f}:{i}:{rnd.choice(vals)}")
        rows.append(r)
    return rows


def _host_ell(rows, nf, nfld, hash_ints, F):
    csr = parse_ffm_rows(rows, nf, nfld, hash_ints=hash_ints)
    return csr.to_ell(F)


def test_arrow_buffers_honour_slices():
    arr = ingest.to_arrow_lists([["a:1", "bb"], [], ["ccc:2.5"], ["d"]])
    data, so, lo = ingest.arrow_buffers(arr.slice(1, 3))
    assert data.tobytes() == b"ccc:2.5d"
    assert so.tolist() == [0, 7, 8]
    assert lo.tolist() == [0, 0, 1, 2]


def test_to_arrow_lists_accepts_series_and_lists():
    import pandas as pd

    s = pd.Series([["1:2"], ["3:4", "5:6"]], dtype=pd.ArrowDtype(pa.list_(pa.string())))
    assert ingest.is_arrow_like(s)
    assert ingest.to_arrow_lists(s).to_pylist() == [["1:2"], ["3:4", "5:6"]]
    _, _, lo = ingest.arrow_buffers(ingest.to_arrow_lists([["1:2"], None]))
    assert lo.tolist() == [0, 1, 1]      # a NULL row is an empty row


@pytest.mark.parametrize("hash_ints", [False, True])
def test_ffm_ingest_host_path_equals_parser(hash_ints):
    rows = _ffm_rows(300, seed=1)
    nf = 1 << 21 if not hash_ints else 1 << 12
    idx, fld, val, st = ingest.ffm_ell_device(rows, nf, 39, hash_ints, device="cpu", chunk_rows=64)
    F = idx.shape[1]
    i, v, f = _host_ell(rows, nf, 39, hash_ints, F)
    np.testing.assert_array_equal(idx.numpy(), i)
    np.testing.assert_array_equal(fld.numpy(), f)
    np.testing.assert_array_equal(val.numpy(), v)
    assert st.rows == 300 and st.host_fallback_chunks == 5


def test_csr_ingest_host_path_equals_encoder():
    rows = [["a:2", "b"], [], ["c:0.5", "a"]]
    ip, idx, val, _ = ingest.csr_device(rows, "hash", 1 << 10, device="cpu", chunk_rows=2)
    ref = FeatureEncoder("hash", num_features=1 << 10).encode(rows)
    assert ip.tolist() == ref.indptr.tolist()
    assert idx.tolist() == ref.idx.tolist()
    np.testing.assert_array_equal(val.numpy(), ref.val)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("hash_ints,odd,chunk", [(False, False, 1 << 20), (True, False, 97),
                                                 (False, True, 128)])
def test_ffm_ingest_device_equals_host(hash_ints, odd, chunk):
    rows = _ffm_rows(2000, seed=2, odd=odd)
    nf = 1 << 21 if not hash_ints else 1 << 14
    idx, fld, val, st = ingest.ffm_ell_device(rows, nf, 39, hash_ints, device="cuda", chunk_rows=chunk)
    F = idx.shape[1]
    i, v, f = _host_ell(rows, nf, 39, hash_ints, F)
    np.testing.assert_array_equal(idx.cpu().numpy(), i)
    np.testing.assert_array_equal(fld.cpu().numpy(), f)
    np.testing.assert_array_equal(val.cpu().numpy(), v)
    assert st.chunks == (2000 + chunk - 1) // chunk
    if not odd:
        assert st.host_fallback_chunks == 0, st.refused     # everything parsed by the kernel
    else:
        assert 0 < st.host_fallback_chunks <= st.chunks


@pytest.mark.gpu
def test_ffm_ingest_device_malformed_raises_host_error():
    rows = [["1:2:0.5"], ["nocolon"], ["3:4"]]
    with pytest.raises(UDFArgumentException, match="nocolon"):
        ingest.ffm_ell_device(rows, 1 << 10, 8, True, device="cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["hash", "int"])
def test_csr_ingest_device_equals_encoder(mode):
    rnd = random.Random(3)
    if mode == "hash":
        rows = [[f"f{rnd.randint(0, 5000)}" + (f":{rnd.choice(['0.5', '2', '1e-2'])}" if rnd.random() < .5 else "")
                 for _ in range(rnd.randint(0, 20))] for _ in range(3000)]
    else:
        rows = [[f"{rnd.randint(0, 1 << 30)}:{rnd.choice(['0.5', '2', '-3.25'])}"
                 for _ in range(rnd.randint(0, 20))] for _ in range(3000)]
    ip, idx, val, st = ingest.csr_device(rows, mode, 1 << 18, device="cuda", chunk_rows=1000)
    ref = FeatureEncoder(mode, num_features=1 << 18).encode(rows)
    assert ip.cpu().tolist() == ref.indptr.tolist()
    assert idx.cpu().tolist() == ref.idx.tolist()
    np.testing.assert_array_equal(val.cpu().numpy(), ref.val)
    assert st.chunks == 3 and st.host_fallback_chunks == 0, st.refused


@pytest.mark.gpu
def test_train_ffm_sql_udtf_ingests_on_device():
    """train_ffm over string rows on the GPU goes through the device parser, and the model it
    trains equals the one trained from host-parsed batches."""
    from hivemall_amd.models.ffm import FFMTrainer

    rows = _ffm_rows(4000, seed=4, odd=False)
    y = [1 if random.Random(i).random() < 0.3 else 0 for i in range(4000)]
    opts = "-c -feature_hashing 16 -num_fields 39 -iters 1 -disable_cv -seed 7"
    a = FFMTrainer(opts, device="cuda")
    ba = a.prepare(rows, y)
    assert ingest.LAST_STATS.chunks >= 1 and ingest.LAST_STATS.host_fallback_chunks == 0
    import os

    os.environ["HM_INGEST_HOST"] = "1"
    try:
        b = FFMTrainer(opts, device="cuda")
        bb = b.prepare(rows, y)
    finally:
        os.environ.pop("HM_INGEST_HOST")
    for x, z in ((ba.idx, bb.idx), (ba.fld, bb.fld), (ba.val, bb.val), (ba.y, bb.y)):
        assert torch.equal(x.cpu(), z.cpu())


@pytest.mark.gpu
def test_linear_learner_ingests_integer_features_on_device():
    """train_classifier over "idx:value" strings: the GPU path parses them on the device and
    trains the same model as host-parsed rows; non-integer names fall back to the host
    dictionary encoder."""
    from hivemall_amd.models.linear import TrainClassifier

    rnd = random.Random(7)
    rows = [[f"{rnd.randint(1, 500)}:{rnd.choice(['0.5', '1', '2.25'])}" for _ in range(12)] + ["0:1.0"]
            for _ in range(3000)]
    y = [rnd.randint(0, 1) for _ in range(3000)]
    a = TrainClassifier("-loss logloss -replicas 4", device="cuda")
    ra = a.prepare(rows, y)
    assert ingest.LAST_STATS.chunks >= 1 and ingest.LAST_STATS.host_fallback_chunks == 0
    b = TrainClassifier("-loss logloss -replicas 4", device="cpu")
    rb = b.prepare(rows, y)
    assert torch.equal(ra.indptr.cpu(), rb.indptr) and torch.equal(ra.idx.cpu(), rb.idx)
    assert torch.equal(ra.val.cpu(), rb.val) and torch.equal(ra.y.cpu(), rb.y)
    a.fit(rows=ra)
    tab = a.model_table()
    assert tab["feature"].map(type).eq(str).all()          # string names stay strings
    c = TrainClassifier("-loss logloss", device="cuda")
    rc = c.prepare([["a:1", "b:2"], ["c"]], [1, 0])          # dictionary names: host encoder
    assert c.encoder.mode == "dict" and rc.n == 2
