"""Property-based parity tests (hypothesis), SURVEY.md §4.2 item 2: random inputs, native
engines / HIP kernels against plain-Python or PyTorch references of the same operation.

* Murmur3 / mhash: the C++ batch hasher (and the gfx950 kernel, GPU marker) must be bit-exact
  with the pure-Python restatement of MurmurHash3_x86_32 for arbitrary UTF-8 text and seeds.
* FFM feature parsing: the C++ parser against a Python parse of generated ``field:index:value``.
* AUC: the device rank-sum implementation against scikit-learn (ties included).
* Top-k inner-product search: the CPU contract against a brute-force (score desc, index asc)
  ranking, and the gfx950 kernel against the CPU path on integer operands (exact).
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from hivemall_amd.utils.hashing import (mhash, mhash_batch, murmur3_batch,
                                        murmurhash3_x86_32_py, to_signed32)

SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])

words = st.lists(st.text(min_size=0, max_size=40), min_size=1, max_size=50)


@SETTINGS
@given(words, st.integers(min_value=0, max_value=2**32 - 1))
def test_murmur3_native_bit_exact(ws, seed):
    got = murmur3_batch(ws, seed=seed)
    want = [to_signed32(murmurhash3_x86_32_py(w.encode("utf-8"), seed)) for w in ws]
    assert got.tolist() == want


@SETTINGS
@given(words, st.integers(min_value=1, max_value=1 << 24))
def test_mhash_native_matches_python(ws, nf):
    assert mhash_batch(ws, num_features=nf).tolist() == [mhash(w, nf) for w in ws]


@SETTINGS
@given(st.lists(st.tuples(st.integers(0, 38), st.integers(0, 10**6),
                          st.floats(-1e3, 1e3, allow_nan=False, width=32)), min_size=1, max_size=40))
def test_ffm_feature_parser_matches_python(feats):
    from hivemall_amd.utils.features import parse_ffm_rows

    strs = [f"{f}:{i}:{v!r}" for f, i, v in feats]
    csr = parse_ffm_rows([strs], num_features=1 << 20, num_fields=39)
    assert csr.fld.tolist() == [f for f, _, _ in feats]
    assert csr.idx.tolist() == [i % (1 << 20) for _, i, _ in feats]
    np.testing.assert_allclose(csr.val, np.array([v for _, _, v in feats], dtype=np.float32), rtol=1e-6)


@SETTINGS
@given(st.lists(st.tuples(st.integers(-5, 5), st.booleans()), min_size=2, max_size=200))
def test_auc_matches_sklearn(pairs):
    from sklearn.metrics import roc_auc_score

    from hivemall_amd.evaluation.metrics import auc

    s = [float(a) for a, _ in pairs]
    y = [int(b) for _, b in pairs]
    got = auc(s, y)
    if 0 < sum(y) < len(y):
        assert got == pytest.approx(roc_auc_score(y, s), abs=1e-12)
    else:
        assert np.isnan(got)


def _brute_topk(Q, I, k, bias):
    S = Q.double() @ I.double().T + bias.double()[None, :]
    out = []
    for q in range(S.shape[0]):
        order = sorted(range(S.shape[1]), key=lambda n: (-S[q, n].item(), n))[:k]
        out.append(order + [-1] * (k - len(order)))
    return out


mips_shapes = st.tuples(st.integers(1, 70), st.integers(1, 150), st.integers(1, 40),
                        st.integers(1, 64), st.integers(0, 2**31 - 1))


@SETTINGS
@given(mips_shapes)
def test_mips_topk_cpu_contract(shape):
    from hivemall_amd.ops.topk_mips import mips_topk

    M, N, d, k, seed = shape
    g = torch.Generator().manual_seed(seed)
    Q = torch.randint(-2, 3, (M, d), generator=g).float()
    I = torch.randint(-2, 3, (N, d), generator=g).float()
    b = torch.randint(-1, 2, (N,), generator=g).float()
    ix, _ = mips_topk(Q, I, k, item_bias=b)
    assert ix.tolist() == _brute_topk(Q, I, k, b)


@pytest.mark.gpu
@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(mips_shapes)
def test_mips_topk_gpu_equals_cpu(shape):
    from hivemall_amd.ops.topk_mips import mips_topk

    M, N, d, k, seed = shape
    g = torch.Generator().manual_seed(seed)
    Q = torch.randint(-2, 3, (M, d), generator=g).float()
    I = torch.randint(-2, 3, (N, d), generator=g).float()
    b = torch.randint(-1, 2, (N,), generator=g).float()
    ci, cs = mips_topk(Q, I, k, item_bias=b)
    gi, gs = mips_topk(Q.cuda(), I.cuda(), k, item_bias=b.cuda())
    assert torch.equal(gi.cpu(), ci)
    assert torch.equal(gs.cpu(), cs)


@pytest.mark.gpu
@SETTINGS
@given(words, st.integers(min_value=0, max_value=1 << 24))
def test_mhash_kernel_bit_exact(ws, nf):
    from hivemall_amd.utils.hashing import mhash_device

    got = mhash_device(ws, num_features=nf, device="cuda").cpu().tolist()
    want = mhash_batch(ws, num_features=nf).tolist() if nf > 0 else murmur3_batch(ws).tolist()
    assert got == want


@SETTINGS
@given(st.lists(st.integers(-(2**63), 2**63 - 1), max_size=200))
def test_zigzag_leb128_roundtrip(vals):
    from hivemall_amd.utils.codec import zigzag_leb128_decode, zigzag_leb128_encode

    enc = zigzag_leb128_encode(vals)
    assert zigzag_leb128_decode(enc).tolist() == vals
    # small magnitudes of either sign take one byte
    if vals and all(-64 <= v < 64 for v in vals):
        assert len(enc) == len(vals)


@SETTINGS
@given(st.lists(st.integers(0, 2**64 - 1), max_size=200))
def test_vbyte_roundtrip_and_layout(vals):
    from hivemall_amd.utils.codec import vbyte_decode, vbyte_encode

    enc = vbyte_encode(vals)
    assert vbyte_decode(enc).tolist() == vals
    assert len(enc) == sum(max(1, (v.bit_length() + 6) // 7) for v in vals)


def test_vbyte_known_bytes():
    from hivemall_amd.utils.codec import vbyte_encode, zigzag_encode

    assert vbyte_encode([0, 1, 127, 128, 300]) == bytes([0, 1, 0x7F, 0x80, 0x01, 0xAC, 0x02])
    assert [zigzag_encode(v) for v in (0, -1, 1, -2, 2)] == [0, 1, 2, 3, 4]
