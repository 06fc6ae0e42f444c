"""Matrix containers / builders and seeded PRNGs."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from hivemall_amd.utils import prng
from hivemall_amd.utils.matrix import (CSCMatrix, CSRMatrix, DenseMatrix2d, DoKMatrix,
                                       MatrixBuilder)


def test_builder_kinds_agree():
    rows = [["1:0.5", "3:2"], [], ["0", "3:-1", "3:1.5"], [(2, 4.0)]]
    ref = np.array([[0, 0.5, 0, 2], [0, 0, 0, 0], [1, 0, 0, 0.5], [0, 0, 4, 0]], dtype=np.float64)
    for kind in MatrixBuilder.KINDS:
        m = MatrixBuilder(kind).next_rows(rows).build()
        assert m.shape == (4, 4)
        np.testing.assert_allclose(m.to_dense(), ref)
        assert m.get(2, 3) == pytest.approx(0.5) and m.get(1, 1) == 0.0
        cols, vals = m.row(0)
        assert list(map(int, cols)) == [1, 3] and list(vals) == [0.5, 2.0]
        np.testing.assert_allclose(m.matvec(np.arange(4.0)), ref @ np.arange(4.0))
    dense = MatrixBuilder("dense_colmajor").next_rows(rows).build()
    assert isinstance(dense, DenseMatrix2d) and dense.data.flags.f_contiguous
    assert MatrixBuilder("csr", n_cols=10).next_rows(rows).build().shape == (4, 10)
    with pytest.raises(ValueError):
        MatrixBuilder("csr", n_cols=2).next_rows(rows).build()


def test_dense_rows_and_dok_growth():
    m = MatrixBuilder("csr").next_row([0.0, 1.5, 0.0]).next_row(np.array([2.0, 0.0, 0.0])).build()
    np.testing.assert_allclose(m.to_dense(), [[0, 1.5, 0], [2, 0, 0]])
    d = DoKMatrix()
    d.set(3, 5, 1.0)
    d.add(3, 5, 2.0)
    d.set(0, 0, 7.0)
    d.set(0, 0, 0.0)           # zero deletes the key
    assert d.shape == (4, 6) and d.nnz() == 1 and d.get(3, 5) == 3.0


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 12), st.integers(1, 12), st.integers(0, 10_000))
def test_csr_csc_roundtrip(n, m, seed):
    rng = np.random.default_rng(seed)
    a = rng.normal(size=(n, m)) * (rng.random((n, m)) < 0.3)
    csr = CSRMatrix.from_dense(a)
    csc = csr.to_csc()
    assert isinstance(csc, CSCMatrix) and csc.nnz() == np.count_nonzero(a)
    np.testing.assert_allclose(csc.to_dense(), a)
    np.testing.assert_allclose(csc.to_csr().to_dense(), a)
    x = rng.normal(size=m)
    np.testing.assert_allclose(csr.matvec(x), a @ x, atol=1e-12)
    np.testing.assert_allclose(csc.matvec(x), a @ x, atol=1e-12)
    j = int(rng.integers(m))
    rws, vals = csc.column(j)
    np.testing.assert_allclose(vals, a[rws, j])


def test_to_torch_sparse_matches_dense():
    import torch

    a = np.array([[0, 1.0, 0], [2.0, 0, 3.0]])
    t = CSRMatrix.from_dense(a).to_torch()
    assert t.layout == torch.sparse_csr
    np.testing.assert_allclose(t.to_dense().numpy(), a)
    np.testing.assert_allclose(DenseMatrix2d(a, row_major=False).to_torch().numpy(), a)


def test_java_random_bit_exact():
    # values of java.util.Random from the JDK (well-known seeds)
    assert prng.JavaRandom(0).next_int() == -1155484576
    assert prng.JavaRandom(42).next_int() == -1170105035
    assert prng.JavaRandom(0).next_double() == 0.730967787376657
    assert prng.JavaRandom(42).next_double() == 0.7275636800328681
    assert prng.JavaRandom(0).next_gaussian() == 0.8025330637390305
    r = prng.JavaRandom(7)
    r2 = prng.JavaRandom(7)
    assert [r.next_int(10) for _ in range(50)] == [r2.nextInt(10) for _ in range(50)]


def test_java_random_bounded_and_gaussian_stats():
    r = prng.create("java", 123)
    xs = [r.next_int(7) for _ in range(7000)]
    assert min(xs) == 0 and max(xs) == 6
    assert np.bincount(xs).min() > 850
    p2 = [r.next_int(16) for _ in range(2000)]
    assert 0 <= min(p2) and max(p2) == 15
    g = np.array([r.next_gaussian() for _ in range(20000)])
    assert abs(g.mean()) < 0.03 and abs(g.std() - 1) < 0.03
    assert -(1 << 63) <= r.next_long() < (1 << 63)
    assert 0.0 <= r.next_float() < 1.0


def test_prng_factory_kinds():
    for kind in ("java", "smile", "commons"):
        a, b = prng.create(kind, 5), prng.create(kind, 5)
        assert [a.next_double() for _ in range(5)] == [b.next_double() for _ in range(5)]
        assert 0 <= a.next_int(3) < 3
    assert isinstance(prng.create("smile", 1), prng.SmileRandom)
    with pytest.raises(ValueError):
        prng.create("xorshift", 1)
