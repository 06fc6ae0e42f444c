"""Host collections (C11), HalfFloat codec (C14)."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from hivemall_amd.utils.collections import (BoundedPriorityQueue, Int2FloatOpenHashTable,
                                            Int2LongOpenHashTable, float_to_half_bits,
                                            half_bits_to_float, is_representable_as_half)


def test_bounded_priority_queue_keeps_top():
    q = BoundedPriorityQueue(3)
    kept = [q.offer(x) for x in [5, 1, 9, 3, 7, 2]]
    assert kept == [True, True, True, True, True, False]
    assert q.sorted() == [9, 7, 5]
    assert q.peek() == 5 and len(q) == 3
    q2 = BoundedPriorityQueue(2, key=lambda t: t[0])
    for t in [(1, "a"), (3, "b"), (2, "c")]:
        q2.offer(t)
    assert [t[1] for t in q2.sorted()] == ["b", "c"]


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.integers(-2**40, 2**40), st.floats(-1e6, 1e6, width=32)),
                max_size=300))
def test_open_hash_table_matches_dict(pairs):
    t = Int2FloatOpenHashTable(4)
    ref = {}
    half = len(pairs) // 2
    for k, v in pairs[:half]:
        t.put(k, v)
        ref[k] = np.float32(v)
    if pairs[half:]:
        ks = np.array([k for k, _ in pairs[half:]], dtype=np.int64)
        vs = np.array([v for _, v in pairs[half:]], dtype=np.float32)
        t.put_many(ks, vs)
        for k, v in zip(ks, vs):      # last write wins
            ref[int(k)] = v
    assert len(t) == len(ref)
    for k, v in ref.items():
        assert t.get(k) == v and k in t
    probe = np.array(list(ref) + [2**50, -(2**50)], dtype=np.int64)
    got = t.get_many(probe, default=-1.0)
    assert np.array_equal(got[:-2], np.array([ref[int(k)] for k in probe[:-2]], np.float32))
    assert (got[-2:] == -1.0).all()
    ks, _ = t.to_arrays()
    assert sorted(ref) == ks.tolist()


def test_int2long_table_offsets():
    t = Int2LongOpenHashTable()
    keys = np.arange(0, 5000, 3, dtype=np.int64)
    t.put_many(keys, keys * 16)
    assert t.get_many(keys).tolist() == (keys * 16).tolist()
    assert t.get(1, -1) == -1


def test_half_float_codec():
    x = np.array([0.0, -0.0, 1.0, -2.5, 65504.0, 1e-7, 3.14159, np.inf, np.nan], np.float32)
    h = float_to_half_bits(x)
    assert h[2] == 0x3C00 and h[3] == 0xC100 and h[4] == 0x7BFF and h[7] == 0x7C00
    back = half_bits_to_float(h)
    assert np.allclose(back[:7], x[:7], rtol=1e-3, atol=1e-7) and np.isnan(back[8])
    # truncation never rounds up in magnitude and agrees on exactly representable values
    r = np.random.default_rng(0).normal(size=1000).astype(np.float32) * 100
    tr = half_bits_to_float(float_to_half_bits(r, "truncate"))
    assert (np.abs(tr) <= np.abs(r)).all()
    assert np.array_equal(float_to_half_bits(back[:7], "truncate"), h[:7])
    assert is_representable_as_half(65504.0) and not is_representable_as_half(70000.0)


def test_function_catalogue_covers_registry():
    """docs/funcs.md analogue (upstream hivemall-docs): every registered name is described."""
    from hivemall_amd import registry
    from hivemall_amd.ddl import function_catalogue

    text = function_catalogue()
    registry.load_all()
    for name in registry.names():
        assert f"| `{name}`" in text
    assert "(see hivemall" not in text


def test_checked_in_catalogue_and_ddl_are_current():
    """docs/funcs.md and resources/ddl/define-all.hive are regenerated whenever a function or its
    description changes (``python -m hivemall_amd.ddl --funcs docs/funcs.md``;
    ``python -m hivemall_amd.ddl resources/ddl``)."""
    import os

    from hivemall_amd.ddl import define_all, function_catalogue

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "docs", "funcs.md")) as f:
        assert f.read() == function_catalogue()
    with open(os.path.join(root, "resources", "ddl", "define-all.hive")) as f:
        assert f.read() == define_all()
