"""Feature engineering functions (upstream core/src/main/java/hivemall/ftvec/
{AddBiasUDF,AddFeatureIndexUDF,ExtractFeatureUDF,ExtractWeightUDF,FeatureUDF,FeatureIndexUDF,
SortByFeatureUDF}, ftvec/hashing/*, ftvec/scaling/*, ftvec/amplify/*, ftvec/conv/*,
ftvec/binning/*, ftvec/pairing/*, ftvec/ranking/*, ftvec/selection/*, ftvec/text/*,
ftvec/trans/*).

Feature grammar: ``"name:value"`` (split at the last ``:`` for FFM-style strings is NOT done;
the value is everything after the FIRST ``:`` unless the string has two ``:`` in which case it
is ``field:index:value``), bare ``"name"`` = value 1.0.  Index 0 is reserved for the bias.
"""
from __future__ import annotations

import hashlib
import math
from collections import Counter, defaultdict
from typing import Iterable, Sequence

import numpy as np

from ..registry import udaf, udf, udtf
from ..utils.hashing import DEFAULT_SEED, mhash as _mhash, murmurhash3
from ..utils.options import Options, UDFArgumentException, flag, opt


def _split(f) -> tuple[str, float]:
    s = str(f)
    p = s.find(":")
    if p < 0:
        return s, 1.0
    q = s.find(":", p + 1)
    if q >= 0:  # field:index:value
        return s[:q], float(s[q + 1:])
    return s[:p], float(s[p + 1:])


def _fmt(v: float) -> str:
    v = float(v)
    return repr(v) if v != int(v) or abs(v) > 1e15 else f"{v:.1f}"


# ------------------------------------------------------------------ vectorised column paths
# The SQL executor hands vectorised UDFs whole columns.  A column of feature lists becomes one
# Arrow list<string> array (zero-copy when the table is Arrow-backed) whose flat string buffer
# is processed by the native host library in one call; the result is an Arrow-backed Series, so
# a learner downstream parses it from the buffers again without any Python object per feature.

def _list_column(col):
    """Arrow list<string> array of a Series of feature lists, or None (mixed / non-string
    content: the per-row path handles it)."""
    import pandas as pd
    import pyarrow as pa

    if not isinstance(col, pd.Series):
        return None
    if isinstance(col.dtype, pd.ArrowDtype):
        a = col.array._pa_array
        if isinstance(a, pa.ChunkedArray):      # one chunk: its array as is (combine_chunks copies)
            a = a.chunk(0) if a.num_chunks == 1 else a.combine_chunks()
        if (pa.types.is_list(a.type) or pa.types.is_large_list(a.type)) and \
                (pa.types.is_string(a.type.value_type) or pa.types.is_large_string(a.type.value_type)):
            return a
        return None
    vals = col.to_numpy(dtype=object)
    for r in vals[:64]:
        if r is not None and not (isinstance(r, (list, tuple, np.ndarray)) and all(isinstance(v, str) for v in r)):
            return None
    try:
        return pa.array([None if r is None else list(r) for r in vals], type=pa.list_(pa.string()))
    except (pa.ArrowInvalid, pa.ArrowTypeError):
        return None


def _arrow_series(arr, index):
    import pandas as pd

    return pd.Series(pd.arrays.ArrowExtensionArray(arr), index=index)


def _hash_list_column(arr, num_features: int):
    """feature_hashing over every string of a list<string> array (hm_feature_hash_strs)."""
    import pyarrow as pa

    from .. import _native
    from ..io.ingest import arrow_buffers

    data, so, lo = arrow_buffers(arr)
    n = len(so) - 1
    out = np.empty(max(1, int(so[-1]) + 11 * n), dtype=np.uint8)
    oo = np.empty(n + 1, dtype=np.int64)
    if n:
        d = data if len(data) else np.zeros(1, np.uint8)
        tot = _native.host().hm_feature_hash_strs(d.ctypes.data, np.ascontiguousarray(so).ctypes.data, n,
                                                  int(num_features), DEFAULT_SEED, out.ctypes.data,
                                                  oo.ctypes.data)
    else:
        oo[0], tot = 0, 0
    vals = pa.LargeStringArray.from_buffers(n, pa.py_buffer(oo), pa.py_buffer(out[:max(1, tot)]))
    return pa.LargeListArray.from_arrays(pa.array(lo, pa.int64()), vals.cast(pa.string()),
                                         mask=arr.is_null())


def _append_const(arr, const: str):
    """list<string> rows with ``const`` appended to every non-null row (nulls stay null):
    one native pass over the string buffer (hm_list_append_str)."""
    import pyarrow as pa

    from .. import _native
    from ..io.ingest import arrow_buffers

    data, so, lo = arrow_buffers(arr)
    n = len(arr)
    valid = None
    if arr.null_count:
        valid = np.ascontiguousarray(~np.asarray(arr.is_null().to_numpy(zero_copy_only=False), dtype=bool),
                                     dtype=np.uint8)
    c = np.frombuffer(const.encode("utf-8"), dtype=np.uint8)
    nrows_valid = n if valid is None else int(valid.sum())
    out = np.empty(max(1, len(data) + len(c) * n), dtype=np.uint8)
    oo = np.empty(int(lo[-1]) + nrows_valid + 1, dtype=np.int64)
    orow = np.empty(n + 1, dtype=np.int64)
    d = data if len(data) else np.zeros(1, np.uint8)
    so = np.ascontiguousarray(so, dtype=np.int64)
    lo = np.ascontiguousarray(lo, dtype=np.int64)
    tot = _native.host().hm_list_append_str(d.ctypes.data, so.ctypes.data, lo.ctypes.data,
                                            None if valid is None else valid.ctypes.data, n, c.ctypes.data,
                                            len(c), out.ctypes.data, oo.ctypes.data, orow.ctypes.data)
    vals = pa.LargeStringArray.from_buffers(len(oo) - 1, pa.py_buffer(oo), pa.py_buffer(out[:max(1, tot)]))
    return pa.LargeListArray.from_arrays(pa.array(orow, pa.int64()), vals.cast(pa.string()),
                                         mask=arr.is_null())


# ------------------------------------------------------------------ basic
def _add_bias1(features):
    if features is None:
        return None
    fs = list(features)
    if fs and isinstance(fs[0], (int, np.integer)):
        return fs + [0]
    return fs + ["0:1.0"]


@udf("add_bias", vectorized=True)
def add_bias(features):
    """Append the bias feature ``0:1.0`` (index 0 is reserved for the bias)."""
    import pandas as pd

    if isinstance(features, pd.Series):
        arr = _list_column(features)
        if arr is None:
            return _rowwise(_add_bias1, features)
        return _arrow_series(_append_const(arr, "0:1.0"), features.index)
    return _add_bias1(features)


def _add_feature_index1(values):
    if values is None:
        return None
    return [f"{i + 1}:{_fmt(v)}" for i, v in enumerate(values) if v is not None]


def _numeric_list_column(col):
    """Arrow list<double> array of a Series of numeric lists, or None (strings, bools, mixed
    content: the per-row path handles those)."""
    import pandas as pd
    import pyarrow as pa

    if isinstance(col.dtype, pd.ArrowDtype):
        a = col.array._pa_array
        if isinstance(a, pa.ChunkedArray):      # one chunk: its array as is (combine_chunks copies)
            a = a.chunk(0) if a.num_chunks == 1 else a.combine_chunks()
        if not (pa.types.is_list(a.type) or pa.types.is_large_list(a.type)):
            return None
        vt = a.type.value_type
        if not (pa.types.is_integer(vt) or pa.types.is_floating(vt)):
            return None
        return a.cast(pa.large_list(pa.float64()))
    vals = col.to_numpy(dtype=object)
    for r in vals[:64]:
        if r is not None and not (isinstance(r, (list, tuple, np.ndarray)) and all(
                v is None or (isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool))
                for v in r)):
            return None
    try:
        return pa.array([None if r is None else list(r) for r in vals], type=pa.large_list(pa.float64()))
    except (pa.ArrowInvalid, pa.ArrowTypeError, OverflowError):
        return None


@udf("add_feature_index", vectorized=True)
def add_feature_index(values):
    """[v1, v2, ...] -> ["1:v1", "2:v2", ...]"""
    import pandas as pd

    if not isinstance(values, pd.Series):
        return _add_feature_index1(values)
    arr = _numeric_list_column(values)
    if arr is None:
        return _rowwise(_add_feature_index1, values)
    import pyarrow as pa

    from .. import _native

    n = len(arr)
    lo = np.array(arr.offsets, dtype=np.int64)
    flat = arr.values.slice(int(lo[0]), int(lo[-1] - lo[0]))
    v = np.ascontiguousarray(flat.to_numpy(zero_copy_only=False), dtype=np.float64)
    valid = None
    if flat.null_count:
        valid = np.ascontiguousarray(flat.is_valid().to_numpy(zero_copy_only=False), dtype=np.uint8)
        v = np.where(valid.astype(bool), v, 0.0)
    nv = len(v)
    oo = np.empty(nv + 1, dtype=np.int64)
    lib = _native.host()
    vp = (v if nv else np.zeros(1)).ctypes.data
    tot = lib.hm_format_feature_index(vp, None if valid is None else valid.ctypes.data, lo.ctypes.data, n,
                                      None, oo.ctypes.data)
    if tot < -1:                       # a non-finite value: the per-row path raises as before
        return _rowwise(_add_feature_index1, values)
    out = np.empty(max(1, int(tot)), dtype=np.uint8)
    lib.hm_format_feature_index(vp, None if valid is None else valid.ctypes.data, lo.ctypes.data, n,
                                out.ctypes.data, oo.ctypes.data)
    strs = pa.LargeStringArray.from_buffers(nv, pa.py_buffer(oo), pa.py_buffer(out))
    if valid is not None:              # null values are skipped, their positions kept
        keep = pa.array(valid.astype(bool))
        strs = strs.filter(keep)
        cnt = np.concatenate([[0], np.cumsum(valid, dtype=np.int64)])
        lo = cnt[lo - lo[0]]
    else:
        lo = lo - lo[0]
    res = pa.LargeListArray.from_arrays(pa.array(lo, pa.int64()), strs.cast(pa.string()), mask=arr.is_null())
    return _arrow_series(res, values.index)


_FV_RE = r"^([^:]*:[^:]*|[^:]*):(.*)$"     # _split: value after the 2nd ':' when there is one


def _vec_split(col):
    """Vectorised _split over a Series of feature strings (Arrow compute, C++ regex): (names
    Series, values Series), or None when the column holds anything but strings (the per-row
    path handles those)."""
    import pandas as pd
    import pyarrow as pa
    import pyarrow.compute as pc

    try:
        arr = pa.array(col.to_numpy(dtype=object), type=pa.string(), from_pandas=True)
    except (pa.ArrowInvalid, pa.ArrowTypeError):
        return None
    sp = pc.split_pattern(arr, ":", max_splits=2)          # <=3 parts: name | f:i | value
    lens = pc.fill_null(pc.list_value_length(sp), 0).to_numpy()
    offs = sp.offsets.to_numpy()[:-1].astype(np.int64)
    flat = pc.list_flatten(sp)
    last = max(len(flat) - 1, 0)

    def part(j):
        return flat.take(pa.array(np.minimum(offs + j, last))) if len(flat) else pa.nulls(len(arr), pa.string())
    three, two = pa.array(lens == 3), pa.array(lens == 2)
    name = pc.if_else(three, pc.binary_join_element_wise(part(0), part(1), ":"),
                      pc.if_else(two, part(0), arr))
    vs = pc.if_else(three, part(2), pc.if_else(two, part(1), pa.scalar("1")))
    try:
        val = pc.cast(pc.if_else(pc.is_valid(arr), vs, pa.scalar(None, pa.string())), pa.float64())
    except pa.ArrowInvalid as e:
        raise ValueError(f"could not convert feature value to float: {e}") from None
    names = pd.Series(name.to_numpy(zero_copy_only=False), index=col.index, dtype=object)
    vals = pd.Series(val.to_numpy(zero_copy_only=False), index=col.index, dtype=np.float64)
    return names, vals


def _rowwise(fn, col):
    import pandas as pd

    return pd.Series([fn(v) for v in col.tolist()], dtype=object).infer_objects()


def _extract_feature1(f):
    if f is None:
        return None
    if isinstance(f, (list, tuple, np.ndarray)):
        return [_split(x)[0] for x in f]
    return _split(f)[0]


def _extract_weight1(f):
    if f is None:
        return None
    if isinstance(f, (list, tuple, np.ndarray)):
        return [_split(x)[1] for x in f]
    return _split(f)[1]


@udf("extract_feature", vectorized=True)
def extract_feature(f):
    import pandas as pd

    if isinstance(f, pd.Series):
        sp = _vec_split(f)
        return sp[0] if sp is not None else _rowwise(_extract_feature1, f)
    return _extract_feature1(f)


@udf("extract_weight", vectorized=True)
def extract_weight(f):
    import pandas as pd

    if isinstance(f, pd.Series):
        sp = _vec_split(f)
        if sp is None:
            return _rowwise(_extract_weight1, f)
        return sp[1].where(f.notna(), None) if f.isna().any() else sp[1]
    return _extract_weight1(f)


@udf("feature")
def feature(name, value):
    if name is None:
        return None
    return f"{name}:{_fmt(value) if isinstance(value, float) else value}"


@udf("feature_index")
def feature_index(features):
    if features is None:
        return None
    if isinstance(features, (list, tuple, np.ndarray)):
        return [int(_split(x)[0]) for x in features]
    return int(_split(features)[0])


@udf("sort_by_feature")
def sort_by_feature(m):
    if m is None:
        return None
    return dict(sorted(m.items(), key=lambda kv: kv[0]))


# ------------------------------------------------------------------ hashing
@udf("mhash", vectorized=True)
def mhash(word, num_features: int = 1 << 24):
    """MurmurHash3 x86_32 (seed 0x9747b28c) of the UTF-8 word, mod num_features, 1-based."""
    import pandas as pd

    from ..utils.hashing import mhash_batch

    if isinstance(word, pd.Series):
        nf = int(num_features.iloc[0]) if isinstance(num_features, pd.Series) else int(num_features)
        if isinstance(num_features, pd.Series) and num_features.nunique(dropna=False) > 1:
            return pd.Series([None if w is None else _mhash(str(w), int(k))
                              for w, k in zip(word.tolist(), num_features.tolist())], index=word.index,
                             dtype=object)
        ok = word.notna().to_numpy()
        h = mhash_batch([str(w) for w in word[ok].tolist()], nf) if ok.any() else np.zeros(0, np.int64)
        if ok.all():
            return pd.Series(np.asarray(h, dtype=np.int64), index=word.index)
        out = np.full(len(word), None, dtype=object)
        out[ok] = [int(x) for x in h]
        return pd.Series(out, index=word.index, dtype=object)
    if word is None:
        return None
    return _mhash(str(word), int(num_features))


_FH_OPTS = Options([opt("num_features", "features", 1 << 24, int, "Number of hashed features"),
                    flag("libsvm", None, "Output libsvm-style index:value (default)")],
                   "feature_hashing")


def _feature_hashing1(features, n):
    if features is None:
        return None

    def one(f):
        name, v = _split(f)
        h = _mhash(name, n)
        return str(h) if ":" not in str(f) else f"{h}:{str(f)[len(name) + 1:]}"
    if isinstance(features, (list, tuple, np.ndarray)):
        return [one(f) for f in features if f is not None]
    return one(features)


@udf("feature_hashing", vectorized=True)
def feature_hashing(features, options=None):
    """Hash feature names (keeping values): ``"name:v"`` -> ``"mhash(name):v"``.

    Column form (SQL): the option string is parsed once and the whole column is hashed in one
    native call over its Arrow string buffer (hm_feature_hash_strs) — bit-identical to the
    per-row form."""
    import pandas as pd

    if isinstance(options, pd.Series):
        options = options.iloc[0] if len(options) else None
    n = _FH_OPTS.parse(options)["num_features"]
    if isinstance(features, pd.Series):
        arr = _list_column(features)
        if arr is None:
            return _rowwise(lambda f: _feature_hashing1(f, n), features)
        return _arrow_series(_hash_list_column(arr, n), features.index)
    return _feature_hashing1(features, n)


@udf("sha1")
def sha1(word, num_features: int = 1 << 24):
    """SHA-1 of the UTF-8 word; the first 4 bytes as a signed int, mod num_features, 1-based."""
    if word is None:
        return None
    d = hashlib.sha1(str(word).encode("utf-8")).digest()
    h = int.from_bytes(d[:4], "big", signed=True)
    r = h % int(num_features) if h >= 0 else -((-h) % int(num_features))
    if r < 0:
        r += int(num_features)
    return r + 1


@udf("array_hash_values")
def array_hash_values(values, prefix: str | None = None, num_features: int = 1 << 24,
                      seed: int = DEFAULT_SEED):
    if values is None:
        return None
    p = prefix or ""
    return [_mhash(p + str(v), int(num_features), seed) for v in values if v is not None]


@udf("prefixed_hash_values")
def prefixed_hash_values(values, prefix: str, use_index_as_prefix: bool = False):
    if values is None:
        return None
    out = []
    for i, v in enumerate(values):
        if v is None:
            continue
        pre = f"{i}{prefix}" if use_index_as_prefix else prefix
        out.append(f"{pre}{_mhash(str(v))}")
    return out


# ------------------------------------------------------------------ scaling
def _rescale1(value, mn, mx):
    if value is None:
        return None
    if isinstance(value, str):
        name, v = _split(value)
        return f"{name}:{_fmt(_rescale1(v, mn, mx))}"
    mn, mx = float(mn), float(mx)
    if mx == mn:
        return 0.5
    return min(1.0, max(0.0, (float(value) - mn) / (mx - mn)))


def _zscore1(value, mean, stddev):
    if value is None:
        return None
    if isinstance(value, str):
        name, v = _split(value)
        return f"{name}:{_fmt(_zscore1(v, mean, stddev))}"
    sd = float(stddev)
    return (float(value) - float(mean)) / sd if sd != 0 else 0.0


def _num_cols(*args):
    """float64 arrays of numeric Series / scalars (one length), or None for the per-row path."""
    import pandas as pd

    from ..tools.functions import _numeric_values

    out = []
    for a in args:
        if isinstance(a, pd.Series):
            v = _numeric_values(a)
            if v is None:
                return None
            out.append(v)
        elif isinstance(a, (int, float, np.integer, np.floating)) and not isinstance(a, bool):
            out.append(np.float64(a))
        else:
            return None
    return out


def _scalar_or_rows(fn, args, index):
    import pandas as pd

    cols = [a.tolist() if isinstance(a, pd.Series) else None for a in args]
    n = len(index)
    rows = [fn(*[c[i] if c is not None else a for c, a in zip(cols, args)]) for i in range(n)]
    return pd.Series(rows, index=index, dtype=object).infer_objects()


@udf("rescale", vectorized=True)
def rescale(value, mn, mx):
    """Min-max scaling to [0, 1]; also accepts a ``name:value`` feature string."""
    import pandas as pd

    if not isinstance(value, pd.Series):
        return _rescale1(value, mn, mx)
    c = _num_cols(value, mn, mx)
    if c is None:
        return _scalar_or_rows(_rescale1, (value, mn, mx), value.index)
    v, lo, hi = c
    with np.errstate(divide="ignore", invalid="ignore"):
        x = (v - lo) / (hi - lo)
    y = np.where(x > 0.0, x, 0.0)                  # Python max(0.0, x): x only when x > 0.0
    z = np.where(y < 1.0, y, 1.0)                  # min(1.0, y)
    return pd.Series(np.where(hi == lo, 0.5, z), index=value.index)


@udf("zscore", vectorized=True)
def zscore(value, mean, stddev):
    import pandas as pd

    if not isinstance(value, pd.Series):
        return _zscore1(value, mean, stddev)
    c = _num_cols(value, mean, stddev)
    if c is None:
        return _scalar_or_rows(_zscore1, (value, mean, stddev), value.index)
    v, m, sd = c
    with np.errstate(divide="ignore", invalid="ignore"):
        r = (v - m) / sd
    return pd.Series(np.where(sd != 0, r, 0.0), index=value.index)


def _normalize(features, p):
    if features is None:
        return None
    parsed = [_split(f) for f in features]
    if p == 1:
        norm = sum(abs(v) for _, v in parsed)
    else:
        norm = math.sqrt(sum(v * v for _, v in parsed))
    if norm == 0:
        return list(features)
    return [f"{n}:{_fmt(v / norm)}" for n, v in parsed]


def _normalize_column(col, p: int):
    """l1 / l2_normalize over a whole list<string> column (hm_normalize_features: the per-row
    rule, bit-identical); None when the column needs the per-row path."""
    import pyarrow as pa

    from .. import _native
    from ..io.ingest import arrow_buffers

    arr = _list_column(col)
    if arr is None:
        return None
    data, so, lo = arrow_buffers(arr)
    n = len(lo) - 1
    ns = len(so) - 1
    d = data if len(data) else np.zeros(1, np.uint8)
    so = np.ascontiguousarray(so, dtype=np.int64)
    lo = np.ascontiguousarray(lo, dtype=np.int64)
    oo = np.empty(ns + 1, dtype=np.int64)
    norm = np.empty(max(1, n), dtype=np.float64)
    lib = _native.host()
    tot = lib.hm_normalize_features(d.ctypes.data, so.ctypes.data, lo.ctypes.data, n, p, None,
                                    oo.ctypes.data, norm.ctypes.data)
    if tot < -1:
        return None
    out = np.empty(max(1, int(tot)), dtype=np.uint8)
    lib.hm_normalize_features(d.ctypes.data, so.ctypes.data, lo.ctypes.data, n, p, out.ctypes.data,
                              oo.ctypes.data, norm.ctypes.data)
    strs = pa.LargeStringArray.from_buffers(ns, pa.py_buffer(oo), pa.py_buffer(out))
    res = pa.LargeListArray.from_arrays(pa.array(lo, pa.int64()), strs.cast(pa.string()),
                                        mask=arr.is_null())
    return _arrow_series(res, col.index)


@udf("l1_normalize", vectorized=True)
def l1_normalize(features):
    import pandas as pd

    if isinstance(features, pd.Series):
        r = _normalize_column(features, 1)
        return r if r is not None else _rowwise(lambda f: _normalize(f, 1), features)
    return _normalize(features, 1)


@udf("l2_normalize", "normalize", vectorized=True)
def l2_normalize(features):
    import pandas as pd

    if isinstance(features, pd.Series):
        r = _normalize_column(features, 2)
        return r if r is not None else _rowwise(lambda f: _normalize(f, 2), features)
    return _normalize(features, 2)


# ------------------------------------------------------------------ amplify
@udtf("amplify", per_row=True)
def amplify(xtimes, *cols):
    """Emit every input row ``xtimes`` times (epoch emulation)."""
    for _ in range(int(xtimes)):
        yield tuple(cols)


class RandAmplifier:
    """``rand_amplify(xtimes, num_buffers, *cols [, '-seed N'])``: rows are amplified and
    emitted in a shuffled order through a reservoir of ``num_buffers`` rows (upstream
    ftvec/amplify/RandomAmplifierUDTF.java + utils/collections/RandomizedAmplifier.java).
    ``run`` is a generator: it holds at most ``num_buffers`` rows, never the whole input.
    Draws come from ``java.util.Random`` (``JavaRandom``) seeded with ``seed``."""

    def __init__(self, xtimes: int, num_buffers: int, seed: int = 43):
        from ..utils.prng import JavaRandom

        self.x, self.nb = int(xtimes), int(num_buffers)
        if self.x < 1 or self.nb < 1:
            raise ValueError("rand_amplify: xtimes and num_buffers must be >= 1")
        self.rng = JavaRandom(seed)

    def run(self, rows: Iterable[tuple]):
        buf = []
        for r in rows:
            for _ in range(self.x):
                if len(buf) < self.nb:
                    buf.append(r)
                else:
                    i = self.rng.next_int(len(buf))
                    yield buf[i]
                    buf[i] = r
        for i in range(len(buf) - 1, 0, -1):          # Fisher-Yates drain of the reservoir
            j = self.rng.next_int(i + 1)
            buf[i], buf[j] = buf[j], buf[i]
        yield from buf


_AMPLIFY_OPTS = Options([opt("seed", None, 43, int, "Seed of the reservoir draws")], "rand_amplify")


@udtf("rand_amplify", per_row=False)
def rand_amplify(xtimes, num_buffers, *cols):
    """Emit every row xtimes, shuffled through num_buffers buffers (multi-epoch emulation);
    a trailing ``'-seed N'`` option string seeds the shuffle.

    Whole-input form: ``cols`` are columns; the output frame is built from the streamed rows
    chunk by chunk."""
    x = xtimes[0] if isinstance(xtimes, (list, tuple)) else xtimes
    nb = num_buffers[0] if isinstance(num_buffers, (list, tuple)) else num_buffers
    seed = 43
    if cols and isinstance(cols[-1], str):
        seed = _AMPLIFY_OPTS.parse(cols[-1])["seed"]
        cols = cols[:-1]
    import pandas as pd
    names = [f"c{i}" for i in range(len(cols))]
    it = RandAmplifier(x, nb, seed).run(zip(*cols))
    chunks, chunk = [], []
    for r in it:
        chunk.append(r)
        if len(chunk) == 65536:
            chunks.append(pd.DataFrame(chunk, columns=names))
            chunk = []
    if chunk or not chunks:
        chunks.append(pd.DataFrame(chunk, columns=names))
    return chunks[0] if len(chunks) == 1 else pd.concat(chunks, ignore_index=True)


# ------------------------------------------------------------------ conversion
@udaf("conv2dense")
def conv2dense(features, weights, n_dims):
    nd = int(n_dims[0] if isinstance(n_dims, (list, tuple)) else n_dims)
    out = [0.0] * nd
    for f, w in zip(features, weights):
        if f is not None and 0 <= int(f) < nd:
            out[int(f)] = float(w)
    return out


@udf("to_dense_features", "to_dense")
def to_dense_features(features, dims):
    if features is None:
        return None
    out = [0.0] * (int(dims) + 1)
    for f in features:
        n, v = _split(f)
        i = int(n)
        if 0 <= i <= int(dims):
            out[i] = v
    return out


@udf("to_sparse_features", "to_sparse")
def to_sparse_features(values):
    if values is None:
        return None
    return [f"{i}:{_fmt(v)}" for i, v in enumerate(values) if v is not None and v != 0]


@udtf("quantify", per_row=False)
def quantify(output_flags, *cols):
    """Map every non-numeric column value to a dense integer id (first-seen order)."""
    import pandas as pd
    out_cols = []
    for c in cols:
        vals = list(c)
        if all(v is None or isinstance(v, (int, float, np.integer, np.floating)) for v in vals):
            out_cols.append(vals)
            continue
        ids = {}
        out_cols.append([None if v is None else ids.setdefault(v, len(ids)) for v in vals])
    return pd.DataFrame({f"c{i}": c for i, c in enumerate(out_cols)})


# ------------------------------------------------------------------ binning
@udaf("build_bins")
def build_bins(values, num_bins, auto_shrink=None):
    """Quantile bin boundaries [-inf, q1, ..., +inf] (auto_shrink drops duplicates)."""
    nb = int(num_bins[0] if isinstance(num_bins, (list, tuple)) else num_bins)
    shrink = bool(auto_shrink[0]) if isinstance(auto_shrink, (list, tuple)) and auto_shrink else False
    v = np.asarray([x for x in values if x is not None], dtype=np.float64)
    qs = np.quantile(v, np.linspace(0, 1, nb + 1)[1:-1]) if v.size else np.array([])
    edges = [-math.inf] + qs.tolist() + [math.inf]
    if shrink:
        edges = sorted(set(edges))
    return edges


@udf("feature_binning")
def feature_binning(features, quantiles):
    """``feature_binning(array<features>, map<name, bins>)`` -> ``name:bin`` features, or
    ``feature_binning(double, array<double> bins)`` -> bin index."""
    if features is None:
        return None
    if isinstance(features, (int, float, np.integer, np.floating)):
        return int(np.searchsorted(np.asarray(quantiles[1:-1]), float(features), side="right"))
    out = []
    for f in features:
        n, v = _split(f)
        if n in quantiles:
            b = int(np.searchsorted(np.asarray(quantiles[n][1:-1]), v, side="right"))
            out.append(f"{n}:{b}")
        else:
            out.append(f)
    return out


# ------------------------------------------------------------------ pairing
@udf("polynomial_features")
def polynomial_features(features, degree: int = 2, interaction_only: bool = False,
                        truncate: bool = True):
    """Products of up to ``degree`` features: ``a^b:v_a*v_b`` (names joined with ``^``)."""
    if features is None:
        return None
    parsed = [_split(f) for f in features]
    out = list(features)
    deg = int(degree)

    def rec(start, names, val, d):
        if d > 1:
            out.append(f"{'^'.join(names)}:{_fmt(val)}")
        if d == deg:
            return
        for j in range(start, len(parsed)):
            n, v = parsed[j]
            if interaction_only and n in names:
                continue
            if truncate and (v == 0 or v == 1) and d >= 1 and n in names:
                continue
            rec(j if not interaction_only else j + 1, names + [n], val * v, d + 1)
    for i, (n, v) in enumerate(parsed):
        rec(i if not interaction_only else i + 1, [n], v, 1)
    return out


@udf("powered_features")
def powered_features(features, degree: int = 2, truncate: bool = True):
    if features is None:
        return None
    out = list(features)
    for f in features:
        n, v = _split(f)
        if truncate and (v == 0 or v == 1):
            continue
        for d in range(2, int(degree) + 1):
            out.append(f"{n}^{d}:{_fmt(v ** d)}")
    return out


_FP_OPTS = Options([flag("kpa", None, "Emit (h, hk, xh, xk) for kernel-expanded PA"),
                    flag("ffm", None, "Emit (i, j, xi, xj) pairs for FFM prediction"),
                    opt("feature_hashing", None, -1, int, "FFM: hash bits"),
                    opt("num_fields", None, 256, int, "FFM: number of fields"),
                    flag("no_bias", None, "FFM: omit the bias row")], "feature_pairs")


@udtf("feature_pairs", per_row=True, cols=("i", "j", "xi", "xj"))
def feature_pairs(features, options=None):
    """``-ffm``: one row (i, NULL, xi, NULL) per linear term and (i, j, xi, xj) per field pair
    where i/j are the model keys V(feature, field of the partner).  ``-kpa``: (h, hk, xh, xk)."""
    cl = _FP_OPTS.parse(options)
    if features is None:
        return
    if cl["ffm"]:
        from ..models.ffm_keys import ffm_pair_rows
        yield from ffm_pair_rows(features, cl)
        return
    parsed = [_split(f) for f in features]
    for a in range(len(parsed)):
        ha, xa = parsed[a]
        yield (ha, None, xa, None)
        for b in range(a + 1, len(parsed)):
            hb, xb = parsed[b]
            yield (ha, hb, xa, xb)


def _feature_pairs_batch(features, options=None):
    """Column-at-once ``feature_pairs(features, '-ffm ...')`` for LATERAL VIEW (a constant option
    string); None -> the per-row path."""
    if options is not None:
        ops = set(map(str, options))
        if len(ops) != 1:
            return None
        options = ops.pop()
    cl = _FP_OPTS.parse(options)
    if not cl["ffm"]:
        return None
    from ..models.ffm_keys import ffm_pair_columns
    rows_idx, cols = ffm_pair_columns(features, cl)
    return rows_idx, [cols["i"], cols["j"], cols["xi"], cols["xj"]]


feature_pairs.batch = _feature_pairs_batch


# ------------------------------------------------------------------ ranking / sampling
_BPR_OPTS = Options([opt("sampling_rate", None, 1.0, float, "Sampling rate"),
                     flag("with_replacement", None, "Sample with replacement"),
                     flag("without_replacement", None, "Sample without replacement (default)"),
                     flag("pairwise_sampling", None, "Sample (pos, neg) per positive"),
                     opt("max_item_id", None, None, int, "Max item id"),
                     opt("seed", None, 31, int, "Seed")], "bpr_sampling")


@udtf("bpr_sampling", per_row=True, cols=("user", "pos_item", "neg_item"))
def bpr_sampling(user, pos_items, max_item_id=None, options=None):
    """Negative sampling for BPR: for each positive item of the user draw a negative item
    uniformly from [0, max_item_id] \\ positives."""
    if isinstance(max_item_id, str) and options is None:
        options, max_item_id = max_item_id, None
    cl = _BPR_OPTS.parse(options)
    mx = int(max_item_id if max_item_id is not None else (cl["max_item_id"] or max(pos_items)))
    pos = set(int(p) for p in pos_items)
    if len(pos) > mx:
        return
    # the per-user stream is seeded from a stable hash of str(user) (MurmurHash3), never
    # Python's salted hash(): the same -seed replays the same triples in every process
    from ..utils.hashing import murmurhash3
    from ..utils.prng import JavaRandom

    rng = JavaRandom((int(cl["seed"]) * 1000003) ^ (murmurhash3(str(user)) & 0xFFFFFFFF))
    n = max(1, int(round(len(pos) * cl["sampling_rate"])))
    plist = sorted(pos)
    for k in range(n):
        p = plist[k % len(plist)] if k < len(plist) else plist[rng.next_int(len(plist))]
        while True:
            j = rng.next_int(mx + 1)
            if j not in pos:
                break
        yield (user, p, j)


@udtf("item_pairs_sampling", per_row=True, cols=("pos_item", "neg_item"))
def item_pairs_sampling(pos_items, max_item_id, options=None):
    for user, p, j in bpr_sampling(0, pos_items, max_item_id, options):
        yield (p, j)


@udtf("populate_not_in", per_row=True, cols=("item",))
def populate_not_in(items, max_item_id, options=None):
    """Items in [0, max_item_id] not contained in ``items``."""
    s = set(int(i) for i in items) if items is not None else set()
    for i in range(int(max_item_id) + 1):
        if i not in s:
            yield (i,)


# ------------------------------------------------------------------ selection
@udf("chi2")
def chi2(observed, expected):
    """Per-feature chi-square statistic and p-value of observed vs expected counts
    (rows = classes, columns = features)."""
    from scipy.stats import chi2 as _chi2
    O = np.asarray(observed, dtype=np.float64)
    E = np.asarray(expected, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        terms = np.where(E > 0, (O - E) ** 2 / E, 0.0)
    stat = terms.sum(0)
    dof = O.shape[0] - 1
    p = _chi2.sf(stat, dof)
    return {"chi2": stat.tolist(), "pvalue": p.tolist()}


@udaf("snr")
def snr(features, labels):
    """Signal-to-noise ratio per feature for one-hot labels: Σ_{pairs of classes}
    |μ_i − μ_j| / (σ_i + σ_j)."""
    X = np.asarray([list(f) for f in features], dtype=np.float64)
    Y = np.asarray([list(l) for l in labels], dtype=np.int64)
    cls = Y.argmax(1)
    k = Y.shape[1]
    out = np.zeros(X.shape[1])
    stats = []
    for c in range(k):
        Xc = X[cls == c]
        stats.append((Xc.mean(0) if len(Xc) else np.zeros(X.shape[1]),
                      Xc.std(0) if len(Xc) else np.zeros(X.shape[1])))
    for a in range(k):
        for b in range(a + 1, k):
            den = stats[a][1] + stats[b][1]
            with np.errstate(divide="ignore", invalid="ignore"):
                out += np.where(den > 0, np.abs(stats[a][0] - stats[b][0]) / den, 0.0)
    return out.tolist()


# ------------------------------------------------------------------ text
@udaf("tf")
def tf(terms):
    """Term frequency map of the group's terms: count / total."""
    c = Counter(t for t in terms if t is not None)
    tot = sum(c.values())
    return {k: v / tot for k, v in c.items()} if tot else {}


@udf("bm25")
def bm25(term_freq, doc_len, avg_doc_len, num_docs, num_docs_with_term, k1: float = 1.2,
         b: float = 0.75, delta: float = 0.0):
    """Okapi BM25 score of one term in one document (BM25+ with delta > 0)."""
    idf = math.log(1 + (num_docs - num_docs_with_term + 0.5) / (num_docs_with_term + 0.5))
    tf_ = float(term_freq)
    norm = tf_ * (k1 + 1) / (tf_ + k1 * (1 - b + b * float(doc_len) / float(avg_doc_len)))
    return idf * (norm + delta)


@udf("tfidf")
def tfidf(tf_value, df, num_docs):
    """tf * log10(N / max(1, df)) + 1 (the define-macros.hive ``tfidf`` macro)."""
    return float(tf_value) * (math.log10(float(num_docs) / max(1.0, float(df))) + 1.0)


@udf("idf")
def idf(df, num_docs):
    return math.log10(float(num_docs) / max(1.0, float(df))) + 1.0


# ------------------------------------------------------------------ transformation
def _is_num(v):
    return isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool)


@udf("vectorize_features")
def vectorize_features(names, *values):
    """Quantitative values -> ``name:value`` (0/NULL dropped); strings -> ``name#value``."""
    out = []
    for n, v in zip(names, values):
        if v is None:
            continue
        if _is_num(v):
            if float(v) != 0:
                out.append(f"{n}:{_fmt(v)}")
        elif isinstance(v, bool):
            if v:
                out.append(f"{n}")
        else:
            out.append(f"{n}#{v}")
    return out


@udf("categorical_features")
def categorical_features(names, *values):
    return [f"{n}#{v}" for n, v in zip(names, values) if v is not None]


@udf("quantitative_features")
def quantitative_features(names, *values):
    return [f"{n}:{_fmt(v)}" for n, v in zip(names, values) if v is not None and float(v) != 0]


@udf("indexed_features")
def indexed_features(*values):
    return [f"{i + 1}:{_fmt(v)}" for i, v in enumerate(values) if v is not None]


@udtf("quantified_features", per_row=False, cols=("features",))
def quantified_features(output_flags, *cols):
    import pandas as pd
    q = quantify(output_flags, *cols)
    rows = [list(map(lambda x: float(x) if x is not None else None, r)) for r in q.itertuples(index=False)]
    return pd.DataFrame({"features": rows})


@udtf("binarize_label", per_row=True)
def binarize_label(n_pos, n_neg, *cols):
    """Emit the row ``n_pos`` times with label 1 and ``n_neg`` times with label 0."""
    for _ in range(int(n_pos or 0)):
        yield tuple(cols) + (1,)
    for _ in range(int(n_neg or 0)):
        yield tuple(cols) + (0,)


@udaf("onehot_encoding")
def onehot_encoding(*cols):
    """One map per column: distinct value -> consecutive one-hot index (global across columns,
    starting at 1)."""
    out = []
    nxt = 1
    for c in cols:
        m = {}
        for v in c:
            if v is not None and v not in m:
                m[v] = nxt
                nxt += 1
        out.append(m)
    return out


_FFMF_OPTS = Options([opt("feature_hashing", None, -1, int, "Hash bits for the index"),
                      opt("num_fields", None, 256, int, "Number of fields"),
                      flag("no_hash", None, "Keep indices unhashed (names must be integers)")],
                     "ffm_features")


@udf("ffm_features")
def ffm_features(names, *values_and_opts):
    """``ffm_features(array<string> names, v1, v2, ... [, options])`` -> ``field:index:value``.
    Field = column position; index = mhash("name#value") (categorical) or mhash(name)."""
    vals = list(values_and_opts)
    options = None
    if vals and isinstance(vals[-1], str) and vals[-1].startswith("-") and len(vals) > len(names):
        options = vals.pop()
    cl = _FFMF_OPTS.parse(options)
    nf = (1 << cl["feature_hashing"]) if cl["feature_hashing"] > 0 else (1 << 24)
    out = []
    for f, (n, v) in enumerate(zip(names, vals)):
        if v is None:
            continue
        if _is_num(v):
            if float(v) == 0:
                continue
            key = str(n)
            x = float(v)
        else:
            key = f"{n}#{v}"
            x = 1.0
        idx = int(key) if cl["no_hash"] else _mhash(key, nf)
        out.append(f"{f}:{idx}:{_fmt(x)}")
    return out


@udf("add_field_indices")
def add_field_indices(features):
    """Prefix each feature with its 1-based position as the field: ``i:feature``."""
    if features is None:
        return None
    return [f"{i + 1}:{f}" for i, f in enumerate(features)]
