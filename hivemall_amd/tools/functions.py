"""Tool UDFs (upstream core/src/main/java/hivemall/tools/{array,map,list,
bits,compress,text,math,matrix,vector,mapred,json,sanity,timeseries,...}/*.java and
resources/ddl/define-macros.hive).  Host-side Python: these are per-row utilities that never
dominate a pipeline's run time.
"""
from __future__ import annotations

import base64
import json
import math
import re
import unicodedata
import zlib
from collections import OrderedDict
from typing import Any

import numpy as np

from ..registry import udaf, udf, udtf
from ..utils import base91 as _b91
from ..utils.collections import BoundedPriorityQueue


def _arr(x):
    return None if x is None else list(x)


# ------------------------------------------------------------------ arrays
@udf("array_concat", "concat_array")
def array_concat(*arrays):
    out = []
    for a in arrays:
        if a is not None:
            out.extend(list(a))
    return out


@udaf("array_avg")
def array_avg(arrays):
    """Element-wise average of equal-length numeric arrays."""
    arrs = [np.asarray(a, dtype=np.float64) for a in arrays if a is not None]
    if not arrs:
        return None
    return np.mean(np.stack(arrs), 0).tolist()


@udaf("array_sum")
def array_sum(arrays):
    arrs = [np.asarray(a, dtype=np.float64) for a in arrays if a is not None]
    if not arrs:
        return None
    return np.sum(np.stack(arrs), 0).tolist()


@udf("array_remove")
def array_remove(a, target):
    if a is None:
        return None
    ts = set(target) if isinstance(target, (list, tuple)) else {target}
    return [x for x in a if x not in ts]


@udf("array_intersect")
def array_intersect(*arrays):
    arrs = [a for a in arrays if a is not None]
    if not arrs:
        return None
    s = set(arrs[0])
    for a in arrs[1:]:
        s &= set(a)
    return [x for x in dict.fromkeys(arrs[0]) if x in s]


@udf("array_union")
def array_union(*arrays):
    out = []
    seen = set()
    for a in arrays:
        for x in a or []:
            if x not in seen:
                seen.add(x)
                out.append(x)
    return out


@udf("array_slice", "subarray")
def array_slice(a, offset, length=None):
    """0-based ``offset``; negative offsets count from the end (array_slice semantics)."""
    if a is None:
        return None
    a = list(a)
    o = int(offset)
    if o < 0:
        o = len(a) + o
    return a[o:] if length is None else a[o:o + int(length)]


@udf("subarray_endwith")
def subarray_endwith(a, key):
    if a is None:
        return None
    a = list(a)
    for i in range(len(a) - 1, -1, -1):
        if a[i] == key:
            return a[: i + 1]
    return None


@udf("subarray_startwith")
def subarray_startwith(a, key):
    if a is None:
        return None
    a = list(a)
    for i, x in enumerate(a):
        if x == key:
            return a[i:]
    return None


@udf("sort_and_uniq_array")
def sort_and_uniq_array(a):
    return None if a is None else sorted(set(a))


@udf("to_string_array")
def to_string_array(a):
    return None if a is None else [None if x is None else str(x) for x in a]


@udf("array_append")
def array_append(a, x):
    return [x] if a is None else list(a) + [x]


@udf("array_flatten")
def array_flatten(a):
    if a is None:
        return None
    out = []
    for x in a:
        if isinstance(x, (list, tuple, np.ndarray)):
            out.extend(x)
        else:
            out.append(x)
    return out


@udf("first_element")
def first_element(a):
    return None if not a else list(a)[0]


@udf("last_element")
def last_element(a):
    return None if not a else list(a)[-1]


@udf("element_at")
def element_at(a, i):
    if a is None:
        return None
    a = list(a)
    i = int(i)
    if i < 0:
        i += len(a)
    return a[i] if 0 <= i < len(a) else None


@udf("float_array")
def float_array(n):
    return [0.0] * int(n)


@udf("select_k_best")
def select_k_best(values, importance, k):
    """The k elements of ``values`` at the positions of the k largest ``importance``."""
    idx = np.argsort(-np.asarray(importance, dtype=np.float64), kind="stable")[: int(k)]
    v = list(values)
    return [v[i] for i in sorted(idx)]


@udf("conditional_emit")
def conditional_emit(conditions, features):
    return [f for c, f in zip(conditions, features) if c]


@udf("array_to_str")
def array_to_str(a, sep=","):
    return None if a is None else sep.join("" if x is None else str(x) for x in a)


@udf("array_min")
def array_min(a):
    return None if not a else min(x for x in a if x is not None)


@udf("array_max")
def array_max(a):
    return None if not a else max(x for x in a if x is not None)


@udf("arange")
def arange(start, stop=None, step=1):
    if stop is None:
        start, stop = 0, start
    return list(range(int(start), int(stop), int(step)))


# ------------------------------------------------------------------ maps
@udf("map_get_sum")
def map_get_sum(m, keys):
    return float(sum(m.get(k, 0.0) for k in keys)) if m is not None else None


@udf("map_tail_n")
def map_tail_n(m, n):
    if m is None:
        return None
    items = sorted(m.items(), key=lambda kv: kv[0])
    return dict(items[-int(n):])


@udaf("to_map")
def to_map(keys, values):
    return {k: v for k, v in zip(keys, values) if k is not None}


@udaf("to_ordered_map")
def to_ordered_map(keys, values, reverse=None):
    rev = bool(reverse[0]) if isinstance(reverse, (list, tuple)) and reverse else False
    d = {k: v for k, v in zip(keys, values) if k is not None}
    return dict(sorted(d.items(), key=lambda kv: kv[0], reverse=rev))


@udf("map_include_keys")
def map_include_keys(m, keys):
    return None if m is None else {k: v for k, v in m.items() if k in set(keys)}


@udf("map_exclude_keys")
def map_exclude_keys(m, keys):
    return None if m is None else {k: v for k, v in m.items() if k not in set(keys)}


@udf("map_key_values")
def map_key_values(m):
    return None if m is None else [{"key": k, "value": v} for k, v in m.items()]


@udf("map_roulette")
def map_roulette(m, seed=None):
    """Pick a key with probability proportional to its (non-negative) value."""
    if not m:
        return None
    rng = np.random.default_rng(seed)
    keys = list(m.keys())
    w = np.asarray([max(0.0, float(m[k])) for k in keys])
    if w.sum() <= 0:
        return None
    return keys[int(rng.choice(len(keys), p=w / w.sum()))]


@udf("merge_maps")
def merge_maps(*maps):
    out = {}
    for m in maps:
        if m:
            out.update(m)
    return out


@udaf("merge_maps_agg")
def merge_maps_agg(maps):
    out = {}
    for m in maps:
        if m:
            out.update(m)
    return out


# ------------------------------------------------------------------ lists / bits / compress
@udaf("to_ordered_list")
def to_ordered_list(values, keys=None, options=None):
    """Values ordered by ``keys`` (or by value); ``-reverse``, ``-k N`` (top-k by key)."""
    opts = options[0] if isinstance(options, (list, tuple)) and options else options
    if keys is not None and isinstance(keys, (list, tuple)) and keys and isinstance(keys[0], str) \
            and keys[0].startswith("-") and options is None:
        opts, keys = keys[0], None
    reverse = False
    k = None
    if opts:
        toks = str(opts).split()
        reverse = "-reverse" in toks
        if "-k" in toks:
            k = int(toks[toks.index("-k") + 1])
            # -k N: the N largest keys, largest first; -k -N: the N smallest, smallest first;
            # -reverse flips the order in both cases
            reverse = (k > 0) != reverse
            k = abs(k)
    ks = list(values) if keys is None else list(keys)
    if k is not None:
        if k == 0:
            return []
        # top-k through a bounded heap (upstream keeps a BoundedPriorityQueue per group,
        # tools/list/UDAFToOrderedList.java): O(n log k), ties in arrival order
        q = BoundedPriorityQueue(k, key=(lambda i: ks[i]) if reverse else (lambda i: _Desc(ks[i])))
        for i in range(len(ks)):
            q.offer(i)
        return [values[i] for i in q.sorted()]
    order = sorted(range(len(ks)), key=lambda i: ks[i], reverse=reverse)
    return [values[i] for i in order]


class _Desc:
    """Inverts the ordering of a key, so a max-heap keeps the k smallest."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __lt__(self, o):
        return o.v < self.v

    def __gt__(self, o):
        return self.v < o.v

    def __eq__(self, o):
        return self.v == o.v


@udf("to_bits")
def to_bits(indexes):
    """Set bits at the given non-negative indexes -> array<long> bitset."""
    if indexes is None:
        return None
    mx = max(indexes) if indexes else -1
    words = [0] * (mx // 64 + 1)
    for i in indexes:
        words[i // 64] |= 1 << (i % 64)
    return [w - (1 << 64) if w >= (1 << 63) else w for w in words]


@udf("unbits")
def unbits(bitset):
    out = []
    for wi, w in enumerate(bitset or []):
        w &= (1 << 64) - 1
        for b in range(64):
            if w >> b & 1:
                out.append(wi * 64 + b)
    return out


@udf("bits_or")
def bits_or(*bitsets):
    n = max((len(b) for b in bitsets if b), default=0)
    out = [0] * n
    for b in bitsets:
        for i, w in enumerate(b or []):
            out[i] |= w
    return out


@udaf("bits_collect")
def bits_collect(indexes):
    return to_bits([int(i) for i in indexes if i is not None])


@udf("deflate")
def deflate(s, level: int = -1):
    if s is None:
        return None
    return zlib.compress(str(s).encode("utf-8"), int(level))


@udf("inflate")
def inflate(b):
    if b is None:
        return None
    return zlib.decompress(bytes(b)).decode("utf-8")


# ------------------------------------------------------------------ text
@udf("base91")
def base91(b):
    if b is None:
        return None
    data = b.encode("utf-8") if isinstance(b, str) else bytes(b)
    return _b91.encode(data)


@udf("unbase91")
def unbase91(s):
    return None if s is None else _b91.decode(s)


_WORD = re.compile(r"[\w']+", re.UNICODE)


@udf("tokenize")
def tokenize(text, to_lower: bool = False):
    """Split on non-word characters (Hivemall TokenizeUDF: whitespace/punctuation)."""
    if text is None:
        return None
    toks = re.split(r"[\s\p{P}]+" if False else r"[^\w']+", str(text))
    toks = [t for t in toks if t]
    return [t.lower() for t in toks] if to_lower else toks


@udf("split_words")
def split_words(text, regex: str = r"[\s ]+"):
    return None if text is None else [t for t in re.split(regex, str(text)) if t]


_STOPWORDS = set("""a about above after again against all am an and any are as at be because been
before being below between both but by can could did do does doing down during each few for from
further had has have having he her here hers herself him himself his how i if in into is it its
itself just me more most my myself no nor not now of off on once only or other our ours ourselves
out over own same she should so some such than that the their theirs them themselves then there
these they this those through to too under until up very was we were what when where which while
who whom why will with would you your yours yourself yourselves""".split())


@udf("is_stopword")
def is_stopword(word):
    return None if word is None else str(word).lower() in _STOPWORDS


@udf("normalize_unicode")
def normalize_unicode(s, form: str = "NFC"):
    return None if s is None else unicodedata.normalize(str(form).upper(), str(s))


@udf("word_ngrams")
def word_ngrams(words, min_n: int, max_n: int):
    if words is None:
        return None
    w = list(words)
    out = []
    for n in range(int(min_n), int(max_n) + 1):
        out.extend(" ".join(w[i:i + n]) for i in range(len(w) - n + 1))
    return out


_IRREGULAR = {"children": "child", "men": "man", "women": "woman", "people": "person",
              "mice": "mouse", "geese": "goose", "feet": "foot", "teeth": "tooth",
              "data": "datum", "indices": "index", "matrices": "matrix", "analyses": "analysis"}


@udf("singularize")
def singularize(word):
    """English singularization (irregular table + suffix rules)."""
    if word is None:
        return None
    w = str(word)
    lw = w.lower()
    if lw in _IRREGULAR:
        return _IRREGULAR[lw]
    for suf, rep in (("ies", "y"), ("ves", "f"), ("sses", "ss"), ("ches", "ch"), ("shes", "sh"),
                     ("xes", "x"), ("zes", "z"), ("oes", "o")):
        if lw.endswith(suf) and len(lw) > len(suf) + 1:
            return w[: -len(suf)] + rep
    if lw.endswith("s") and not lw.endswith("ss") and not lw.endswith("us") and len(lw) > 3:
        return w[:-1]
    return w


# ------------------------------------------------------------------ math / vectors
def _numeric_values(col):
    """float64 ndarray of a numeric (non-object) Series, else None (the per-row path keeps
    None / strings / mixed content as it is)."""
    import pandas as pd

    if not isinstance(col, pd.Series) or col.dtype == object or not (
            pd.api.types.is_float_dtype(col.dtype) or pd.api.types.is_integer_dtype(col.dtype)):
        return None
    if col.isna().any():
        return None
    return np.ascontiguousarray(col.to_numpy(dtype=np.float64))


def _sigmoid1(x):
    if x is None:
        return None
    x = float(x)
    return 1.0 / (1.0 + math.exp(-x)) if x >= 0 else math.exp(x) / (1.0 + math.exp(x))


@udf("sigmoid", vectorized=True)
def sigmoid(x):
    """1 / (1 + exp(-x)); a numeric column runs in one native pass (hm_sigmoid_f64, the same
    libm exp and branches, bit-identical)."""
    import pandas as pd

    if not isinstance(x, pd.Series):
        return _sigmoid1(x)
    v = _numeric_values(x)
    if v is None:
        return pd.Series([_sigmoid1(e) for e in x.tolist()], index=x.index, dtype=object).infer_objects()
    from .. import _native

    out = np.empty_like(v)
    if len(v):
        _native.host().hm_sigmoid_f64(v.ctypes.data, len(v), out.ctypes.data)
    return pd.Series(out, index=x.index)


@udf("l2_norm")
def l2_norm(x):
    """L2 norm of an array, or (as an aggregate over a group) of the values."""
    return None if x is None else math.sqrt(float(np.sum(np.square(np.asarray(x, dtype=np.float64)))))


@udaf("l2_norm_agg")
def l2_norm_agg(values):
    return math.sqrt(sum(float(v) ** 2 for v in values if v is not None))


@udf("infinity")
def infinity():
    return math.inf


@udf("is_finite")
def is_finite(x):
    return None if x is None else math.isfinite(float(x))


@udf("is_infinite")
def is_infinite(x):
    return None if x is None else math.isinf(float(x))


@udf("nan")
def nan():
    return math.nan


@udf("is_nan")
def is_nan(x):
    return None if x is None else math.isnan(float(x))


@udaf("transpose_and_dot")
def transpose_and_dot(xs, ys):
    """Σ_rows xᵀ y: the outer-product sum of two array columns (matrix)."""
    X = np.asarray([list(x) for x in xs], dtype=np.float64)
    Y = np.asarray([list(y) for y in ys], dtype=np.float64)
    return (X.T @ Y).tolist()


@udf("vector_add")
def vector_add(a, b):
    return (np.asarray(a, dtype=np.float64) + np.asarray(b, dtype=np.float64)).tolist()


@udf("vector_dot")
def vector_dot(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if b.ndim == 0:
        return (a * b).tolist()
    return float(a @ b)


# ------------------------------------------------------------------ map-reduce context
class _Ctx:
    task_id = 0
    job_id = "hivemall_amd"
    conf: dict = {}
    distcache: dict = {}
    row = 0          # rowid()'s sequence
    rownum = 0       # rownum()'s sequence (a separate UDF instance in Hive, so its own counter)


CONTEXT = _Ctx()


@udf("rowid")
def rowid():
    """``<taskid>-<sequence>`` unique row id (task = rank)."""
    CONTEXT.row += 1
    return f"{CONTEXT.task_id}-{CONTEXT.row}"


@udf("rownum")
def rownum():
    """Hivemall's ``sprintf("%d%04d", sequence, taskid)`` as a long: unique per task while the
    task id stays below 10,000."""
    CONTEXT.rownum += 1
    return int(f"{CONTEXT.rownum}{CONTEXT.task_id:04d}")


@udf("taskid")
def taskid():
    return CONTEXT.task_id


@udf("jobid")
def jobid():
    return CONTEXT.job_id


@udf("jobconf_gets")
def jobconf_gets(keys):
    ks = keys.split(",") if isinstance(keys, str) else list(keys)
    return [str(CONTEXT.conf.get(k.strip(), "")) for k in ks]


@udf("distcache_gets")
def distcache_gets(filepath, key, default=None):
    return CONTEXT.distcache.get(filepath, {}).get(key, default)


# ------------------------------------------------------------------ misc
@udtf("generate_series", per_row=True, cols=("value",))
def generate_series(start, end, step=1):
    s, e, st = int(start), int(end), int(step)
    if st == 0:
        raise ValueError("generate_series: step must not be 0")
    rng = range(s, e + (1 if st > 0 else -1), st)
    for v in rng:
        yield (v,)


@udf("convert_label")
def convert_label(label):
    """0/1 <-> -1/+1 label conversion."""
    if label is None:
        return None
    v = float(label)
    if v == 0:
        return -1
    if v == -1:
        return 0
    return 1 if isinstance(label, (int, np.integer)) else 1.0


@udf("x_rank")
def x_rank(key):
    """Sequential rank within consecutive equal keys (the classic Hive rank UDF)."""
    st = getattr(x_rank, "_st", {"key": object(), "n": 0})
    if key != st["key"]:
        st = {"key": key, "n": 0}
    st["n"] += 1
    x_rank._st = st
    return st["n"]


@udf("try_cast")
def try_cast(value, type_name: str):
    try:
        t = str(type_name).lower()
        if t in ("int", "bigint", "smallint", "tinyint"):
            return int(value)
        if t in ("float", "double", "decimal"):
            return float(value)
        if t == "string":
            return str(value)
        if t == "boolean":
            return bool(value)
        if t.startswith("array"):
            return list(value)
        return value
    except (TypeError, ValueError):
        return None


@udf("sessionize")
def sessionize(time_in_sec, threshold_in_sec, subject=None):
    """Session id: a new session starts when the gap to the previous event of the same
    subject exceeds the threshold (stateful over the ordered input)."""
    st = getattr(sessionize, "_st", {})
    key = subject
    last, sid = st.get(key, (None, None))
    t = float(time_in_sec)
    if last is None or t - last > float(threshold_in_sec):
        import uuid
        sid = str(uuid.uuid4())
    st[key] = (t, sid)
    sessionize._st = st
    return sid


@udf("to_json")
def to_json(obj, *rest):
    def conv(o):
        if isinstance(o, np.ndarray):
            return o.tolist()
        if isinstance(o, (np.integer,)):
            return int(o)
        if isinstance(o, (np.floating,)):
            return float(o)
        raise TypeError(str(type(o)))
    return json.dumps(obj, default=conv)


@udf("from_json")
def from_json(s, type_name=None):
    return None if s is None else json.loads(s)


@udf("assert")
def assert_(cond, msg="assertion failed"):
    if not cond:
        raise AssertionError(msg)
    return True


@udf("raise_error")
def raise_error(msg="error"):
    raise RuntimeError(msg)


@udf("moving_avg")
def moving_avg(x, window):
    """Stateful moving average over the ordered input stream."""
    st = getattr(moving_avg, "_st", [])
    st.append(float(x))
    w = int(window)
    if len(st) > w:
        st = st[-w:]
    moving_avg._st = st
    return sum(st) / len(st)


@udf("hivemall_version")
def hivemall_version():
    from .. import __version__
    return __version__


# ------------------------------------------------------------------ macros (define-macros.hive)
@udf("max2")
def max2(a, b):
    return a if b is None or (a is not None and a >= b) else b


@udf("min2")
def min2(a, b):
    return a if b is None or (a is not None and a <= b) else b


@udf("rand_gid")
def rand_gid(k):
    return int(np.random.randint(0, int(k)))
