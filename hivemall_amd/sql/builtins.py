"""Hive built-in functions needed by Hivemall scripts (scalar, aggregate and table functions).

Scalar built-ins are vectorised over pandas Series where cheap and row-wise otherwise; NULL
(None / NaN) propagates like in Hive.
"""
from __future__ import annotations

import hashlib
import json
import math
import random
import re

import numpy as np
import pandas as pd


def is_null(v) -> bool:
    if v is None:
        return True
    if isinstance(v, float) and math.isnan(v):
        return True
    return False


def rowwise(fn, null_prop: bool = True):
    def apply(*cols):
        n = len(cols[0]) if cols else 0
        out = []
        for vals in zip(*[c.tolist() for c in cols]):
            if null_prop and any(is_null(v) for v in vals):
                out.append(None)
            else:
                out.append(fn(*vals))
        return pd.Series(out, dtype=object) if n else pd.Series([], dtype=object)
    return apply


def _num(s: pd.Series) -> pd.Series:
    return pd.to_numeric(s, errors="coerce")


def _vec_math(f):
    def apply(s):
        return pd.Series(f(_num(s).to_numpy(dtype=np.float64)))
    return apply


def _round(s, d=None):
    if d is None:
        return pd.Series(np.round(_num(s).to_numpy(dtype=np.float64)))
    d = int(d.iloc[0])
    return pd.Series(np.round(_num(s).to_numpy(dtype=np.float64), d))


def _if(c, a, b):
    cond = c.map(lambda v: bool(v) if not is_null(v) else False).to_numpy()
    return pd.Series(np.where(cond, a.to_numpy(dtype=object), b.to_numpy(dtype=object)), dtype=object)


def _coalesce(*cols):
    out = []
    for vals in zip(*[c.tolist() for c in cols]):
        out.append(next((v for v in vals if not is_null(v)), None))
    return pd.Series(out, dtype=object)


def _concat(*cols):
    def f(*vals):
        if all(isinstance(v, (list, tuple, np.ndarray)) for v in vals):
            out = []
            for v in vals:
                out.extend(list(v))
            return out
        return "".join(str(v) for v in vals)
    return rowwise(f)(*cols)


def _concat_ws(sep, *cols):
    def f(s, *vals):
        parts = []
        for v in vals:
            if is_null(v):
                continue
            if isinstance(v, (list, tuple, np.ndarray)):
                parts.extend(str(x) for x in v)
            else:
                parts.append(str(v))
        return str(s).join(parts)
    return rowwise(f, null_prop=False)(sep, *cols)


def _size(s):
    return pd.Series([-1 if is_null(v) else len(v) for v in s.tolist()])


def _split(s, pat):
    return rowwise(lambda a, p: re.split(p, str(a)))(s, pat)


def _array(*cols):
    n = len(cols[0]) if cols else 1
    return pd.Series([list(vals) for vals in zip(*[c.tolist() for c in cols])] if cols else [[]] * n,
                     dtype=object)


def _map(*cols):
    out = []
    for vals in zip(*[c.tolist() for c in cols]):
        out.append({vals[i]: vals[i + 1] for i in range(0, len(vals), 2)})
    return pd.Series(out, dtype=object)


def _struct(*cols):
    return pd.Series([{f"col{i + 1}": v for i, v in enumerate(vals)}
                      for vals in zip(*[c.tolist() for c in cols])], dtype=object)


def _named_struct(*cols):
    return pd.Series([{vals[i]: vals[i + 1] for i in range(0, len(vals), 2)}
                      for vals in zip(*[c.tolist() for c in cols])], dtype=object)


def _substr(s, start, length=None):
    def f(a, st, ln=None):
        a = str(a)
        st = int(st)
        i = st - 1 if st > 0 else len(a) + st
        return a[i:] if ln is None else a[i:i + int(ln)]
    if length is None:
        return rowwise(lambda a, st: f(a, st))(s, start)
    return rowwise(f)(s, start, length)


def _rand(seed=None, n=None):
    rng = np.random.default_rng(None if seed is None else int(seed.iloc[0]))
    return pd.Series(rng.random(n))


def _i32(h: int) -> int:
    h &= 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def hive_hash_code(v) -> int:
    """Hive's per-type hash code (``ObjectInspectorUtils.hashCode``): int -> itself, bigint ->
    ``(int)(v ^ v >>> 32)``, double -> ``Double.hashCode``, string -> the 31-polynomial over its
    UTF-8 bytes (signed), boolean -> 1/0, NULL -> 0, arrays -> 31-polynomial of the elements.
    Deterministic across processes (no salted Python hash)."""
    if v is None:
        return 0
    if isinstance(v, (bool, np.bool_)):
        return 1 if v else 0
    if isinstance(v, (int, np.integer)):
        v = int(v)
        if -(1 << 31) <= v < (1 << 31):
            return v
        u = v & 0xFFFFFFFFFFFFFFFF
        return _i32(u ^ (u >> 32))
    if isinstance(v, (float, np.floating)):
        import struct

        u = struct.unpack(">q", struct.pack(">d", float(v)))[0] & 0xFFFFFFFFFFFFFFFF
        return _i32(u ^ (u >> 32))
    if isinstance(v, (list, tuple, np.ndarray)):
        h = 0
        for x in v:
            h = _i32(31 * h + hive_hash_code(x))
        return h
    h = 0
    for b in str(v).encode("utf-8"):
        h = _i32(31 * h + (b - 256 if b > 127 else b))
    return h


def _hash(*cols):
    def f(*vals):
        h = 0
        for v in vals:
            h = _i32(31 * h + hive_hash_code(None if is_null(v) else v))
        return h
    return rowwise(f, null_prop=False)(*cols)


def _greatest(*cols):
    return rowwise(lambda *v: max(v))(*cols)


def _least(*cols):
    return rowwise(lambda *v: min(v))(*cols)


def _array_contains(a, v):
    return rowwise(lambda arr, x: x in list(arr))(a, v)


def _sort_array(a, asc=None):
    return rowwise(lambda arr: sorted(arr))(a)


def _map_keys(m):
    return rowwise(lambda d: list(d.keys()))(m)


def _map_values(m):
    return rowwise(lambda d: list(d.values()))(m)


def _nvl(a, b):
    return _coalesce(a, b)


def _instr(s, sub):
    return rowwise(lambda a, b: str(a).find(str(b)) + 1)(s, sub)


def _get_json_object(s, path):
    def f(js, p):
        obj = json.loads(js)
        for part in str(p).lstrip("$").split("."):
            if not part:
                continue
            m = re.match(r"(\w+)\[(\d+)\]", part)
            if m:
                obj = obj[m.group(1)][int(m.group(2))]
            else:
                obj = obj.get(part) if isinstance(obj, dict) else None
            if obj is None:
                return None
        return obj if not isinstance(obj, (dict, list)) else json.dumps(obj)
    return rowwise(f)(s, path)


# ------------------------------------------------------------------ date / time
# Hive's date functions on 'yyyy-MM-dd[ HH:mm:ss]' strings and Unix seconds.  Times are in UTC
# (Hive uses the session's time zone; a fixed zone keeps query results reproducible).
_JFMT = [("yyyy", "%Y"), ("yy", "%y"), ("MMMM", "%B"), ("MMM", "%b"), ("MM", "%m"), ("dd", "%d"),
         ("HH", "%H"), ("hh", "%I"), ("mm", "%M"), ("ss", "%S"), ("EEEE", "%A"), ("EEE", "%a"),
         ("a", "%p"), ("D", "%j")]
_JFMT_RE = re.compile("|".join(re.escape(j) for j, _ in _JFMT))


def _strftime_fmt(java_fmt: str) -> str:
    """A Java SimpleDateFormat pattern (the subset Hive scripts use) as a strftime format."""
    table = dict(_JFMT)
    return _JFMT_RE.sub(lambda m: table[m.group(0)], str(java_fmt).replace("%", "%%"))


def _ts(v):
    if isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool):
        return pd.Timestamp(int(v), unit="s")
    return pd.Timestamp(str(v))


def _date_col(fn):
    def apply(*cols):
        def f(*vals):
            try:
                return fn(*vals)
            except (ValueError, TypeError, OverflowError):
                return None                      # Hive: unparsable date -> NULL
        return rowwise(f)(*cols)
    return apply


def _from_unixtime(s, fmt=None):
    if fmt is None:
        return _date_col(lambda v: pd.Timestamp(int(v), unit="s").strftime("%Y-%m-%d %H:%M:%S"))(s)
    return _date_col(lambda v, f: pd.Timestamp(int(v), unit="s").strftime(_strftime_fmt(f)))(s, fmt)


def _unix_timestamp(s=None, fmt=None):
    if s is None:
        return pd.Series([int(pd.Timestamp.now(tz="UTC").timestamp())])
    if fmt is None:
        return _date_col(lambda v: int(_ts(v).timestamp()))(s)
    return _date_col(lambda v, f: int(pd.Timestamp(pd.to_datetime(str(v), format=_strftime_fmt(f))).timestamp()))(s, fmt)


def _date_shift(sign):
    return _date_col(lambda d, n: (_ts(d).normalize() + pd.Timedelta(days=sign * int(n))).strftime("%Y-%m-%d"))


SCALAR_DATE = {
    "from_unixtime": _from_unixtime, "unix_timestamp": _unix_timestamp,
    "to_date": _date_col(lambda v: _ts(v).strftime("%Y-%m-%d")),
    "datediff": _date_col(lambda a, b: int((_ts(a).normalize() - _ts(b).normalize()).days)),
    "date_add": _date_shift(1), "date_sub": _date_shift(-1),
    "year": _date_col(lambda v: _ts(v).year), "month": _date_col(lambda v: _ts(v).month),
    "day": _date_col(lambda v: _ts(v).day), "dayofmonth": _date_col(lambda v: _ts(v).day),
    "hour": _date_col(lambda v: _ts(v).hour), "minute": _date_col(lambda v: _ts(v).minute),
    "second": _date_col(lambda v: _ts(v).second),
    "weekofyear": _date_col(lambda v: int(_ts(v).isocalendar()[1])),
    "date_format": _date_col(lambda v, f: _ts(v).strftime(_strftime_fmt(f))),
    "current_date": lambda: pd.Series([pd.Timestamp.now(tz="UTC").strftime("%Y-%m-%d")]),
    "current_timestamp": lambda: pd.Series([pd.Timestamp.now(tz="UTC").strftime("%Y-%m-%d %H:%M:%S")]),
}


SCALAR = {
    "abs": _vec_math(np.abs), "exp": _vec_math(np.exp), "ln": _vec_math(np.log),
    "log10": _vec_math(np.log10), "log2": _vec_math(np.log2), "sqrt": _vec_math(np.sqrt),
    "floor": _vec_math(np.floor), "ceil": _vec_math(np.ceil), "ceiling": _vec_math(np.ceil),
    "sign": _vec_math(np.sign), "signum": _vec_math(np.sign), "sin": _vec_math(np.sin),
    "cos": _vec_math(np.cos), "tan": _vec_math(np.tan), "atan": _vec_math(np.arctan),
    "log": lambda a, b=None: _vec_math(np.log)(a) if b is None else
    pd.Series(np.log(_num(b).to_numpy(dtype=np.float64)) / np.log(_num(a).to_numpy(dtype=np.float64))),
    "pow": lambda a, b: pd.Series(np.power(_num(a).to_numpy(dtype=np.float64), _num(b).to_numpy(dtype=np.float64))),
    "power": lambda a, b: pd.Series(np.power(_num(a).to_numpy(dtype=np.float64), _num(b).to_numpy(dtype=np.float64))),
    "round": _round, "if": _if, "coalesce": _coalesce, "nvl": _nvl, "concat": _concat,
    "concat_ws": _concat_ws, "size": _size, "split": _split, "array": _array, "map": _map,
    "struct": _struct, "named_struct": _named_struct,
    "length": rowwise(lambda a: len(str(a))), "lower": rowwise(lambda a: str(a).lower()),
    "lcase": rowwise(lambda a: str(a).lower()), "upper": rowwise(lambda a: str(a).upper()),
    "ucase": rowwise(lambda a: str(a).upper()), "trim": rowwise(lambda a: str(a).strip()),
    "ltrim": rowwise(lambda a: str(a).lstrip()), "rtrim": rowwise(lambda a: str(a).rstrip()),
    "substr": _substr, "substring": _substr,
    "regexp_replace": rowwise(lambda a, p, r: re.sub(p, re.sub(r"\$(\d)", r"\\\1", str(r)), str(a))),
    "regexp_extract": rowwise(lambda a, p, i=1: (lambda m: m.group(int(i)) if m else "")(re.search(p, str(a)))),
    "rand": None, "hash": _hash, "greatest": _greatest, "least": _least,
    "array_contains": _array_contains, "sort_array": _sort_array, "map_keys": _map_keys,
    "map_values": _map_values, "instr": _instr, "get_json_object": _get_json_object,
    "md5": rowwise(lambda a: hashlib.md5(str(a).encode()).hexdigest()),
    "pmod": rowwise(lambda a, b: a % b), "isnull": lambda a: pd.Series([is_null(v) for v in a.tolist()]),
    "isnotnull": lambda a: pd.Series([not is_null(v) for v in a.tolist()]),
    "nullif": rowwise(lambda a, b: None if a == b else a, null_prop=False),
    "format_number": rowwise(lambda a, d: f"{float(a):,.{int(d)}f}"),
    "ascii": rowwise(lambda a: ord(str(a)[0]) if str(a) else 0),
    "repeat": rowwise(lambda a, n: str(a) * int(n)), "reverse": rowwise(lambda a: str(a)[::-1] if isinstance(a, str) else list(a)[::-1]),
    "space": rowwise(lambda n: " " * int(n)),
    "lpad": rowwise(lambda a, n, p: str(a).rjust(int(n), str(p))[: int(n)]),
    "rpad": rowwise(lambda a, n, p: str(a).ljust(int(n), str(p))[: int(n)]),
    "e": lambda *a: pd.Series([math.e]), "pi": lambda *a: pd.Series([math.pi]),
    "collect_array": None,
    **SCALAR_DATE,
}


# ------------------------------------------------------------------ aggregates
def _vals(c):
    return [v for v in c if not is_null(v)]


def _percentile(c, p):
    v = np.asarray(_vals(c), dtype=np.float64)
    if not v.size:
        return None
    pv = p[0] if isinstance(p, (list, tuple)) else p
    if isinstance(pv, (list, tuple, np.ndarray)):
        return [float(np.percentile(v, 100 * q)) for q in pv]
    return float(np.percentile(v, 100 * float(pv)))


AGGREGATE = {
    "count": lambda *cols: (len(cols[0]) if not cols else
                            sum(1 for vals in zip(*cols) if not any(is_null(x) for x in vals))),
    "sum": lambda c: (lambda v: sum(v) if v else None)(_vals(c)),
    "avg": lambda c: (lambda v: float(np.mean(np.asarray(v, dtype=np.float64))) if v else None)(_vals(c)),
    "mean": lambda c: (lambda v: float(np.mean(np.asarray(v, dtype=np.float64))) if v else None)(_vals(c)),
    "min": lambda c: (lambda v: min(v) if v else None)(_vals(c)),
    "max": lambda c: (lambda v: max(v) if v else None)(_vals(c)),
    "collect_list": lambda c: _vals(c),
    "collect_set": lambda c: list(dict.fromkeys(_vals(c))),
    "stddev": lambda c: (lambda v: float(np.std(v)) if v else None)(_vals(c)),
    "stddev_pop": lambda c: (lambda v: float(np.std(v)) if v else None)(_vals(c)),
    "stddev_samp": lambda c: (lambda v: float(np.std(v, ddof=1)) if len(v) > 1 else None)(_vals(c)),
    "variance": lambda c: (lambda v: float(np.var(v)) if v else None)(_vals(c)),
    "var_pop": lambda c: (lambda v: float(np.var(v)) if v else None)(_vals(c)),
    "var_samp": lambda c: (lambda v: float(np.var(v, ddof=1)) if len(v) > 1 else None)(_vals(c)),
    "percentile": _percentile, "percentile_approx": _percentile,
    "first": lambda c: c[0] if len(c) else None, "first_value": lambda c: c[0] if len(c) else None,
    "last": lambda c: c[-1] if len(c) else None, "last_value": lambda c: c[-1] if len(c) else None,
    "corr": lambda a, b: float(np.corrcoef(np.asarray(a, float), np.asarray(b, float))[0, 1]),
}

# fast pandas paths for the common numeric aggregates
PANDAS_AGG = {"sum": "sum", "avg": "mean", "mean": "mean", "min": "min", "max": "max", "count": "count"}

WINDOW_ONLY = {"row_number", "rank", "dense_rank", "percent_rank", "cume_dist", "ntile", "lag",
               "lead"}


# ------------------------------------------------------------------ table functions
def explode(v):
    if is_null(v):
        return
    if isinstance(v, dict):
        for k, x in v.items():
            yield (k, x)
    else:
        for x in v:
            yield (x,)


def posexplode(v):
    if is_null(v):
        return
    for i, x in enumerate(v):
        yield (i, x)


def inline(v):
    if is_null(v):
        return
    for s in v:
        yield tuple(s.values()) if isinstance(s, dict) else tuple(s)


def stack(n, *vals):
    n = int(n)
    k = len(vals) // n
    for i in range(n):
        yield tuple(vals[i * k:(i + 1) * k])


def json_tuple(js, *keys):
    d = json.loads(js) if not is_null(js) else {}
    yield tuple(None if d.get(k) is None else str(d.get(k)) for k in keys)


TABLE = {"explode": explode, "posexplode": posexplode, "inline": inline, "stack": stack,
         "json_tuple": json_tuple}
TABLE_COLS = {"explode": ("col",), "posexplode": ("pos", "val"), "inline": None, "stack": None,
              "json_tuple": None}
