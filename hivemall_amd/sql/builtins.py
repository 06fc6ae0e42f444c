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


# ------------------------------------------------------------------ more Hive string / math UDFs
def _conv(v, fb, tb):
    """conv(num, from_base, to_base): base conversion of an integer string (Hive: negative
    to_base = signed output; invalid digits end the number)."""
    digits = "0123456789abcdefghijklmnopqrstuvwxyz"
    fb, tb = int(fb), int(tb)
    txt = str(v).strip().lower()
    neg = txt.startswith("-")
    n = 0
    for ch in txt[1:] if neg else txt:
        d = digits.find(ch)
        if d < 0 or d >= abs(fb):
            break
        n = n * abs(fb) + d
    if neg:
        n = -n
    if tb > 0 and n < 0:
        n &= 0xFFFFFFFFFFFFFFFF                 # Hive prints the unsigned 64-bit pattern
    if n == 0:
        return "0"
    out, m = [], abs(n)
    while m:
        out.append(digits[m % abs(tb)])
        m //= abs(tb)
    return ("-" if n < 0 else "") + "".join(reversed(out)).upper()


def _soundex(v):
    s = "".join(c for c in str(v).upper() if c.isalpha())
    if not s:
        return ""
    codes = {**dict.fromkeys("BFPV", "1"), **dict.fromkeys("CGJKQSXZ", "2"), **dict.fromkeys("DT", "3"),
             "L": "4", **dict.fromkeys("MN", "5"), "R": "6"}
    out, prev = s[0], codes.get(s[0], "")
    for c in s[1:]:
        d = codes.get(c, "")
        if d and d != prev:
            out += d
        if c not in "HW":
            prev = d
    return (out + "000")[:4]


def _levenshtein(a, b):
    a, b = str(a), str(b)
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i]
        for j, cb in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
        prev = cur
    return prev[-1]


def _parse_url(url, part, key=None):
    from urllib.parse import parse_qs, urlsplit

    u = urlsplit(str(url))
    p = str(part).upper()
    if p == "QUERY" and key is not None:
        vals = parse_qs(u.query, keep_blank_values=True).get(str(key))
        return vals[0] if vals else None
    return {"HOST": u.hostname, "PATH": u.path, "QUERY": u.query or None, "REF": u.fragment or None,
            "PROTOCOL": u.scheme or None, "FILE": (u.path + ("?" + u.query if u.query else "")) or None,
            "AUTHORITY": u.netloc or None, "USERINFO": (u.netloc.rpartition("@")[0] or None)}.get(p)


def _add_months(d, n):
    t = _ts(d)
    m = t.month - 1 + int(n)
    y, m = t.year + m // 12, m % 12 + 1
    last = pd.Timestamp(year=y, month=m, day=1).days_in_month
    day = last if t.day == t.days_in_month else min(t.day, last)
    return pd.Timestamp(year=y, month=m, day=day).strftime("%Y-%m-%d")


def _months_between(a, b):
    ta, tb = _ts(a), _ts(b)
    if ta.day == tb.day or (ta.day == ta.days_in_month and tb.day == tb.days_in_month):
        return float((ta.year - tb.year) * 12 + ta.month - tb.month)
    secs = lambda t: (t.day - 1) * 86400 + t.hour * 3600 + t.minute * 60 + t.second
    return round((ta.year - tb.year) * 12 + ta.month - tb.month + (secs(ta) - secs(tb)) / (31 * 86400.0), 8)


_DOW = {"MO": 0, "TU": 1, "WE": 2, "TH": 3, "FR": 4, "SA": 5, "SU": 6}


def _next_day(d, dow):
    t = _ts(d).normalize()
    w = _DOW[str(dow).strip().upper()[:2]]
    return (t + pd.Timedelta(days=(w - t.dayofweek - 1) % 7 + 1)).strftime("%Y-%m-%d")


def _trunc_date(d, fmt):
    t = _ts(d)
    f = str(fmt).upper()
    if f in ("MONTH", "MON", "MM"):
        return t.replace(day=1).strftime("%Y-%m-%d")
    if f in ("YEAR", "YYYY", "YY"):
        return t.replace(month=1, day=1).strftime("%Y-%m-%d")
    if f in ("QUARTER", "Q"):
        return t.replace(month=3 * ((t.month - 1) // 3) + 1, day=1).strftime("%Y-%m-%d")
    return None


def _bround(s, d=None):
    dd = 0 if d is None else int(d.iloc[0])
    return pd.Series(np.round(_num(s).to_numpy(dtype=np.float64), dd))      # numpy rounds half-even


def _translate(v, frm, to):
    frm, to = str(frm), str(to)
    table = {}
    for i, c in enumerate(frm):
        if c not in table:
            table[c] = to[i] if i < len(to) else None
    return "".join(table.get(c, c) or "" for c in str(v))


def _printf(fmt, *vals):
    return str(fmt) % tuple(vals)            # Java's %s / %d / %f / %x / %e behave the same


def _sentences(v, *_):
    out = []
    for sent in re.split(r"(?<=[.!?])\s+", str(v).strip()):
        words = re.findall(r"[\w']+", sent)
        if words:
            out.append(words)
    return out


SCALAR_MORE = {
    "conv": rowwise(_conv), "bin": rowwise(lambda a: format(int(a) & 0xFFFFFFFFFFFFFFFF if int(a) < 0 else int(a), "b")),
    "hex": rowwise(lambda a: (format(int(a) & 0xFFFFFFFFFFFFFFFF, "X") if isinstance(a, (int, np.integer))
                              else str(a).encode().hex().upper())),
    "unhex": rowwise(lambda a: bytes.fromhex(str(a)).decode("utf-8", "replace")),
    "base64": rowwise(lambda a: __import__("base64").b64encode(a if isinstance(a, bytes) else str(a).encode()).decode()),
    "unbase64": rowwise(lambda a: __import__("base64").b64decode(str(a)).decode("utf-8", "replace")),
    "decode": rowwise(lambda a, cs: (a if isinstance(a, bytes) else str(a).encode()).decode(str(cs))),
    "encode": rowwise(lambda a, cs: str(a).encode(str(cs))),
    "translate": rowwise(_translate), "initcap": rowwise(lambda a: " ".join(w.capitalize() for w in str(a).split(" "))),
    "levenshtein": rowwise(_levenshtein), "soundex": rowwise(_soundex),
    "str_to_map": rowwise(lambda a, d1=",", d2=":": {k: v for k, _, v in (p.partition(str(d2)) for p in str(a).split(str(d1)))}),
    "find_in_set": rowwise(lambda a, lst: (str(lst).split(",").index(str(a)) + 1) if "," not in str(a) and str(a) in str(lst).split(",") else 0),
    "locate": rowwise(lambda sub, a, pos=1: str(a).find(str(sub), int(pos) - 1) + 1),
    "field": rowwise(lambda a, *xs: next((i + 1 for i, x in enumerate(xs) if x == a), 0), null_prop=False),
    "elt": rowwise(lambda n, *xs: xs[int(n) - 1] if 1 <= int(n) <= len(xs) else None),
    "char_length": rowwise(lambda a: len(str(a))), "character_length": rowwise(lambda a: len(str(a))),
    "octet_length": rowwise(lambda a: len(str(a).encode("utf-8"))),
    "parse_url": rowwise(_parse_url), "sentences": rowwise(_sentences),
    "printf": rowwise(_printf), "sha2": rowwise(lambda a, bits: hashlib.new(f"sha{int(bits) if int(bits) != 0 else 256}", str(a).encode()).hexdigest()),
    "crc32": rowwise(lambda a: __import__("zlib").crc32(str(a).encode())),
    "factorial": rowwise(lambda a: math.factorial(int(a)) if 0 <= int(a) <= 20 else None),
    "bround": _bround, "cbrt": _vec_math(np.cbrt), "degrees": _vec_math(np.degrees),
    "radians": _vec_math(np.radians), "asin": _vec_math(np.arcsin), "acos": _vec_math(np.arccos),
    "shiftleft": rowwise(lambda a, n: _i32(int(a) << int(n))), "shiftright": rowwise(lambda a, n: int(a) >> int(n)),
    "positive": rowwise(lambda a: a), "negative": rowwise(lambda a: -a), "mod": rowwise(lambda a, b: math.fmod(a, b) if isinstance(a, float) or isinstance(b, float) else int(math.fmod(a, b))),
    "quarter": _date_col(lambda v: (_ts(v).month - 1) // 3 + 1),
    "last_day": _date_col(lambda v: _ts(v).replace(day=_ts(v).days_in_month).strftime("%Y-%m-%d")),
    "add_months": _date_col(_add_months), "months_between": _date_col(_months_between),
    "next_day": _date_col(_next_day), "trunc": _date_col(_trunc_date),
    "current_user": lambda: pd.Series([__import__("getpass").getuser()]),
    "current_database": lambda: pd.Series(["default"]),
    "uuid": lambda: pd.Series([str(__import__("uuid").uuid4())]),
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
    **SCALAR_MORE,
}


# ------------------------------------------------------------------ aggregates
def _vals(c):
    return [v for v in c if not is_null(v)]


def _pairs(a, b):
    """The (a, b) pairs with neither side NULL, as float arrays (Hive's bivariate aggregates)."""
    keep = [(x, y) for x, y in zip(a, b) if not is_null(x) and not is_null(y)]
    if not keep:
        return None
    arr = np.asarray(keep, dtype=np.float64)
    return arr[:, 0], arr[:, 1]


def _covar(a, b, ddof):
    p = _pairs(a, b)
    if p is None or len(p[0]) <= ddof:
        return None
    return float(np.cov(p[0], p[1], ddof=ddof)[0, 1]) if len(p[0]) > 1 else 0.0


def _histogram_numeric(c, nb):
    """histogram_numeric(col, b): b (x, y) bin centres and heights, built as Hive does — one
    bin per value, the two closest bins merged until b remain (Ben-Haim & Tom-Tov)."""
    b = int(nb[0]) if isinstance(nb, (list, tuple, pd.Series)) else int(nb)
    bins: list = []
    for v in sorted(float(x) for x in _vals(c)):
        if bins and bins[-1][0] == v:
            bins[-1][1] += 1.0
        else:
            bins.append([v, 1.0])
    while len(bins) > b:
        i = min(range(len(bins) - 1), key=lambda k: bins[k + 1][0] - bins[k][0])
        (x1, y1), (x2, y2) = bins[i], bins[i + 1]
        bins[i:i + 2] = [[(x1 * y1 + x2 * y2) / (y1 + y2), y1 + y2]]
    return [{"x": x, "y": y} for x, y in bins]


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
    "covar_pop": lambda a, b: _covar(a, b, 0), "covar_samp": lambda a, b: _covar(a, b, 1),
    "regr_slope": lambda y, x: (lambda p: None if p is None or p[1].var() == 0 else
                                float(np.cov(p[0], p[1], ddof=0)[0, 1] / p[1].var()))(_pairs(y, x)),
    "regr_intercept": lambda y, x: (lambda p: None if p is None or p[1].var() == 0 else
                                    float(p[0].mean() - np.cov(p[0], p[1], ddof=0)[0, 1] / p[1].var() * p[1].mean()))(_pairs(y, x)),
    "histogram_numeric": lambda c, nb: _histogram_numeric(c, nb),
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


def parse_url_tuple(url, *parts):
    if is_null(url):
        yield tuple(None for _ in parts)
        return
    out = []
    for p in parts:
        p = str(p)
        if p.upper().startswith("QUERY:"):
            out.append(_parse_url(url, "QUERY", p.split(":", 1)[1]))
        else:
            out.append(_parse_url(url, p))
    yield tuple(out)


TABLE = {"explode": explode, "posexplode": posexplode, "inline": inline, "stack": stack,
         "json_tuple": json_tuple, "parse_url_tuple": parse_url_tuple}
TABLE_COLS = {"explode": ("col",), "posexplode": ("pos", "val"), "inline": None, "stack": None,
              "json_tuple": None, "parse_url_tuple": None}
