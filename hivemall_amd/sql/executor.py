"""HiveQL executor over pandas tables — the SQL frontend that lets Hivemall scripts run on
this engine.

A :class:`Session` holds named tables (pandas DataFrames), ``SET`` variables, macros and the
function registry.  Statements: SELECT (joins, LATERAL VIEW, GROUP BY/HAVING, window
functions, ORDER/SORT/CLUSTER BY, LIMIT, UNION ALL, CTEs, subqueries), CREATE TABLE [AS],
CREATE VIEW, INSERT OVERWRITE/INTO, DROP, CREATE TEMPORARY FUNCTION/MACRO, SET, ADD JAR /
SOURCE (accepted), SHOW FUNCTIONS, DESCRIBE FUNCTION; files come in through ``CREATE [EXTERNAL]
TABLE ... [ROW FORMAT DELIMITED ...] [STORED AS ...] LOCATION '...'`` and ``LOAD DATA [LOCAL]
INPATH`` and go out through ``INSERT OVERWRITE [LOCAL] DIRECTORY`` (io/tables.py: Hive text,
parquet, libsvm, jsonl).  Learner UDTFs (``train_*``) execute on
the session's device (``SET hivemall.device=cuda``) through the gfx950 kernels.
"""
from __future__ import annotations

import fnmatch
import itertools
import logging
import math
import os
import re
from dataclasses import dataclass, replace

import numpy as np
import pandas as pd

from .. import registry
from . import builtins as B
from .lexer import split_statements
from .parser import (Between, BinOp, Case, Cast, Col, CreateFunction, CreateMacro, CreateTable,
                     DescribeFunction, Drop, Exists, Expr, Field, Func, Index, InList, Insert,
                     InsertDirectory, IsNull, Join, LateralView, Like, Lit, LoadData, MultiInsert, NoOp, Query, RenameTable,
                     Select, SelectItem, SetStmt, ShowTables, DescribeTable,
                     ShowFunctions, Star, SubqueryExpr, SubqueryRef, TableRef, Truncate, UnOp, Union, parse)


# Hivemall classes whose function name is not the snake_case of the class name
_HIVEMALL_CLASSES = {
    "GeneralClassifierUDTF": "train_classifier", "GeneralRegressorUDTF": "train_regressor",
    "GeneralRegressionUDTF": "train_regressor", "FactorizationMachineUDTF": "train_fm",
    "FieldAwareFactorizationMachineUDTF": "train_ffm", "FMPredictGenericUDAF": "fm_predict",
    "FFMPredictGenericUDAF": "ffm_predict", "FFMPredictUDF": "ffm_predict",
    "RandomForestClassifierUDTF": "train_randomforest_classifier",
    "RandomForestRegressionUDTF": "train_randomforest_regressor",
    "GradientTreeBoostingClassifierUDTF": "train_gradient_tree_boosting_classifier",
    "TreePredictUDF": "tree_predict", "RandomForestEnsembleUDAF": "rf_ensemble",
    "MurmurHash3UDF": "mhash", "LogressUDTF": "logress", "AdaGradRDAUDTF": "train_adagrad_rda",
    "PerceptronUDTF": "train_perceptron", "PassiveAggressiveUDTF": "train_pa",
    "AROWClassifierUDTF": "train_arow", "ConfidenceWeightedUDTF": "train_cw",
    "BPRMatrixFactorizationUDTF": "train_bprmf", "MatrixFactorizationSGDUDTF": "train_mf_sgd",
    "MatrixFactorizationAdaGradUDTF": "train_mf_adagrad", "LDAUDTF": "train_lda",
    "PLSAUDTF": "train_plsa", "SigmoidGenericUDF": "sigmoid", "AUCUDAF": "auc",
    "LogarithmicLossUDAF": "logloss", "L2NormalizationUDF": "l2_normalize",
    "L1NormalizationUDF": "l1_normalize", "XGBoostClassifierUDTF": "train_xgboost_classifier",
    "XGBoostRegressionUDTF": "train_xgboost_regr", "XGBoostTrainUDTF": "train_xgboost",
}


def _resolve_function_class(cls: str) -> str | None:
    """Registry name behind a CREATE TEMPORARY FUNCTION class: one of this engine's own
    implementations (define-all.hive names them), or a Hivemall class by its simple name."""
    for name in registry.names():
        impl = registry.REGISTRY[name].impl
        if f"{getattr(impl, '__module__', '')}.{getattr(impl, '__qualname__', '')}" == cls:
            return name
    simple = cls.rsplit(".", 1)[-1]
    if simple in _HIVEMALL_CLASSES and registry.lookup(_HIVEMALL_CLASSES[simple]) is not None:
        return _HIVEMALL_CLASSES[simple]
    base = re.sub(r"(Generic)?(UDTF|UDAF|UDF)$", "", simple)
    snake = re.sub(r"(?<=[a-z0-9])(?=[A-Z])|(?<=[A-Z])(?=[A-Z][a-z])", "_", base).lower()
    for cand in (snake, "train_" + snake):
        if registry.lookup(cand) is not None:
            return cand
    return None


def _hive_type(col: pd.Series) -> str:
    """Hive type name of a table column (DESCRIBE)."""
    dt = col.dtype
    if isinstance(dt, pd.ArrowDtype):
        import pyarrow as pa

        t = dt.pyarrow_dtype
        if pa.types.is_list(t) or pa.types.is_large_list(t):
            inner = t.value_type
            return "array<" + ("string" if pa.types.is_string(inner) or pa.types.is_large_string(inner)
                               else "double" if pa.types.is_floating(inner) else
                               "bigint" if pa.types.is_integer(inner) else str(inner)) + ">"
        return "string" if pa.types.is_string(t) or pa.types.is_large_string(t) else str(t)
    if pd.api.types.is_bool_dtype(dt):
        return "boolean"
    if pd.api.types.is_integer_dtype(dt):
        return "bigint" if dt.itemsize >= 8 else "int"
    if pd.api.types.is_float_dtype(dt):
        return "double" if dt.itemsize >= 8 else "float"
    first = next((v for v in col if v is not None and not (isinstance(v, float) and v != v)), None)
    if isinstance(first, (list, tuple, np.ndarray)):
        inner = next((x for x in first if x is not None), None)
        return "array<" + ("string" if isinstance(inner, str) else "double" if isinstance(inner, float)
                           else "bigint" if isinstance(inner, (int, np.integer)) else "string") + ">"
    if isinstance(first, dict):
        return "map<string,double>"
    return "string"


# UDFs that see NULL arguments themselves (everything else: NULL first argument -> NULL)
_NULL_AWARE_UDFS = frozenset({"assert", "raise_error", "sessionize", "rowid", "rownum", "taskid"})


log = logging.getLogger("hivemall_amd.sql")


class SQLError(Exception):
    pass


# ------------------------------------------------------------------ frames
@dataclass
class Frame:
    df: pd.DataFrame            # columns are positional c0..cN
    cols: list                  # [(qualifier|None, name)]

    @staticmethod
    def from_df(df: pd.DataFrame, qualifier: str | None = None) -> "Frame":
        d = df.copy()
        names = [str(c) for c in d.columns]
        d.columns = [f"c{i}" for i in range(len(names))]
        d = d.reset_index(drop=True)
        return Frame(d, [(qualifier, n) for n in names])

    @property
    def n(self) -> int:
        return len(self.df)

    def series(self, i: int) -> pd.Series:
        return self.df[f"c{i}"]

    def requalify(self, q: str | None) -> "Frame":
        return Frame(self.df, [(q, n) for _, n in self.cols])

    def resolve(self, name: str, table: str | None) -> int | None:
        lname = name.lower()
        hits = [i for i, (q, n) in enumerate(self.cols)
                if n.lower() == lname and (table is None or (q is not None and q.lower() == table.lower()))]
        if not hits:
            return None
        if len(hits) > 1 and table is None:
            quals = {self.cols[i][0] for i in hits}
            if len(quals) > 1:
                raise SQLError(f"ambiguous column reference '{name}' ({', '.join(str(q) for q in quals)})")
        return hits[0]

    def to_df(self) -> pd.DataFrame:
        d = self.df.copy()
        d.columns = [n for _, n in self.cols]
        return d

    def take(self, idx) -> "Frame":
        return Frame(self.df.iloc[idx].reset_index(drop=True), list(self.cols))

    @staticmethod
    def concat_cols(a: "Frame", b: "Frame") -> "Frame":
        da = a.df.reset_index(drop=True)
        db = b.df.reset_index(drop=True)
        db.columns = [f"c{i + len(a.cols)}" for i in range(len(b.cols))]
        return Frame(pd.concat([da, db], axis=1), a.cols + b.cols)


def _ser(v, n: int) -> pd.Series:
    if isinstance(v, pd.Series):
        return v.reset_index(drop=True)
    if isinstance(v, np.ndarray):
        return pd.Series(list(v) if v.ndim > 1 else v)
    if isinstance(v, (list, tuple, dict)):
        return pd.Series([v] * n, dtype=object)
    return pd.Series([v] * n, dtype=object if isinstance(v, str) or v is None else None)


def _running_agg(name: str, vals, m: int) -> list:
    """Prefix sum / count / avg / min / max over a sorted partition, NULLs skipped."""
    out, cnt, acc = [], 0, None
    for r in range(m):
        v = None if vals is None else vals[r]
        if vals is None or not B.is_null(v):
            cnt += 1
            if vals is not None:
                if acc is None:
                    acc = v
                elif name in ("sum", "avg"):
                    acc = acc + v
                elif name == "min":
                    acc = min(acc, v)
                elif name == "max":
                    acc = max(acc, v)
        if name == "count":
            out.append(cnt)
        elif name == "avg":
            out.append(None if acc is None else float(acc) / cnt)
        else:
            out.append(acc)
    return out


def _peer_bounds(okey: list):
    """First / last index of each row's peer group (equal ORDER BY keys) in a sorted partition."""
    m = len(okey)
    lo, hi = [0] * m, [0] * m
    start = 0
    for r in range(1, m + 1):
        if r == m or okey[r] != okey[start]:
            for q in range(start, r):
                lo[q], hi[q] = start, r - 1
            start = r
    return lo, hi


def _frame_rows(frame, r: int, m: int, peers, pos) -> tuple[int, int]:
    """Inclusive row range [a, b] of row r's window frame in a sorted partition of m rows.
    ROWS counts rows; RANGE takes whole peer groups (CURRENT ROW) or, with an offset, the
    rows whose ORDER BY value lies within it (``pos``: the key in sort direction)."""
    unit, lo, hi = frame
    if unit == "rows":
        return (0 if lo is None else max(0, r + lo)), (m - 1 if hi is None else min(m - 1, r + hi))
    if pos is None:
        return (0 if lo is None else peers[0][r]), (m - 1 if hi is None else peers[1][r])
    x = pos[r]
    a = 0 if lo is None else next((q for q in range(m) if pos[q] >= x + lo), m)
    b = m - 1 if hi is None else max((q for q in range(m) if pos[q] <= x + hi), default=-1)
    return a, b


def _null_out(e, targets: list):
    """``e`` with every sub-expression equal to one of ``targets`` replaced by NULL."""
    if any(e == t for t in targets):
        return Lit(None)
    if isinstance(e, Expr) and hasattr(e, "__dataclass_fields__"):
        ch = {}
        for f, v in vars(e).items():
            if isinstance(v, Expr):
                ch[f] = _null_out(v, targets)
            elif isinstance(v, list):
                ch[f] = [_null_out(x, targets) if isinstance(x, Expr) else
                         (tuple(_null_out(y, targets) if isinstance(y, Expr) else y for y in x)
                          if isinstance(x, tuple) else x) for x in v]
        return replace(e, **ch) if ch else e
    return e


def _has_star_arg(e) -> bool:
    return isinstance(e, Func) and any(isinstance(a, Star) or _has_star_arg(a) for a in e.args)


def _expand_star_args(e, src: "Frame"):
    """``f(x, *)`` -> ``f(x, c1, c2, ...)`` over the source's visible columns (``t.*``: those of
    table alias ``t``), in order, as Hive passes them."""
    if not isinstance(e, Func):
        return e
    args = []
    for a in e.args:
        if isinstance(a, Star):
            cols = [(q, n) for q, n in src.cols if n != "__dummy__" and (a.table is None or q == a.table)]
            if not cols:
                raise SQLError(f"{a.table or ''}.* matches no column")
            args.extend(Col(n, q) for q, n in cols)
        else:
            args.append(_expand_star_args(a, src))
    return replace(e, args=args)


def _hashable(v):
    if isinstance(v, (list, np.ndarray)):
        return tuple(_hashable(x) for x in v)
    if isinstance(v, dict):
        return tuple(sorted((k, _hashable(x)) for k, x in v.items()))
    if isinstance(v, float) and math.isnan(v):
        return None
    return v


def _truthy(s: pd.Series) -> np.ndarray:
    return np.array([bool(v) if not B.is_null(v) else False for v in s.tolist()], dtype=bool)


_TYPE_CAST = {
    "int": int, "integer": int, "bigint": int, "smallint": int, "tinyint": int,
    "double": float, "float": float, "decimal": float, "string": str, "varchar": str,
    "char": str, "boolean": bool,
}


def _cast_value(v, ty: str):
    if B.is_null(v):
        return None
    base = re.split(r"[<(]", ty)[0]
    if base.startswith("array"):
        inner = ty[ty.find("<") + 1:ty.rfind(">")] if "<" in ty else "string"
        return [_cast_value(x, inner) for x in v]
    if base.startswith("map"):
        return dict(v)
    f = _TYPE_CAST.get(base)
    if f is None:
        return v
    try:
        if f is int:
            return int(float(v)) if not isinstance(v, str) or re.match(r"^\s*-?\d+(\.\d*)?\s*$", v) else None
        if f is bool:
            return v if isinstance(v, bool) else (str(v).lower() == "true" if isinstance(v, str) else bool(v))
        return f(v)
    except (TypeError, ValueError):
        return None


def _like_to_regex(p: str) -> str:
    out = []
    for ch in p:
        if ch == "%":
            out.append(".*")
        elif ch == "_":
            out.append(".")
        else:
            out.append(re.escape(ch))
    return "^" + "".join(out) + "$"


def _contains_agg(e, session) -> bool:
    if isinstance(e, Func):
        if e.window is None and session.is_aggregate(e.name):
            return True
        return any(_contains_agg(a, session) for a in e.args)
    for ch in _children(e):
        if _contains_agg(ch, session):
            return True
    return False


def _children(e):
    if isinstance(e, BinOp):
        return [e.left, e.right]
    if isinstance(e, UnOp):
        return [e.operand]
    if isinstance(e, Func):
        return list(e.args)
    if isinstance(e, Case):
        out = [] if e.base is None else [e.base]
        for c, v in e.whens:
            out += [c, v]
        return out + ([] if e.default is None else [e.default])
    if isinstance(e, Cast):
        return [e.expr]
    if isinstance(e, InList):
        return [e.expr] + list(e.items)
    if isinstance(e, Between):
        return [e.expr, e.lo, e.hi]
    if isinstance(e, (IsNull,)):
        return [e.expr]
    if isinstance(e, Like):
        return [e.expr, e.pattern]
    if isinstance(e, Index):
        return [e.base, e.index]
    if isinstance(e, Field):
        return [e.base]
    return []


def _collect_aggs(e, session, out: list):
    if isinstance(e, Func) and e.window is None and session.is_aggregate(e.name):
        out.append(e)
        return
    for ch in _children(e):
        _collect_aggs(ch, session, out)


def _collect_windows(e, out: list):
    if isinstance(e, Func) and e.window is not None:
        out.append(e)
        return
    for ch in _children(e):
        _collect_windows(ch, out)


def _expr_name(e, i: int) -> str:
    if isinstance(e, Col):
        return e.name
    if isinstance(e, Field):
        return e.name
    return f"_c{i}"


# ------------------------------------------------------------------ session
class Session:
    """A HiveQL session.  Under ``torch.distributed`` (one process per GPU, world > 1) every rank
    runs the same script over the same (replicated) tables, and the learner UDTFs train data-
    parallel: each rank takes its 1/world of the UDTF's input rows and the replicas are mixed over
    RCCL (the mappers + MixServer of a Hive job), so every rank materialises the same model table
    and every later query returns the same global result on every rank.
    ``distributed=False`` keeps a session rank-local."""

    def __init__(self, device=None, distributed: bool | None = None):
        self.ctx = None
        self._prebuilt = {}          # Join id -> (L, R) frames already built by the fused path
        self.last_plan = None        # "fused_join_predict" when the last GROUP BY ran fused
        if distributed is not False:
            import torch.distributed as tdist

            if tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1:
                from ..parallel.dist import context

                self.ctx = context()
            elif distributed:
                raise SQLError("Session(distributed=True) needs an initialised process group")
        self.tables: dict[str, pd.DataFrame] = {}
        self.table_meta: dict[str, dict] = {}    # declared columns / types / ROW FORMAT of CREATE TABLE
        self.views: dict[str, Query] = {}
        self.vars: dict[str, str] = {}
        self.macros: dict[str, tuple] = {}
        self.functions_declared: dict[str, str] = {}
        self.function_aliases: dict[str, str] = {}   # CREATE TEMPORARY FUNCTION alias -> registry name
        if device is not None:
            self.vars["hivemall.device"] = str(device)
        registry.load_all()

    # -- public API
    def _lookup(self, name: str):
        """Registry entry of a function name, through CREATE TEMPORARY FUNCTION aliases."""
        fd = registry.lookup(name)
        if fd is None:
            target = self.function_aliases.get(name.lower())
            if target is not None:
                fd = registry.lookup(target)
        return fd

    def register(self, name: str, df: pd.DataFrame) -> None:
        self.tables[name.lower()] = df.reset_index(drop=True)

    def table(self, name: str) -> pd.DataFrame:
        n = name.lower()
        if n in self.tables:
            return self.tables[n]
        if n.split(".")[-1] in self.tables:
            return self.tables[n.split(".")[-1]]
        raise SQLError(f"Table not found: {name}")

    def sql(self, text: str) -> pd.DataFrame | None:
        """Execute one or more ``;``-separated statements; returns the last result."""
        out = None
        for stmt in split_statements(self._substitute(text)):
            out = self.execute(stmt)
        return out

    def execute(self, stmt: str):
        ast = parse(stmt)
        return self._exec(ast)

    def run_script(self, path: str):
        with open(path) as f:
            return self.sql(f.read())

    @property
    def device(self):
        return self.vars.get("hivemall.device")

    def _substitute(self, text: str) -> str:
        def rep(m):
            key = m.group(1)
            for k in (key, "hivevar:" + key, "hiveconf:" + key):
                if k in self.vars:
                    return self.vars[k]
            return m.group(0)
        return re.sub(r"\$\{(?:hivevar:|hiveconf:)?([^}]+)\}", rep, text)

    def is_aggregate(self, name: str) -> bool:
        n = name.lower()
        if n in self.macros:
            return False
        fd = self._lookup(n)
        if fd is not None:
            return fd.kind == registry.UDAF
        return n in B.AGGREGATE

    # -- statements
    def _exec(self, ast):
        if isinstance(ast, tuple) and ast[0] == "explain":
            return pd.DataFrame({"plan": [repr(ast[1])]})
        if isinstance(ast, Query):
            return self.run_query(ast).to_df()
        if isinstance(ast, CreateTable):
            name = ast.name.lower()
            if ast.if_not_exists and (name in self.tables or name in self.views):
                return None
            if ast.view:
                self.views[name] = ast.query
                self.tables.pop(name, None)
                return None
            self.views.pop(name, None)
            if ast.like:
                src = ast.like.lower()
                base = self.run_query(self.views[src]).to_df() if src in self.views else self.table(src)
                self.tables[name] = base.iloc[:0].reset_index(drop=True)
                if src in self.table_meta:
                    self.table_meta[name] = dict(self.table_meta[src])
                return None
            if ast.query is None and ast.storage.get("location"):
                # CREATE [EXTERNAL] TABLE ... LOCATION '<file or directory>' (io/tables.py)
                from ..io.tables import read_table

                st = ast.storage
                self.tables[name] = read_table(st["location"], st.get("stored_as"), ast.columns or None,
                                               ast.types or None, st.get("field_delim"),
                                               st.get("collection_delim")).reset_index(drop=True)
                self.table_meta[name] = dict(columns=ast.columns, types=ast.types, storage=dict(st))
            elif ast.query is None:
                self.tables[name] = pd.DataFrame({c: pd.Series(dtype=object) for c in ast.columns})
                self.table_meta[name] = dict(columns=ast.columns, types=ast.types, storage=dict(ast.storage))
            else:
                self.tables[name] = self.run_query(ast.query).to_df()
            return None
        if isinstance(ast, Insert):
            name = ast.table.lower()
            if isinstance(ast.query.body, tuple) and ast.query.body[0] == "values":
                rows = [[self.eval_const(e) for e in r] for r in ast.query.body[1]]
                cols = list(self.tables[name].columns) if name in self.tables else \
                    [f"col{i + 1}" for i in range(len(rows[0]))]
                df = pd.DataFrame(rows, columns=cols)
            else:
                df = self.run_query(ast.query).to_df()
            if name in self.tables and len(self.tables[name].columns) == len(df.columns):
                df.columns = list(self.tables[name].columns)
            if ast.overwrite or name not in self.tables:
                self.tables[name] = df.reset_index(drop=True)
            else:
                self.tables[name] = pd.concat([self.tables[name], df], ignore_index=True)
            return None
        if isinstance(ast, LoadData):
            # LOAD DATA [LOCAL] INPATH '<path>' [OVERWRITE] INTO TABLE t: the file is read with
            # t's declared columns, types and ROW FORMAT
            from ..io.tables import read_table

            name = ast.table.lower()
            meta = self.table_meta.get(name, {})
            st = meta.get("storage", {})
            cols = meta.get("columns") or (list(self.tables[name].columns) if name in self.tables else None)
            df = read_table(ast.path, st.get("stored_as"), cols or None, meta.get("types") or None,
                            st.get("field_delim"), st.get("collection_delim"))
            if ast.overwrite or name not in self.tables or len(self.tables[name]) == 0:
                self.tables[name] = df.reset_index(drop=True)
            else:
                self.tables[name] = pd.concat([self.tables[name], df], ignore_index=True)
            return None
        if isinstance(ast, InsertDirectory):
            from ..io.tables import write_table

            st = ast.storage
            write_table(self.run_query(ast.query).to_df(), ast.path, st.get("stored_as"),
                        st.get("field_delim"), st.get("collection_delim"), overwrite_dir=True)
            return None
        if isinstance(ast, Drop):
            n = ast.name.lower()
            if ast.what in ("table", "view"):
                if n not in self.tables and n not in self.views and not ast.if_exists:
                    raise SQLError(f"Table not found: {ast.name}")
                self.tables.pop(n, None)
                self.views.pop(n, None)
            elif ast.what == "function":
                self.functions_declared.pop(n, None)
            elif ast.what == "macro":
                self.macros.pop(n, None)
            return None
        if isinstance(ast, CreateFunction):
            n = ast.name.lower()
            self.functions_declared[n] = ast.class_name
            if registry.lookup(n) is None:
                target = _resolve_function_class(ast.class_name)
                if target is None:
                    # as Hive with the class missing from the classpath, except that the script
                    # goes on (a define-all.hive may name functions the script never calls)
                    log.warning("CREATE TEMPORARY FUNCTION %s: no implementation of '%s'; calls "
                                "to %s will fail", ast.name, ast.class_name, ast.name)
                else:
                    self.function_aliases[n] = target
            return None
        if isinstance(ast, CreateMacro):
            self.macros[ast.name.lower()] = (ast.params, ast.body)
            return None
        if isinstance(ast, SetStmt):
            if ast.key is None:
                return pd.DataFrame({"set": [f"{k}={v}" for k, v in self.vars.items()]})
            if ast.value is None:
                return pd.DataFrame({"set": [f"{ast.key}={self.vars.get(ast.key, '<undefined>')}"]})
            self.vars[ast.key] = ast.value
            return None
        if isinstance(ast, NoOp):
            return None
        if isinstance(ast, MultiInsert):
            for ins in ast.inserts:
                self._exec(ins)
            return None
        if isinstance(ast, Truncate):
            n = ast.table.lower()
            if n not in self.tables:
                raise SQLError(f"Table not found: {ast.table}")
            self.tables[n] = self.tables[n].iloc[:0].reset_index(drop=True)
            return None
        if isinstance(ast, RenameTable):
            o, n = ast.old.lower(), ast.new.lower()
            if n in self.tables or n in self.views:
                raise SQLError(f"Table already exists: {ast.new}")
            if o in self.tables:
                self.tables[n] = self.tables.pop(o)
                if o in self.table_meta:
                    self.table_meta[n] = self.table_meta.pop(o)
            elif o in self.views:
                self.views[n] = self.views.pop(o)
            else:
                raise SQLError(f"Table not found: {ast.old}")
            return None
        if isinstance(ast, ShowFunctions):
            names = registry.names() + sorted(set(B.SCALAR) | set(B.AGGREGATE) | set(B.TABLE))
            if ast.pattern:
                pat = ast.pattern.replace("*", ".*")
                names = [n for n in names if re.fullmatch(pat, n)]
            return pd.DataFrame({"tab_name": sorted(set(names))})
        if isinstance(ast, ShowTables):
            names = sorted(set(self.tables) | set(self.views))
            if ast.pattern:
                pat = ast.pattern.replace("*", ".*")
                names = [n for n in names if re.fullmatch(pat, n)]
            return pd.DataFrame({"tab_name": names})
        if isinstance(ast, DescribeTable):
            n = ast.name.lower()
            meta = self.table_meta.get(n, {})
            if n in self.views:
                df = self.run_query(self.views[n]).to_df().head(0)
            else:
                df = self.table(ast.name)
            declared = dict(zip(meta.get("columns") or [], meta.get("types") or []))
            return pd.DataFrame({"col_name": list(df.columns),
                                 "data_type": [declared.get(c) or _hive_type(df[c]) for c in df.columns]})
        if isinstance(ast, DescribeFunction):
            fd = self._lookup(ast.name)
            if fd is None:
                return pd.DataFrame({"tab_name": [f"Function '{ast.name}' does not exist."]})
            return pd.DataFrame({"tab_name": [f"{fd.name} ({fd.kind}): {fd.doc or ''}"]})
        raise SQLError(f"unsupported statement {type(ast).__name__}")

    # -- queries
    def run_query(self, q: Query, outer_ctes: dict | None = None) -> Frame:
        ctes = dict(outer_ctes or {})
        for name, cq in q.ctes:
            ctes[name.lower()] = self.run_query(cq, ctes).to_df()
        return self._run_body(q.body, ctes)

    def _run_body(self, body, ctes) -> Frame:
        if isinstance(body, Query):
            return self.run_query(body, ctes)
        if isinstance(body, Union):
            frames = [self._run_body(p, ctes) for p in body.parts]
            ncols = len(frames[0].cols)
            dfs = []
            for f in frames:
                if len(f.cols) != ncols:
                    raise SQLError("UNION ALL: column count mismatch")
                dfs.append(f.df.set_axis([f"c{i}" for i in range(ncols)], axis=1))
            df = pd.concat(dfs, ignore_index=True)
            fr = Frame(df, [(None, n) for _, n in frames[0].cols])
            if not body.all:
                fr = fr.take(self._distinct_index(fr))
            if body.order_by:
                fr = self._order(fr, fr, body.order_by, ctes)
            if body.limit is not None:
                fr = fr.take(np.arange(min(body.offset, fr.n), min(body.offset + body.limit, fr.n)))
            return fr
        return self.run_select(body, ctes)

    def _source(self, src, ctes) -> Frame:
        if src is None:
            return Frame(pd.DataFrame({"c0": [0]}), [(None, "__dummy__")])
        if isinstance(src, TableRef):
            n = src.name.lower()
            alias = src.alias or src.name.split(".")[-1]
            if n in ctes:
                fr = Frame.from_df(ctes[n], alias)
            elif n in self.views:
                fr = self.run_query(self.views[n], ctes).requalify(alias)
            else:
                fr = Frame.from_df(self.table(n), alias)
            return self._sample(fr, src.sample, ctes) if src.sample else fr
        if isinstance(src, SubqueryRef):
            fr = self.run_query(src.query, ctes).requalify(src.alias)
            return self._sample(fr, src.sample, ctes) if src.sample else fr
        if isinstance(src, Join):
            return self._join(src, ctes)
        if isinstance(src, LateralView):
            return self._lateral(src, ctes)
        raise SQLError(f"bad FROM item {src}")

    def _sample(self, fr: Frame, spec: tuple, ctes) -> Frame:
        """TABLESAMPLE.  BUCKET x OUT OF y ON expr keeps the rows whose Hive hash of expr is
        x - 1 mod y (``ON rand()`` a seeded random split; no ON: by row position, as for a
        table without buckets).  n PERCENT / n ROWS keep a prefix (Hive samples whole input
        splits, so its rows are a prefix of each split too)."""
        kind = spec[0]
        if kind == "rows":
            return fr.take(np.arange(min(spec[1], fr.n)))
        if kind == "percent":
            return fr.take(np.arange(min(fr.n, int(math.ceil(fr.n * spec[1] / 100.0)))))
        _, x, y, on = spec
        if on is None:
            h = np.arange(fr.n, dtype=np.int64)
        else:
            h = np.array([B.hive_hash_code(None if B.is_null(v) else v)
                          for v in _ser(self.eval(on, fr, ctes), fr.n).tolist()], dtype=np.int64)
            h = h & 0x7FFFFFFF
        return fr.take(np.nonzero(h % y == x - 1)[0])

    # -- joins
    def _split_conj(self, e):
        if isinstance(e, BinOp) and e.op == "and":
            return self._split_conj(e.left) + self._split_conj(e.right)
        return [e]

    def _refs_only(self, e, fr: Frame) -> bool:
        if isinstance(e, Col):
            try:
                return fr.resolve(e.name, e.table) is not None
            except SQLError:
                return True
        if isinstance(e, (Lit,)):
            return True
        ch = _children(e)
        return all(self._refs_only(c, fr) for c in ch) if ch else not isinstance(e, (SubqueryExpr, Exists))

    def _exists(self, e: Exists, fr: Frame, ctes, vals) -> pd.Series:
        """[NOT] EXISTS (subquery).  Uncorrelated: one run.  Correlated through equality
        conjuncts ``inner_expr = outer_expr`` in the subquery's WHERE (Hive's supported form): a
        semi-join — the subquery runs once without them, projecting the inner keys, and each
        outer row looks its key tuple up."""
        body = e.query.body
        if not isinstance(body, Select) or body.source is None:
            return _ser(self.run_query(e.query, ctes).n > 0, fr.n)
        qctes = dict(ctes)
        for name, q in e.query.ctes:
            qctes[name.lower()] = self.run_query(q, qctes)
        inner = self._source(body.source, qctes)
        keep, ikeys, okeys = [], [], []
        for c in (self._split_conj(body.where) if body.where is not None else []):
            if self._refs_only(c, inner):
                keep.append(c)
            elif isinstance(c, BinOp) and c.op == "=" and self._refs_only(c.left, inner) and self._refs_only(c.right, fr):
                ikeys.append(c.left); okeys.append(c.right)
            elif isinstance(c, BinOp) and c.op == "=" and self._refs_only(c.right, inner) and self._refs_only(c.left, fr):
                ikeys.append(c.right); okeys.append(c.left)
            else:
                raise SQLError("EXISTS subquery: outer references only in equality conjuncts are supported")
        if not ikeys:
            return _ser(self.run_query(e.query, ctes).n > 0, fr.n)
        where = None
        for c in keep:
            where = c if where is None else BinOp("and", where, c)
        sel = replace(body, items=[SelectItem(k) for k in ikeys], where=where, order_by=[], limit=None,
                      distinct=False)
        sub = self.run_select(sel, qctes)
        pool = set(zip(*[[_hashable(x) for x in sub.series(i).tolist()] for i in range(len(ikeys))]))
        outer = [_ser(self.eval(k, fr, ctes, vals), fr.n).tolist() for k in okeys]
        return pd.Series([not any(B.is_null(x) for x in t) and tuple(_hashable(x) for x in t) in pool
                          for t in zip(*outer)], dtype=object)

    def _join(self, j: Join, ctes) -> Frame:
        if id(j) in self._prebuilt:
            L, R = self._prebuilt.pop(id(j))
        else:
            L = self._source(j.left, ctes)
            R = self._source(j.right, ctes)
        if j.kind == "cross" or j.on is None:
            li = np.repeat(np.arange(L.n), R.n)
            ri = np.tile(np.arange(R.n), L.n)
            fr = Frame.concat_cols(L.take(li), R.take(ri))
            if j.on is not None:
                fr = fr.take(np.nonzero(_truthy(_ser(self.eval(j.on, fr, ctes), fr.n)))[0])
            return fr
        lkeys, rkeys, resid = [], [], []
        for c in self._split_conj(j.on):
            if isinstance(c, BinOp) and c.op == "=":
                if self._refs_only(c.left, L) and self._refs_only(c.right, R) and not self._refs_only(c.left, R):
                    lkeys.append(c.left)
                    rkeys.append(c.right)
                    continue
                if self._refs_only(c.left, R) and self._refs_only(c.right, L) and not self._refs_only(c.left, L):
                    lkeys.append(c.right)
                    rkeys.append(c.left)
                    continue
            resid.append(c)
        if not lkeys:
            li = np.repeat(np.arange(L.n), R.n)
            ri = np.tile(np.arange(R.n), L.n)
            fr = Frame.concat_cols(L.take(li), R.take(ri))
            keep = _truthy(_ser(self.eval(j.on, fr, ctes), fr.n))
            if j.kind == "inner":
                return fr.take(np.nonzero(keep)[0])
            return self._outer_fill(L, R, li[keep], ri[keep], j.kind)
        lk = pd.DataFrame({f"k{i}": [_hashable(v) for v in _ser(self.eval(e, L, ctes), L.n).tolist()]
                           for i, e in enumerate(lkeys)})
        rk = pd.DataFrame({f"k{i}": [_hashable(v) for v in _ser(self.eval(e, R, ctes), R.n).tolist()]
                           for i, e in enumerate(rkeys)})
        lk["__li"] = np.arange(L.n)
        rk["__ri"] = np.arange(R.n)
        keys = [f"k{i}" for i in range(len(lkeys))]
        for k in keys:  # Hive compares mismatched key types as doubles (else as strings)
            lt = {type(v) for v in lk[k].tolist()[:4096] if v is not None}
            rt = {type(v) for v in rk[k].tolist()[:4096] if v is not None}
            mixed = len(lt | rt) > 1 and (str in (lt | rt))
            if mixed or (lk[k].dtype != rk[k].dtype and (lk[k].dtype == object or rk[k].dtype == object)):
                ln = pd.to_numeric(lk[k], errors="coerce")
                rn = pd.to_numeric(rk[k], errors="coerce")
                if ln.notna().sum() == lk[k].notna().sum() and rn.notna().sum() == rk[k].notna().sum():
                    lk[k], rk[k] = ln.astype(np.float64), rn.astype(np.float64)
                else:
                    lk[k] = lk[k].map(lambda v: None if v is None else str(v))
                    rk[k] = rk[k].map(lambda v: None if v is None else str(v))
        # NULL keys never match
        lk_nn = lk.dropna(subset=keys)
        rk_nn = rk.dropna(subset=keys)
        try:
            m = lk_nn.merge(rk_nn, on=keys, how="inner")
        except TypeError:
            for k in keys:
                lk_nn[k] = lk_nn[k].map(repr)
                rk_nn[k] = rk_nn[k].map(repr)
            m = lk_nn.merge(rk_nn, on=keys, how="inner")
        li = m["__li"].to_numpy()
        ri = m["__ri"].to_numpy()
        if resid:
            fr = Frame.concat_cols(L.take(li), R.take(ri))
            cond = resid[0]
            for c in resid[1:]:
                cond = BinOp("and", cond, c)
            keep = _truthy(_ser(self.eval(cond, fr, ctes), fr.n))
            li, ri = li[keep], ri[keep]
        if j.kind == "semi":
            return L.take(np.unique(li))
        if j.kind == "inner":
            return Frame.concat_cols(L.take(li), R.take(ri))
        return self._outer_fill(L, R, li, ri, j.kind)

    def _outer_fill(self, L: Frame, R: Frame, li, ri, kind) -> Frame:
        parts_l, parts_r = [li], [ri]
        if kind in ("left", "full"):
            miss = np.setdiff1d(np.arange(L.n), li)
            parts_l.append(miss)
            parts_r.append(np.full(len(miss), -1))
        if kind in ("right", "full"):
            miss = np.setdiff1d(np.arange(R.n), ri)
            parts_l.append(np.full(len(miss), -1))
            parts_r.append(miss)
        li = np.concatenate(parts_l).astype(np.int64)
        ri = np.concatenate(parts_r).astype(np.int64)
        return Frame.concat_cols(self._take_null(L, li), self._take_null(R, ri))

    @staticmethod
    def _take_null(F: Frame, idx) -> Frame:
        idx = np.asarray(idx)
        valid = idx >= 0
        d = {}
        for c in F.df.columns:
            s = F.df[c]
            vals = s.to_numpy(dtype=object)
            out = np.empty(len(idx), dtype=object)
            out[valid] = vals[idx[valid]]
            out[~valid] = None
            try:
                d[c] = pd.Series(out).infer_objects()
            except Exception:  # pragma: no cover
                d[c] = pd.Series(out)
        return Frame(pd.DataFrame(d, columns=list(F.df.columns)), list(F.cols))

    # -- lateral view
    def _table_fn(self, name: str):
        fd = self._lookup(name)
        if fd is not None and fd.kind == registry.UDTF:
            return fd.impl, fd.per_row, fd.cols
        if name in B.TABLE:
            return B.TABLE[name], True, B.TABLE_COLS.get(name)
        raise SQLError(f"'{name}' is not a table function")

    def _lateral(self, lv: LateralView, ctes) -> Frame:
        src = self._source(lv.source, ctes)
        impl, per_row, default_cols = self._table_fn(lv.func.name)
        args = [_ser(self.eval(a, src, ctes), src.n).tolist() for a in lv.func.args]
        if impl is B.explode and len(args) == 1:
            fast = self._explode_lists(src, lv, args[0])
            if fast is not None:
                return fast
        batch = getattr(impl, "batch", None)
        if per_row and batch is not None and not lv.outer and os.environ.get("HM_SQL_BATCH_UDTF", "1") != "0":
            # column-at-once form of a per-row UDTF (e.g. feature_pairs '-ffm'): same rows, same
            # order, no Python generator per input row
            res = batch(*args)
            if res is not None:
                rows_idx, cols = res
                names = lv.col_aliases or list(default_cols or [f"col{i}" for i in range(len(cols))])
                if len(names) == len(cols):
                    new = Frame(pd.DataFrame({f"c{i}": c for i, c in enumerate(cols)}),
                                [(lv.table_alias, n) for n in names])
                    return Frame.concat_cols(src.take(np.asarray(rows_idx, dtype=np.int64)), new)
        rows_idx, out_rows = [], []
        if per_row:
            for r in range(src.n):
                produced = False
                for t in impl(*[a[r] for a in args]):
                    rows_idx.append(r)
                    out_rows.append(tuple(t))
                    produced = True
                if not produced and lv.outer:
                    rows_idx.append(r)
                    out_rows.append(None)
        else:
            raise SQLError(f"{lv.func.name} cannot be used in LATERAL VIEW")
        width = max((len(t) for t in out_rows if t is not None), default=len(lv.col_aliases) or 1)
        names = lv.col_aliases or list(default_cols or [f"col{i}" for i in range(width)])
        if len(names) < width:
            names = names + [f"col{i}" for i in range(len(names), width)]
        data = {f"c{i}": [None if t is None else (t[i] if i < len(t) else None) for t in out_rows]
                for i in range(len(names))}
        new = Frame(pd.DataFrame(data, columns=[f"c{i}" for i in range(len(names))]),
                    [(lv.table_alias, n) for n in names])
        return Frame.concat_cols(src.take(np.asarray(rows_idx, dtype=np.int64)), new)

    def _explode_lists(self, src: Frame, lv: LateralView, vals: list) -> Frame | None:
        """explode() of an array column without a Python generator per row: one flat list in C
        (itertools.chain) and a repeat of the source row index.  Maps / non-list cells -> None
        (the generic path handles them)."""
        import itertools

        lens = np.empty(len(vals), dtype=np.int64)
        for i, v in enumerate(vals):
            if isinstance(v, (list, tuple, np.ndarray)):
                lens[i] = len(v)
            elif v is None or (isinstance(v, float) and math.isnan(v)):
                lens[i] = 0
            else:
                return None
        if lv.outer:
            return None
        rows_idx = np.repeat(np.arange(len(vals), dtype=np.int64), lens)
        flat = list(itertools.chain.from_iterable(v for v in vals if isinstance(v, (list, tuple, np.ndarray))))
        names = lv.col_aliases or ["col"]
        if len(names) != 1:
            return None
        col = pd.Series(flat, dtype=object).infer_objects() if flat else pd.Series([], dtype=object)
        new = Frame(pd.DataFrame({"c0": col}), [(lv.table_alias, names[0])])
        return Frame.concat_cols(src.take(rows_idx), new)

    # -- select
    def run_select(self, s: Select, ctes) -> Frame:
        if s.grouping_sets is not None:
            return self._grouping_sets(s, ctes)
        if isinstance(s.source, Join) and s.group_by:
            from .fused import try_fused

            fused = try_fused(self, s, ctes)
            if fused is not None:
                return fused
        src = self._source(s.source, ctes)
        if any(_has_star_arg(it.expr) for it in s.items):
            s = replace(s, items=[replace(it, expr=_expand_star_args(it.expr, src)) for it in s.items])
        if s.where is not None:
            src = src.take(np.nonzero(_truthy(_ser(self.eval(s.where, src, ctes), src.n)))[0])
        # UDTF in the select list
        if len(s.items) == 1 and isinstance(s.items[0].expr, Func) and s.items[0].expr.window is None:
            fname = s.items[0].expr.name
            fd = self._lookup(fname)
            if (fd is not None and fd.kind == registry.UDTF) or fname in B.TABLE:
                out = self._select_udtf(s.items[0], src, ctes)
                return self._finish(out, out, s, ctes)
        has_agg = bool(s.group_by) or any(_contains_agg(it.expr, self) for it in s.items) or \
            (s.having is not None and _contains_agg(s.having, self))
        if has_agg:
            out, base = self._aggregate(s, src, ctes)
        else:
            out = self._project(s.items, src, ctes, {})
            base = src
        return self._finish(out, base, s, ctes)

    def _grouping_sets(self, s: Select, ctes) -> Frame:
        """GROUPING SETS / ROLLUP / CUBE: one aggregation per key subset, the keys left out of a
        set read as NULL in its rows, the results appended in set order (Hive's UNION ALL
        semantics); ORDER BY / LIMIT apply to the whole."""
        frames = []
        for keep in s.grouping_sets:
            dropped = [k for i, k in enumerate(s.group_by) if i not in keep]
            sub = replace(s, grouping_sets=None, group_by=[s.group_by[i] for i in keep], order_by=[],
                          limit=None, distinct=False,
                          items=[replace(it, expr=_null_out(it.expr, dropped)) for it in s.items],
                          having=None if s.having is None else _null_out(s.having, dropped))
            if not sub.group_by and not any(_contains_agg(it.expr, self) for it in sub.items):
                sub = replace(sub, items=sub.items + [SelectItem(Func("count", [], False, True), "__gs__")])
                fr = self.run_select(sub, ctes)
                fr = Frame(fr.df.iloc[:, :-1], fr.cols[:-1])
            else:
                fr = self.run_select(sub, ctes)
            frames.append(fr)
        names = [n for _, n in frames[0].cols]
        df = pd.concat([f.to_df().set_axis(names, axis=1) for f in frames], ignore_index=True)
        out = Frame.from_df(df)
        return self._finish(out, out, replace(s, grouping_sets=None), ctes)

    def _finish(self, out: Frame, base: Frame, s: Select, ctes) -> Frame:
        if s.distinct:
            keep = self._distinct_index(out)
            out = out.take(keep)
            base = base.take(keep) if base.n == len(keep) or True else base
        if s.order_by:
            out = self._order(out, base if base.n == out.n else out, s.order_by, ctes)
        if s.limit is not None:
            out = out.take(np.arange(min(s.offset, out.n), min(s.offset + s.limit, out.n)))
        return out

    def _distinct_index(self, fr: Frame):
        seen = set()
        keep = []
        cols = [fr.series(i).tolist() for i in range(len(fr.cols))]
        for r in range(fr.n):
            key = tuple(_hashable(c[r]) for c in cols)
            if key not in seen:
                seen.add(key)
                keep.append(r)
        return np.asarray(keep, dtype=np.int64)

    def _order(self, out: Frame, base: Frame, order, ctes) -> Frame:
        keys = []
        for e, asc in order:
            v = None
            if isinstance(e, Lit) and isinstance(e.value, int):
                v = out.series(e.value - 1)
            else:
                try:
                    v = _ser(self.eval(e, out, ctes), out.n)
                except SQLError:
                    v = _ser(self.eval(e, base, ctes), base.n)
            keys.append((v.tolist(), asc))
        idx = list(range(out.n))

        def sort_key_fn(vals):
            def k(i):
                v = vals[i]
                return (1, 0) if B.is_null(v) else (0, v)
            return k
        for vals, asc in reversed(keys):
            idx.sort(key=lambda i: (B.is_null(vals[i]), vals[i] if not B.is_null(vals[i]) else 0),
                     reverse=not asc)
            if not asc:  # NULLs last for DESC too
                nn = [i for i in idx if not B.is_null(vals[i])]
                nl = [i for i in idx if B.is_null(vals[i])]
                idx = nn + nl
        return out.take(np.asarray(idx, dtype=np.int64))

    def _project(self, items, src: Frame, ctes, agg_values) -> Frame:
        cols, names = [], []
        win = []
        for it in items:
            _collect_windows(it.expr, win)
        wvals = {id(w): self._window(w, src, ctes) for w in win}
        vals = dict(agg_values)
        vals.update(wvals)
        for i, it in enumerate(items):
            if isinstance(it.expr, Star):
                for j, (q, n) in enumerate(src.cols):
                    if n == "__dummy__":
                        continue
                    if it.expr.table is None or (q is not None and q.lower() == it.expr.table.lower()):
                        cols.append(src.series(j))
                        names.append(n)
                continue
            v = self.eval(it.expr, src, ctes, vals)
            if it.aliases:
                # struct/array-returning expression with AS (a, b)
                s = _ser(v, src.n).tolist()
                for k, a in enumerate(it.aliases):
                    cols.append(pd.Series([x[k] if isinstance(x, (list, tuple)) else
                                           (list(x.values())[k] if isinstance(x, dict) else None)
                                           for x in s], dtype=object))
                    names.append(a)
                continue
            cols.append(_ser(v, src.n))
            names.append(it.alias or _expr_name(it.expr, i))
        df = pd.DataFrame({f"c{i}": c.reset_index(drop=True) for i, c in enumerate(cols)})
        if not cols:
            df = pd.DataFrame(index=range(src.n))
        return Frame(df, [(None, n) for n in names])

    def _select_udtf(self, item: SelectItem, src: Frame, ctes) -> Frame:
        f = item.expr
        impl, per_row, default_cols = self._table_fn(f.name)
        if not per_row and getattr(impl, "accepts_series", False):
            # learner UDTFs take whole columns; an Arrow-backed column reaches the device
            # ingest as its buffers instead of millions of Python lists
            dev_feats = None
            if getattr(impl, "device_features", False) and f.args:
                # [add_bias(]feature_hashing(col)[)] hashed on the GPU into device CSR
                from .device_ftvec import try_device_features

                dev_feats = try_device_features(self, f.args[0], src, ctes)
            # a constant string (the options) is read once: no n-row object column for it
            args = [dev_feats if (k == 0 and dev_feats is not None) else
                    pd.Series([a.value], dtype=object) if (isinstance(a, Lit) and isinstance(a.value, str)) else
                    _ser(self.eval(a, src, ctes), src.n).reset_index(drop=True) for k, a in enumerate(f.args)]
        else:
            args = [_ser(self.eval(a, src, ctes), src.n).tolist() for a in f.args]
        if per_row:
            rows = []
            for r in range(src.n):
                rows.extend(tuple(t) for t in impl(*[a[r] for a in args]))
            width = max((len(t) for t in rows), default=len(item.aliases or default_cols or [1]))
            names = item.aliases or ([item.alias] if item.alias else None) or \
                list(default_cols or [f"col{i}" for i in range(width)])
            data = {f"c{i}": [t[i] if i < len(t) else None for t in rows] for i in range(len(names))}
            return Frame(pd.DataFrame(data, columns=[f"c{i}" for i in range(len(names))]),
                         [(None, n) for n in names])
        kwargs = {}
        if getattr(impl, "wants_session", False):
            kwargs["session"] = self
        df = impl(*args, **kwargs)
        if not isinstance(df, pd.DataFrame):
            df = pd.DataFrame(list(df))
        names = item.aliases or ([item.alias] if item.alias else None) or list(df.columns)
        if len(names) != len(df.columns):
            if len(names) < len(df.columns):
                df = df.iloc[:, : len(names)]
            else:
                raise SQLError(f"{f.name} returns {len(df.columns)} columns, {len(names)} aliases given")
        df = df.copy()
        df.columns = names
        return Frame.from_df(df)

    # -- aggregation
    def _aggregate(self, s: Select, src: Frame, ctes):
        aggs = []
        for it in s.items:
            _collect_aggs(it.expr, self, aggs)
        if s.having is not None:
            _collect_aggs(s.having, self, aggs)
        for e, _ in s.order_by:
            _collect_aggs(e, self, aggs)
        if s.group_by:
            key_cols = []
            for g in s.group_by:
                if isinstance(g, Lit) and isinstance(g.value, int):
                    g = s.items[g.value - 1].expr
                key_cols.append([_hashable(v) for v in _ser(self.eval(g, src, ctes), src.n).tolist()])
            kdf = pd.DataFrame({f"k{i}": k for i, k in enumerate(key_cols)})
            try:
                codes = kdf.groupby(list(kdf.columns), sort=False, dropna=False).ngroup().to_numpy()
            except TypeError:
                codes = pd.factorize(pd.Series(list(zip(*key_cols))))[0]
            n_groups = int(codes.max()) + 1 if len(codes) else 0
        else:
            codes = np.zeros(src.n, dtype=np.int64)
            n_groups = 1
        order = np.argsort(codes, kind="stable")
        bounds = np.searchsorted(codes[order], np.arange(n_groups + 1))
        first_idx = order[bounds[:-1]] if src.n else np.zeros(0, dtype=np.int64)
        # group frame: first row of every group (bare columns resolve to it)
        if src.n == 0 and not s.group_by:
            gframe = Frame(pd.DataFrame({c: [None] for c in src.df.columns}), list(src.cols))
        else:
            gframe = src.take(first_idx)
        agg_values = {}
        for a in aggs:
            agg_values[id(a)] = self._agg_values(a, src, ctes, order, bounds, n_groups, codes)
        out = self._project(s.items, gframe, ctes, agg_values)
        if s.having is not None:
            keep = _truthy(_ser(self.eval(s.having, gframe, ctes, agg_values), gframe.n))
            idx = np.nonzero(keep)[0]
            out, gframe = out.take(idx), gframe.take(idx)
            for k in list(agg_values):
                agg_values[k] = _ser(agg_values[k], len(keep))[keep].reset_index(drop=True)
        self._last_agg_values = agg_values
        return out, _GroupBase(gframe, agg_values, self)

    def _agg_values(self, a: Func, src, ctes, order, bounds, n_groups, codes) -> pd.Series:
        name = a.name.lower()
        if name == "count" and (a.star or not a.args):
            return pd.Series(np.diff(bounds))
        arg_vals = [_ser(self.eval(x, src, ctes), src.n) for x in a.args]
        fd = self._lookup(name)
        if fd is None and name in B.PANDAS_AGG and len(arg_vals) == 1 and not a.distinct:
            s = arg_vals[0]
            numeric = pd.api.types.is_numeric_dtype(s) or name == "count"
            if numeric:
                if name == "count":
                    ok = ~pd.isna(s)
                    return pd.Series(np.bincount(codes[ok.to_numpy()], minlength=n_groups))
                g = s.groupby(codes).agg(B.PANDAS_AGG[name])
                res = g.reindex(range(n_groups))
                return res.reset_index(drop=True)
        impl = fd.impl if fd is not None else B.AGGREGATE.get(name)
        if impl is None:
            raise SQLError(f"unknown aggregate function {name}")
        lists = [v.tolist() for v in arg_vals]
        out = []
        for g in range(n_groups):
            idx = order[bounds[g]:bounds[g + 1]]
            cols = [[l[i] for i in idx] for l in lists]
            if a.distinct:
                seen = set()
                keep = []
                for r in range(len(idx)):
                    key = tuple(_hashable(c[r]) for c in cols)
                    if key not in seen:
                        seen.add(key)
                        keep.append(r)
                cols = [[c[r] for r in keep] for c in cols]
            out.append(impl(*cols))
        return pd.Series(out, dtype=object)

    # -- windows
    def _window(self, f: Func, src: Frame, ctes) -> pd.Series:
        w = f.window
        n = src.n
        if w.partition:
            parts = [[_hashable(v) for v in _ser(self.eval(p, src, ctes), n).tolist()] for p in w.partition]
            codes = pd.factorize(pd.Series(list(zip(*parts))))[0] if n else np.zeros(0, dtype=np.int64)
        else:
            codes = np.zeros(n, dtype=np.int64)
        okeys = [(_ser(self.eval(e, src, ctes), n).tolist(), asc) for e, asc in w.order]
        idx = list(range(n))
        for vals, asc in reversed(okeys):
            idx.sort(key=lambda i: (B.is_null(vals[i]), vals[i] if not B.is_null(vals[i]) else 0),
                     reverse=not asc)
        idx.sort(key=lambda i: codes[i])  # stable: keeps the order within partitions
        out = [None] * n
        name = f.name.lower()
        args = [_ser(self.eval(a, src, ctes), n).tolist() for a in f.args]
        for _, grp in itertools.groupby(idx, key=lambda i: codes[i]):
            grp = list(grp)
            okey = [tuple(_hashable(v[0][i]) for v in okeys) for i in grp]
            if name == "row_number":
                for r, i in enumerate(grp):
                    out[i] = r + 1
            elif name in ("rank", "dense_rank"):
                rank = dense = 0
                prev = object()
                for r, (i, k) in enumerate(zip(grp, okey)):
                    if k != prev:
                        rank = r + 1
                        dense += 1
                        prev = k
                    out[i] = rank if name == "rank" else dense
            elif name in ("lag", "lead"):
                off = int(args[1][0]) if len(args) > 1 else 1
                dflt = args[2][0] if len(args) > 2 else None
                for r, i in enumerate(grp):
                    j = r - off if name == "lag" else r + off
                    out[i] = args[0][grp[j]] if 0 <= j < len(grp) else dflt
            elif name == "ntile":
                k = int(args[0][0])
                for r, i in enumerate(grp):
                    out[i] = r * k // len(grp) + 1
            elif name in ("percent_rank", "cume_dist"):
                m = len(grp)
                lo_, hi_ = _peer_bounds(okey)
                for r, i in enumerate(grp):
                    out[i] = (lo_[r] / (m - 1) if m > 1 else 0.0) if name == "percent_rank" else (hi_[r] + 1) / m
            else:
                impl = self._lookup(name)
                impl = impl.impl if impl is not None else B.AGGREGATE.get(name)
                if impl is None:
                    raise SQLError(f"unknown window function {name}")
                m = len(grp)
                frame = w.frame or (("range", None, 0) if w.order else ("rows", None, None))
                if frame[1] is None and frame[2] is None:      # the whole partition: one value
                    sub = [[a[j] for j in grp] for a in args]
                    v = impl(*sub) if sub else m
                    for i in grp:
                        out[i] = v
                    continue
                pos = None
                if frame[0] == "range" and any(b not in (None, 0) for b in frame[1:]):
                    if len(okeys) != 1:
                        raise SQLError("RANGE with an offset needs exactly one ORDER BY key")
                    sign = 1.0 if okeys[0][1] else -1.0
                    pos = [sign * float(okeys[0][0][i]) for i in grp]
                peers = _peer_bounds(okey)
                if frame[1] is None and frame[2] == 0 and pos is None and \
                        name in ("sum", "count", "avg", "min", "max") and len(args) <= 1 and not f.distinct:
                    # running aggregate (the default frame): one pass instead of a slice per row
                    run = _running_agg(name, [args[0][j] for j in grp] if args else None, m)
                    for r, i in enumerate(grp):
                        out[i] = run[r if frame[0] == "rows" else peers[1][r]]
                    continue
                for r, i in enumerate(grp):
                    a_, b_ = _frame_rows(frame, r, m, peers, pos)
                    sub = [[a[grp[q]] for q in range(a_, b_ + 1)] for a in args]
                    out[i] = impl(*sub) if sub else max(0, b_ - a_ + 1)
        return pd.Series(out, dtype=object)

    # -- expressions
    def eval_const(self, e: Expr):
        fr = Frame(pd.DataFrame({"c0": [0]}), [(None, "__dummy__")])
        return _ser(self.eval(e, fr, {}), 1).iloc[0]

    def eval(self, e: Expr, fr: "Frame", ctes, vals: dict | None = None):
        if vals and id(e) in vals:
            return vals[id(e)]
        if isinstance(e, Lit):
            return e.value
        if isinstance(e, Col):
            i = fr.resolve(e.name, e.table)
            if i is None:
                if isinstance(fr, _GroupBase):
                    return fr.lookup(e, ctes)
                if e.table is not None:
                    # struct field access t.field where t is a column
                    j = fr.resolve(e.table, None)
                    if j is not None:
                        return B.rowwise(lambda v: v.get(e.name) if isinstance(v, dict) else None)(fr.series(j))
                if e.name.lower() in ("true", "false"):
                    return e.name.lower() == "true"
                raise SQLError(f"Invalid column reference '{(e.table + '.') if e.table else ''}{e.name}'")
            return fr.series(i)
        if isinstance(e, BinOp):
            return self._binop(e, fr, ctes, vals)
        if isinstance(e, UnOp):
            v = _ser(self.eval(e.operand, fr, ctes, vals), fr.n)
            if e.op == "not":
                return pd.Series([None if B.is_null(x) else (not bool(x)) for x in v.tolist()], dtype=object)
            if e.op == "-":
                return -pd.to_numeric(v, errors="coerce")
            if e.op == "~":
                return B.rowwise(lambda x: ~int(x))(v)
        if isinstance(e, Func):
            return self._call(e, fr, ctes, vals)
        if isinstance(e, Case):
            n = fr.n
            out = [None] * n
            done = np.zeros(n, dtype=bool)
            base = _ser(self.eval(e.base, fr, ctes, vals), n).tolist() if e.base is not None else None
            for c, v in e.whens:
                cv = _ser(self.eval(c, fr, ctes, vals), n).tolist()
                vv = _ser(self.eval(v, fr, ctes, vals), n).tolist()
                for r in range(n):
                    if done[r]:
                        continue
                    hit = (base[r] == cv[r]) if base is not None else (not B.is_null(cv[r]) and bool(cv[r]))
                    if hit:
                        out[r] = vv[r]
                        done[r] = True
            if e.default is not None:
                dv = _ser(self.eval(e.default, fr, ctes, vals), n).tolist()
                for r in range(n):
                    if not done[r]:
                        out[r] = dv[r]
            return pd.Series(out, dtype=object).infer_objects()
        if isinstance(e, Cast):
            v = _ser(self.eval(e.expr, fr, ctes, vals), fr.n)
            return pd.Series([_cast_value(x, e.type) for x in v.tolist()], dtype=object).infer_objects()
        if isinstance(e, Exists):
            return self._exists(e, fr, ctes, vals)
        if isinstance(e, InList):
            v = _ser(self.eval(e.expr, fr, ctes, vals), fr.n).tolist()
            if len(e.items) == 1 and isinstance(e.items[0], SubqueryExpr):
                sub = self.run_query(e.items[0].query, ctes)
                pool = set(_hashable(x) for x in sub.series(0).tolist())
                res = [None if B.is_null(x) else (_hashable(x) in pool) != e.negate for x in v]
                return pd.Series(res, dtype=object)
            items = [_ser(self.eval(it, fr, ctes, vals), fr.n).tolist() for it in e.items]
            res = []
            for r, x in enumerate(v):
                if B.is_null(x):
                    res.append(None)
                else:
                    res.append(any(x == it[r] for it in items) != e.negate)
            return pd.Series(res, dtype=object)
        if isinstance(e, Between):
            v = _ser(self.eval(e.expr, fr, ctes, vals), fr.n).tolist()
            lo = _ser(self.eval(e.lo, fr, ctes, vals), fr.n).tolist()
            hi = _ser(self.eval(e.hi, fr, ctes, vals), fr.n).tolist()
            return pd.Series([None if B.is_null(x) else ((lo[r] <= x <= hi[r]) != e.negate)
                              for r, x in enumerate(v)], dtype=object)
        if isinstance(e, IsNull):
            v = _ser(self.eval(e.expr, fr, ctes, vals), fr.n).tolist()
            return pd.Series([B.is_null(x) != e.negate for x in v])
        if isinstance(e, Like):
            v = _ser(self.eval(e.expr, fr, ctes, vals), fr.n).tolist()
            p = _ser(self.eval(e.pattern, fr, ctes, vals), fr.n).tolist()
            out = []
            for x, pat in zip(v, p):
                if B.is_null(x) or B.is_null(pat):
                    out.append(None)
                    continue
                rx = pat if e.regex else _like_to_regex(pat)
                hit = re.search(rx, str(x)) is not None if e.regex else re.match(rx, str(x), re.S) is not None
                out.append(hit != e.negate)
            return pd.Series(out, dtype=object)
        if isinstance(e, Index):
            b = _ser(self.eval(e.base, fr, ctes, vals), fr.n).tolist()
            ix = _ser(self.eval(e.index, fr, ctes, vals), fr.n).tolist()
            out = []
            for x, i in zip(b, ix):
                if B.is_null(x) or B.is_null(i):
                    out.append(None)
                elif isinstance(x, dict):
                    out.append(x.get(i))
                else:
                    i = int(i)
                    out.append(x[i] if 0 <= i < len(x) else None)
            return pd.Series(out, dtype=object).infer_objects()
        if isinstance(e, Field):
            b = _ser(self.eval(e.base, fr, ctes, vals), fr.n).tolist()
            return pd.Series([x.get(e.name) if isinstance(x, dict) else None for x in b], dtype=object)
        if isinstance(e, SubqueryExpr):
            sub = self.run_query(e.query, ctes)
            return sub.series(0).iloc[0] if sub.n else None
        if isinstance(e, Star):
            raise SQLError("* is only valid in the select list or count(*)")
        raise SQLError(f"unsupported expression {type(e).__name__}")

    def _binop(self, e: BinOp, fr, ctes, vals):
        n = fr.n
        a = self.eval(e.left, fr, ctes, vals)
        b = self.eval(e.right, fr, ctes, vals)
        op = e.op
        if op in ("and", "or"):
            A = _ser(a, n).tolist()
            Bv = _ser(b, n).tolist()
            out = []
            for x, y in zip(A, Bv):
                xn, yn = B.is_null(x), B.is_null(y)
                if op == "and":
                    if (not xn and not x) or (not yn and not y):
                        out.append(False)
                    elif xn or yn:
                        out.append(None)
                    else:
                        out.append(True)
                else:
                    if (not xn and x) or (not yn and y):
                        out.append(True)
                    elif xn or yn:
                        out.append(None)
                    else:
                        out.append(False)
            return pd.Series(out, dtype=object)
        A = _ser(a, n)
        Bs = _ser(b, n)
        if op in ("+", "-", "*", "/", "%", "div"):
            if op == "+" and (A.dtype == object and any(isinstance(x, str) for x in A.tolist()[:8])):
                return B.rowwise(lambda x, y: x + y)(A, Bs)
            x = pd.to_numeric(A, errors="coerce").to_numpy(dtype=np.float64)
            y = pd.to_numeric(Bs, errors="coerce").to_numpy(dtype=np.float64)
            with np.errstate(divide="ignore", invalid="ignore"):
                if op == "+":
                    r = x + y
                elif op == "-":
                    r = x - y
                elif op == "*":
                    r = x * y
                elif op == "/":
                    r = np.where(y == 0, np.nan, x / np.where(y == 0, 1, y))
                elif op == "%":
                    r = np.where(y == 0, np.nan, np.fmod(x, np.where(y == 0, 1, y)))
                else:
                    r = np.where(y == 0, np.nan, np.trunc(x / np.where(y == 0, 1, y)))   # Java: toward 0
            ints = (pd.api.types.is_integer_dtype(A) and pd.api.types.is_integer_dtype(Bs)
                    and op in ("+", "-", "*", "%", "div"))
            res = pd.Series(r)
            if ints and not np.isnan(r).any():
                res = res.astype(np.int64)
            return res
        if op in ("&", "|", "^"):
            f = {"&": lambda x, y: int(x) & int(y), "|": lambda x, y: int(x) | int(y),
                 "^": lambda x, y: int(x) ^ int(y)}[op]
            return B.rowwise(f)(A, Bs)
        cmp = {"=": lambda x, y: x == y, "!=": lambda x, y: x != y, "<": lambda x, y: x < y,
               "<=": lambda x, y: x <= y, ">": lambda x, y: x > y, ">=": lambda x, y: x >= y}
        if op == "<=>":
            return pd.Series([(B.is_null(x) and B.is_null(y)) or (not B.is_null(x) and x == y)
                              for x, y in zip(A.tolist(), Bs.tolist())])
        f = cmp[op]
        out = []
        for x, y in zip(A.tolist(), Bs.tolist()):
            if B.is_null(x) or B.is_null(y):
                out.append(None)
                continue
            try:
                out.append(bool(f(x, y)))
            except TypeError:
                try:
                    out.append(bool(f(float(x), float(y))))
                except (TypeError, ValueError):
                    out.append(bool(f(str(x), str(y))))
        return pd.Series(out, dtype=object)

    def _call(self, f: Func, fr: Frame, ctes, vals):
        name = f.name.lower()
        n = fr.n
        if f.window is not None:
            return self._window(f, fr, ctes)
        if name in self.macros:
            params, body = self.macros[name]
            sub = {p.lower(): a for p, a in zip(params, f.args)}
            return self.eval(_subst_macro(body, sub), fr, ctes, vals)
        fd = self._lookup(name)
        if fd is not None and fd.kind == registry.UDAF or (fd is None and name in B.AGGREGATE):
            if isinstance(fr, _GroupBase):
                return fr.agg(f, ctes)
            # aggregate over the whole frame (e.g. in a scalar context)
            impl = fd.impl if fd is not None else B.AGGREGATE[name]
            if name == "count" and (f.star or not f.args):
                return n
            cols = [_ser(self.eval(a, fr, ctes, vals), n).tolist() for a in f.args]
            return impl(*cols)
        if name == "rand":
            return B._rand(None if not f.args else _ser(self.eval(f.args[0], fr, ctes, vals), n), n)
        args = [self.eval(a, fr, ctes, vals) for a in f.args]
        if fd is not None and fd.kind == registry.UDF:
            if fd.vectorized:
                res = fd.impl(*[_ser(a, n) if isinstance(a, pd.Series) else a for a in args])
                return _ser(res if not isinstance(res, list) else pd.Series(res, dtype=object), n)
            cols = [_ser(a, n).tolist() if isinstance(a, pd.Series) else None for a in args]
            out = []
            # Hivemall's UDFs return NULL for a NULL principal (first) argument: such rows yield
            # NULL without calling the function (assert / raise_error / sessionize see NULLs)
            null_rule = bool(args) and name not in _NULL_AWARE_UDFS
            for r in range(n):
                row = [c[r] if c is not None else a for c, a in zip(cols, args)]
                if null_rule and row[0] is None:
                    out.append(None)
                    continue
                out.append(fd.impl(*row))
            return pd.Series(out, dtype=object).infer_objects() if out else pd.Series([], dtype=object)
        if fd is not None and fd.kind == registry.UDTF:
            raise SQLError(f"UDTF {name} must be the only expression in SELECT or used in LATERAL VIEW")
        if name in B.SCALAR and B.SCALAR[name] is not None:
            if not args:                # array(), current_date(), pi(): one value for every row
                res = B.SCALAR[name]()
                return _ser(res.iloc[0] if isinstance(res, pd.Series) and len(res) == 1 else res, n)
            return _ser(B.SCALAR[name](*[_ser(a, n) for a in args]), n)
        if name == "sigmoid":
            x = pd.to_numeric(_ser(args[0], n), errors="coerce").to_numpy(dtype=np.float64)
            return pd.Series(1.0 / (1.0 + np.exp(-x)))
        raise SQLError(f"Invalid function '{f.name}'")


class _GroupBase(Frame):
    """The grouped frame: bare columns resolve to the first row of the group; aggregate
    calls resolve to the precomputed per-group values (used by ORDER BY / HAVING)."""

    def __init__(self, gframe: Frame, agg_values: dict, session: Session):
        super().__init__(gframe.df, gframe.cols)
        self._agg = agg_values
        self._s = session

    def take(self, idx):
        idx = np.asarray(idx)
        g = Frame(self.df.iloc[idx].reset_index(drop=True), list(self.cols))
        agg = {k: _ser(v, self.n).iloc[idx].reset_index(drop=True) for k, v in self._agg.items()}
        return _GroupBase(g, agg, self._s)

    def lookup(self, e, ctes):
        raise SQLError(f"Invalid column reference '{e.name}'")

    def agg(self, f: Func, ctes):
        for k, v in self._agg.items():
            pass
        # match structurally identical aggregate calls (ORDER BY sum(x) after SELECT sum(x))
        for node_id, v in self._agg.items():
            node = _AGG_NODES.get(node_id)
            if node is not None and node == f:
                return v
        raise SQLError(f"aggregate {f.name} not available in this context")


_AGG_NODES: dict = {}


def _subst_macro(e, sub: dict):
    if isinstance(e, Col) and e.table is None and e.name.lower() in sub:
        return sub[e.name.lower()]
    if isinstance(e, BinOp):
        return BinOp(e.op, _subst_macro(e.left, sub), _subst_macro(e.right, sub))
    if isinstance(e, UnOp):
        return UnOp(e.op, _subst_macro(e.operand, sub))
    if isinstance(e, Func):
        return Func(e.name, [_subst_macro(a, sub) for a in e.args], e.distinct, e.star, e.window)
    if isinstance(e, Case):
        return Case(None if e.base is None else _subst_macro(e.base, sub),
                    [(_subst_macro(c, sub), _subst_macro(v, sub)) for c, v in e.whens],
                    None if e.default is None else _subst_macro(e.default, sub))
    if isinstance(e, Cast):
        return Cast(_subst_macro(e.expr, sub), e.type)
    if isinstance(e, Index):
        return Index(_subst_macro(e.base, sub), _subst_macro(e.index, sub))
    return e


# keep structural copies of aggregate nodes so ORDER BY / HAVING can reuse their values
_orig_collect = _collect_aggs


def _collect_aggs(e, session, out: list):  # noqa: F811
    before = len(out)
    _orig_collect(e, session, out)
    for node in out[before:]:
        _AGG_NODES[id(node)] = node
