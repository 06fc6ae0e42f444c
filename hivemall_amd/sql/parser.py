"""Recursive-descent parser for the HiveQL subset (AST in plain dataclasses)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

from .lexer import Tok, tokenize

RESERVED = {
    "select", "distinct", "from", "where", "group", "by", "having", "order", "sort", "cluster",
    "distribute", "limit", "as", "on", "join", "inner", "left", "right", "full", "outer", "cross",
    "semi", "lateral", "union", "and", "or", "not", "in", "is", "null", "true", "false", "between",
    "like", "rlike", "regexp", "case", "when", "then", "else", "end", "cast", "over", "with",
    "div", "all",
}


# ------------------------------------------------------------------ expressions
@dataclass
class Expr:
    pass


@dataclass
class Lit(Expr):
    value: Any


@dataclass
class Col(Expr):
    name: str
    table: str | None = None


@dataclass
class Star(Expr):
    table: str | None = None


@dataclass
class Func(Expr):
    name: str
    args: list
    distinct: bool = False
    star: bool = False
    window: "Window | None" = None


@dataclass
class Window:
    partition: list
    order: list          # [(expr, asc)]
    # (unit "rows" | "range", start, end); offsets relative to the current row: None =
    # unbounded, 0 = current row, -n = n preceding, +n = n following.  None = Hive's default
    # (RANGE UNBOUNDED PRECEDING .. CURRENT ROW with ORDER BY, the whole partition without).
    frame: tuple | None = None


@dataclass
class BinOp(Expr):
    op: str
    left: Expr
    right: Expr


@dataclass
class UnOp(Expr):
    op: str
    operand: Expr


@dataclass
class Case(Expr):
    base: Expr | None
    whens: list          # [(cond, value)]
    default: Expr | None


@dataclass
class Cast(Expr):
    expr: Expr
    type: str


@dataclass
class InList(Expr):
    expr: Expr
    items: list
    negate: bool = False


@dataclass
class Between(Expr):
    expr: Expr
    lo: Expr
    hi: Expr
    negate: bool = False


@dataclass
class IsNull(Expr):
    expr: Expr
    negate: bool = False


@dataclass
class Like(Expr):
    expr: Expr
    pattern: Expr
    regex: bool = False
    negate: bool = False


@dataclass
class Index(Expr):
    base: Expr
    index: Expr


@dataclass
class Field(Expr):
    base: Expr
    name: str


@dataclass
class Exists(Expr):
    query: "Query"


@dataclass
class SubqueryExpr(Expr):
    query: "Query"


# ------------------------------------------------------------------ relations / statements
@dataclass
class SelectItem:
    expr: Expr
    alias: str | None = None
    aliases: list | None = None        # UDTF AS (a, b, c)


@dataclass
class TableRef:
    name: str
    alias: str | None = None
    sample: tuple | None = None     # TABLESAMPLE: ("bucket", x, y, expr|None) | ("percent", p) | ("rows", n)


@dataclass
class SubqueryRef:
    query: "Query"
    alias: str | None = None
    sample: tuple | None = None


@dataclass
class Join:
    left: Any
    right: Any
    kind: str            # inner, left, right, full, cross, semi
    on: Expr | None = None


@dataclass
class LateralView:
    source: Any
    func: Func
    table_alias: str | None
    col_aliases: list
    outer: bool = False


@dataclass
class Select:
    items: list
    source: Any = None
    where: Expr | None = None
    group_by: list = field(default_factory=list)
    grouping_sets: list | None = None      # [[index into group_by, ...], ...] (ROLLUP / CUBE / SETS)
    having: Expr | None = None
    order_by: list = field(default_factory=list)      # [(expr, asc)]
    cluster_by: list = field(default_factory=list)
    distinct: bool = False
    limit: int | None = None
    offset: int = 0                 # LIMIT offset, n


@dataclass
class Union:
    parts: list
    all: bool = True
    order_by: list = field(default_factory=list)
    limit: int | None = None
    offset: int = 0                 # LIMIT offset, n


@dataclass
class Query:
    body: Any                           # Select | Union
    ctes: list = field(default_factory=list)     # [(name, Query)]


@dataclass
class CreateTable:
    name: str
    query: Query | None
    columns: list = field(default_factory=list)
    if_not_exists: bool = False
    view: bool = False
    types: list = field(default_factory=list)     # declared Hive types, parallel to columns
    storage: dict = field(default_factory=dict)   # location / stored_as / field_delim / collection_delim
    like: str | None = None                       # CREATE TABLE t LIKE src


@dataclass
class LoadData:
    path: str
    table: str
    overwrite: bool = False


@dataclass
class InsertDirectory:
    path: str
    query: Query
    storage: dict = field(default_factory=dict)


@dataclass
class Insert:
    table: str
    query: Query
    overwrite: bool = True


@dataclass
class Drop:
    name: str
    what: str
    if_exists: bool = False


@dataclass
class CreateFunction:
    name: str
    class_name: str


@dataclass
class CreateMacro:
    name: str
    params: list
    body: Expr


@dataclass
class SetStmt:
    key: str | None
    value: str | None


@dataclass
class NoOp:
    text: str


@dataclass
class MultiInsert:
    inserts: list       # Insert / InsertDirectory statements sharing one FROM source


@dataclass
class Truncate:
    table: str


@dataclass
class RenameTable:
    old: str
    new: str


@dataclass
class ShowFunctions:
    pattern: str | None


@dataclass
class DescribeFunction:
    name: str


@dataclass
class ShowTables:
    pattern: str | None


@dataclass
class DescribeTable:
    name: str


# ------------------------------------------------------------------ parser
class Parser:
    def __init__(self, sql: str):
        self.sql = sql
        self.toks = tokenize(sql)
        self.i = 0

    # -- helpers
    @property
    def t(self) -> Tok:
        return self.toks[self.i]

    def peek(self, k: int = 1) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def error(self, msg: str):
        t = self.t
        ctx = self.sql[max(0, t.pos - 30):t.pos + 30]
        raise SyntaxError(f"{msg} at position {t.pos} near '{t.val}' (…{ctx}…)")

    def accept_kw(self, *ws) -> bool:
        if self.t.is_kw(*ws):
            self.i += 1
            return True
        return False

    def expect_kw(self, *ws):
        if not self.accept_kw(*ws):
            self.error(f"expected {'/'.join(ws).upper()}")

    def accept_op(self, *ops) -> bool:
        if self.t.is_op(*ops):
            self.i += 1
            return True
        return False

    def expect_op(self, op):
        if not self.accept_op(op):
            self.error(f"expected '{op}'")

    def ident(self) -> str:
        t = self.t
        if t.kind == "ident" or (t.kind == "kw" and t.val not in RESERVED):
            self.i += 1
            return t.val
        self.error("expected identifier")

    def is_ident(self) -> bool:
        t = self.t
        return t.kind == "ident" or (t.kind == "kw" and t.val not in RESERVED)

    def qualified_name(self) -> str:
        n = self.ident()
        while self.t.is_op(".") and (self.peek().kind == "ident" or self.peek().kind == "kw"):
            self.next()
            n = n + "." + self.ident()
        return n

    # -- statements
    def statement(self):
        t = self.t
        if t.is_kw("select", "with") or t.is_op("("):
            q = self.query()
        elif t.is_kw("create"):
            q = self.create()
        elif t.is_kw("insert"):
            q = self.insert()
        elif t.is_kw("from"):
            q = self.from_first()
        elif t.is_kw("drop"):
            q = self.drop()
        elif t.is_kw("set"):
            q = self.set_stmt()
        elif t.kind == "ident" and t.val.lower() == "load":
            q = self.load_data()
        elif t.kind == "ident" and t.val.lower() == "truncate":
            self.next()
            self.accept_kw("table")
            q = Truncate(self.qualified_name())
            if self.accept_kw("partition"):
                self.error("TRUNCATE ... PARTITION is not supported (tables are unpartitioned)")
        elif t.kind == "ident" and t.val.lower() == "alter":
            q = self.alter()
        elif t.kind == "ident" and t.val.lower() in ("analyze", "msck"):
            q = NoOp(self.sql)                     # statistics / partition repair: nothing to do
            self.i = len(self.toks) - 1
        elif t.is_kw("add", "source", "use", "reload") or (t.kind == "ident" and t.val.lower() in ("delete", "list")):
            q = NoOp(self.sql)
            self.i = len(self.toks) - 1
        elif t.is_kw("show"):
            self.next()
            tables = self.t.kind == "ident" and self.t.val.lower() == "tables"
            if tables:
                self.next()
            else:
                self.expect_kw("functions")
            pat = None
            if self.t.kind == "str":
                pat = self.next().val
            elif self.accept_kw("like"):
                pat = self.next().val
            q = ShowTables(pat) if tables else ShowFunctions(pat)
        elif t.is_kw("describe"):
            self.next()
            if self.accept_kw("function"):
                if self.t.kind == "ident" and self.t.val.lower() == "extended":
                    self.next()
                q = DescribeFunction(self.ident())
            else:
                self.accept_kw("table")
                if self.t.kind == "ident" and self.t.val.lower() in ("extended", "formatted"):
                    self.next()
                q = DescribeTable(self.qualified_name())
        elif t.is_kw("explain"):
            self.next()
            return ("explain", self.statement())
        else:
            self.error("unsupported statement")
        self.accept_op(";")
        if self.t.kind != "eof":
            self.error("unexpected trailing input")
        return q

    def set_stmt(self):
        self.expect_kw("set")
        start = self.t.pos
        if self.t.kind == "eof":
            return SetStmt(None, None)
        rest = self.sql[start:].strip().rstrip(";")
        self.i = len(self.toks) - 1
        if "=" in rest:
            k, v = rest.split("=", 1)
            return SetStmt(k.strip(), v.strip())
        return SetStmt(rest.strip(), None)

    def alter(self):
        """ALTER TABLE a RENAME TO b; other ALTER TABLE forms (properties, SerDe, partitions,
        file format) describe storage that has no counterpart here and are accepted as no-ops."""
        self.next()
        if self.t.is_kw("table", "view"):
            self.next()
            name = self.qualified_name()
            if self.t.kind == "ident" and self.t.val.lower() == "rename":
                self.next()
                if not (self.t.kind == "ident" and self.t.val.lower() == "to"):
                    self.error("expected RENAME TO")
                self.next()
                return RenameTable(name, self.qualified_name())
        q = NoOp(self.sql)
        self.i = len(self.toks) - 1
        return q

    def create(self):
        self.expect_kw("create")
        if self.t.is_kw("or") and self.peek().kind == "ident" and self.peek().val.lower() == "replace":
            self.next(); self.next()           # CREATE OR REPLACE VIEW: a CREATE replaces anyway
        if self.t.kind == "ident" and self.t.val.lower() in ("database", "schema"):
            q = NoOp(self.sql)                 # one namespace: databases are accepted and ignored
            self.i = len(self.toks) - 1
            return q
        temporary = self.accept_kw("temporary")
        self.accept_kw("external")
        if self.accept_kw("function"):
            name = self.ident()
            self.expect_kw("as")
            cls = self.next().val
            while self.t.kind != "eof" and not self.t.is_op(";"):
                self.next()   # USING JAR '...'
            return CreateFunction(name, cls)
        if self.accept_kw("macro"):
            name = self.ident()
            self.expect_op("(")
            params = []
            while not self.t.is_op(")"):
                params.append(self.ident())
                # optional type
                while not self.t.is_op(",", ")"):
                    self.next()
                self.accept_op(",")
            self.expect_op(")")
            body = self.expr()
            return CreateMacro(name, params, body)
        view = False
        if self.accept_kw("view"):
            view = True
        else:
            self.expect_kw("table")
        ine = False
        if self.accept_kw("if"):
            self.expect_kw("not")
            self.expect_kw("exists")
            ine = True
        name = self.qualified_name()
        if self.accept_kw("like"):
            src = self.qualified_name()
            self.storage_clause(stop_at_query=False)
            return CreateTable(name, None, [], ine, view, [], {}, like=src)
        cols = []
        if self.t.is_op("("):
            self.next()
            depth = 1
            cur = []
            while depth > 0:
                tk = self.next()
                if tk.is_op("("):
                    depth += 1
                elif tk.is_op(")"):
                    depth -= 1
                    if depth == 0:
                        break
                if depth == 1 and tk.is_op(","):
                    cols.append(cur)
                    cur = []
                elif tk.kind != "eof":
                    cur.append(tk.val)
                else:
                    self.error("unterminated column list")
            if cur:
                cols.append(cur)
            cols = [c for c in cols if c]
            types = ["".join(c[1:c.index("comment")] if "comment" in c else c[1:]) for c in cols]
            cols = [c[0] for c in cols]
        else:
            types = []
        query = None
        # ROW FORMAT DELIMITED ..., STORED AS <fmt>, LOCATION '...' are kept (io/tables.py reads
        # the location); TBLPROPERTIES (...), COMMENT '...', PARTITIONED BY (...) are skipped
        storage = self.storage_clause(stop_at_query=True)
        if self.accept_kw("as") or self.t.is_kw("select", "with"):
            query = self.query()
        return CreateTable(name, query, cols, ine, view, types, storage)

    def storage_clause(self, stop_at_query: bool) -> dict:
        st: dict = {}
        while self.t.kind != "eof" and not self.t.is_op(";"):
            if stop_at_query and self.t.is_kw("select", "with"):
                break
            if self.t.is_kw("as") and (self.peek().is_kw("select", "with") or self.peek().is_op("(")):
                break
            if not stop_at_query and self.t.is_kw("select", "with"):
                break
            v = self.t.val.lower() if self.t.kind in ("kw", "ident") else None
            if v == "terminated" and self.peek().is_kw("by") and self.peek(2).kind == "str":
                prev = self.toks[self.i - 1].val.lower() if self.i else ""
                self.next(); self.next()
                key = {"fields": "field_delim", "items": "collection_delim", "keys": "map_key_delim",
                       "lines": "line_delim"}.get(prev)
                d = self.next().val
                if key:
                    st[key] = d
                continue
            if v == "stored" and self.peek().is_kw("as"):
                self.next(); self.next()
                st["stored_as"] = self.next().val.lower()
                continue
            if v == "location" and self.peek().kind == "str":
                self.next()
                st["location"] = self.next().val
                continue
            self.next()
        return st

    def load_data(self):
        self.next()                                   # LOAD
        if not (self.t.kind == "ident" and self.t.val.lower() == "data"):
            self.error("expected LOAD DATA")
        self.next()
        if self.t.kind == "ident" and self.t.val.lower() == "local":
            self.next()
        if not (self.t.kind == "ident" and self.t.val.lower() == "inpath"):
            self.error("expected INPATH")
        self.next()
        if self.t.kind != "str":
            self.error("expected a path string")
        path = self.next().val
        overwrite = self.accept_kw("overwrite")
        self.expect_kw("into")
        self.expect_kw("table")
        return LoadData(path, self.qualified_name(), overwrite)

    def from_first(self):
        """Hive's FROM-first forms: ``FROM src SELECT ...`` and the multi-insert
        ``FROM src INSERT OVERWRITE TABLE a SELECT ... INSERT INTO TABLE b SELECT ...``."""
        self.expect_kw("from")
        src = self.from_clause()

        def bind(q):
            body = q.body
            if not isinstance(body, Select):
                self.error("FROM ... INSERT: each branch must be a single SELECT")
            if body.source is not None:
                self.error("FROM ... INSERT: a branch may not have its own FROM")
            body.source = src
            return q

        if self.t.is_kw("select"):
            return bind(Query(self.select(), []))
        inserts = []
        while self.t.is_kw("insert"):
            ins = self.insert()
            bind(ins.query)
            inserts.append(ins)
        if not inserts:
            self.error("expected INSERT or SELECT after FROM")
        return inserts[0] if len(inserts) == 1 else MultiInsert(inserts)

    def insert(self):
        self.expect_kw("insert")
        overwrite = True
        if self.accept_kw("overwrite"):
            pass
        else:
            self.expect_kw("into")
            overwrite = False
        if self.t.kind == "ident" and self.t.val.lower() in ("local", "directory"):
            if self.t.val.lower() == "local":
                self.next()
            if not (self.t.kind == "ident" and self.t.val.lower() == "directory"):
                self.error("expected DIRECTORY")
            self.next()
            if self.t.kind != "str":
                self.error("expected a directory path string")
            path = self.next().val
            storage = self.storage_clause(stop_at_query=False)
            return InsertDirectory(path, self.query(), storage)
        self.accept_kw("table")
        name = self.qualified_name()
        if self.accept_kw("partition"):
            self.expect_op("(")
            depth = 1
            while depth:
                tk = self.next()
                depth += tk.is_op("(") - tk.is_op(")")
        if self.t.is_kw("values"):
            self.next()
            rows = []
            while True:
                self.expect_op("(")
                vals = [self.expr()]
                while self.accept_op(","):
                    vals.append(self.expr())
                self.expect_op(")")
                rows.append(vals)
                if not self.accept_op(","):
                    break
            return Insert(name, Query(("values", rows)), overwrite)
        return Insert(name, self.query(), overwrite)

    def drop(self):
        self.expect_kw("drop")
        self.accept_kw("temporary")
        what = self.next().val.lower()
        ie = False
        if self.accept_kw("if"):
            self.expect_kw("exists")
            ie = True
        name = self.qualified_name()
        return Drop(name, what, ie)

    # -- queries
    def query(self) -> Query:
        ctes = []
        if self.accept_kw("with"):
            while True:
                name = self.ident()
                self.expect_kw("as")
                self.expect_op("(")
                q = self.query()
                self.expect_op(")")
                ctes.append((name, q))
                if not self.accept_op(","):
                    break
        body = self.set_expr()
        return Query(body, ctes)

    def set_expr(self):
        first = self.select_or_paren()
        parts = [first]
        all_ = True
        while self.accept_kw("union"):
            if self.accept_kw("all"):
                pass
            else:
                self.accept_kw("distinct")
                all_ = False
            parts.append(self.select_or_paren())
        if len(parts) == 1:
            return first
        u = Union(parts, all_)
        last = parts[-1]
        if isinstance(last, Select) and (last.order_by or last.limit is not None):
            # a trailing ORDER BY / LIMIT belongs to the whole UNION (Hive), not its last branch
            u.order_by, u.limit, u.offset = last.order_by, last.limit, last.offset
            last.order_by, last.limit, last.offset = [], None, 0
        if self.t.is_kw("order", "sort"):
            self.next()
            self.expect_kw("by")
            u.order_by = self.order_list()
        if self.accept_kw("limit"):
            u.limit = int(self.next().val)
            if self.accept_op(","):
                u.offset, u.limit = u.limit, int(self.next().val)
        return u

    def select_or_paren(self):
        if self.t.is_op("("):
            self.next()
            q = self.query()
            self.expect_op(")")
            return q
        return self.select()

    def select(self) -> Select:
        self.expect_kw("select")
        distinct = self.accept_kw("distinct")
        self.accept_kw("all")
        items = [self.select_item()]
        while self.accept_op(","):
            items.append(self.select_item())
        s = Select(items, distinct=distinct)
        if self.accept_kw("from"):
            s.source = self.from_clause()
        if self.accept_kw("where"):
            s.where = self.expr()
        if self.t.is_kw("group"):
            self.next()
            self.expect_kw("by")
            s.group_by = [self.expr()]
            while self.accept_op(","):
                s.group_by.append(self.expr())
            s.grouping_sets = self._grouping_sets(s.group_by)
        if self.accept_kw("having"):
            s.having = self.expr()
        while self.t.is_kw("order", "sort", "cluster", "distribute"):
            kw = self.next().val
            self.expect_kw("by")
            if kw in ("order", "sort"):
                s.order_by = self.order_list()
            elif kw == "cluster":
                s.cluster_by = [self.expr()]
                while self.accept_op(","):
                    s.cluster_by.append(self.expr())
                s.order_by = s.order_by or [(e, True) for e in s.cluster_by]
            else:
                self.expr()
                while self.accept_op(","):
                    self.expr()
        if self.accept_kw("limit"):
            s.limit = int(self.next().val)
            if self.accept_op(","):
                s.offset, s.limit = s.limit, int(self.next().val)
        return s

    def order_list(self):
        out = []
        while True:
            e = self.expr()
            asc = True
            if self.accept_kw("asc"):
                asc = True
            elif self.accept_kw("desc"):
                asc = False
            if self.accept_kw("nulls"):
                self.next()
            out.append((e, asc))
            if not self.accept_op(","):
                break
        return out

    def select_item(self) -> SelectItem:
        if self.t.is_op("*"):
            self.next()
            return SelectItem(Star())
        if self.is_ident() and self.peek().is_op(".") and self.peek(2).is_op("*"):
            tname = self.ident()
            self.next()
            self.next()
            return SelectItem(Star(tname))
        e = self.expr()
        if self.accept_kw("as"):
            if self.t.is_op("("):
                self.next()
                names = [self.ident()]
                while self.accept_op(","):
                    names.append(self.ident())
                self.expect_op(")")
                return SelectItem(e, aliases=names)
            name = self.ident()
            if self.t.is_op(","):
                # UDTF AS a, b (Hive also accepts the unparenthesised form for UDTFs)
                if isinstance(e, Func) and self._looks_like_alias_list():
                    names = [name]
                    while self.t.is_op(",") and self._looks_like_alias_list():
                        self.next()
                        names.append(self.ident())
                    return SelectItem(e, aliases=names)
            return SelectItem(e, alias=name)
        if self.is_ident() and not self.t.is_kw("from"):
            return SelectItem(e, alias=self.ident())
        return SelectItem(e)

    def _looks_like_alias_list(self) -> bool:
        return False

    def from_clause(self):
        left = self.table_primary()
        while True:
            if self.accept_op(","):
                right = self.table_primary()
                left = Join(left, right, "cross")
                continue
            kind = None
            if self.t.is_kw("join"):
                kind = "inner"
            elif self.t.is_kw("inner") and self.peek().is_kw("join"):
                self.next()
                kind = "inner"
            elif self.t.is_kw("left", "right", "full"):
                k = self.t.val
                if self.peek().is_kw("semi"):
                    self.next()
                    self.next()
                    kind = "semi"
                else:
                    self.next()
                    self.accept_kw("outer")
                    kind = k
            elif self.t.is_kw("cross"):
                self.next()
                kind = "cross"
            elif self.t.is_kw("lateral"):
                self.next()
                self.expect_kw("view")
                outer = self.accept_kw("outer")
                f = self.primary()
                if not isinstance(f, Func):
                    self.error("LATERAL VIEW needs a table function")
                talias = None
                if self.is_ident() and not self.t.is_kw("as"):
                    talias = self.ident()
                cols = []
                if self.accept_kw("as"):
                    cols = [self.ident()]
                    while self.t.is_op(",") and (self.peek().kind == "ident" or (self.peek().kind == "kw" and self.peek().val not in RESERVED)):
                        self.next()
                        cols.append(self.ident())
                left = LateralView(left, f, talias, cols, outer)
                continue
            if kind is None:
                return left
            self.expect_kw("join")
            right = self.table_primary()
            on = None
            if self.accept_kw("on"):
                on = self.expr()
            left = Join(left, right, kind, on)

    def table_primary(self):
        if self.t.is_op("("):
            self.next()
            if self.t.is_kw("select", "with") or self.t.is_op("("):
                q = self.query()
                self.expect_op(")")
                sample = self._tablesample()
                alias = None
                self.accept_kw("as")
                if self.is_ident():
                    alias = self.ident()
                return SubqueryRef(q, alias, sample)
            f = self.from_clause()
            self.expect_op(")")
            return f
        name = self.qualified_name()
        sample = self._tablesample()
        alias = None
        if self.accept_kw("as"):
            alias = self.ident()
        elif self.is_ident() and not self.t.is_kw("lateral", "left", "right", "full", "cross", "inner",
                                                  "join", "where", "group", "order", "on", "limit",
                                                  "sort", "cluster", "distribute", "having", "union",
                                                  "insert", "select"):
            alias = self.ident()
        return TableRef(name, alias, sample)

    def _tablesample(self):
        """TABLESAMPLE (BUCKET x OUT OF y [ON expr]) | (n PERCENT) | (n ROWS)."""
        if not (self.t.kind == "ident" and self.t.val.lower() == "tablesample"):
            return None
        self.next()
        self.expect_op("(")
        if self.t.kind == "ident" and self.t.val.lower() == "bucket":
            self.next()
            x = int(self.next().val)
            if not (self.t.kind == "ident" and self.t.val.lower() == "out"):
                self.error("expected OUT OF")
            self.next()
            if not self.accept_kw("of"):
                if not (self.t.kind == "ident" and self.t.val.lower() == "of"):
                    self.error("expected OUT OF")
                self.next()
            y = int(self.next().val)
            if not 1 <= x <= y:
                self.error("TABLESAMPLE bucket must be in 1..y")
            on = self.expr() if self.accept_kw("on") else None
            self.expect_op(")")
            return ("bucket", x, y, on)
        if self.t.kind != "num":
            self.error("expected BUCKET, n PERCENT or n ROWS")
        v = self.next().val
        unit = self.next().val.lower()
        self.expect_op(")")
        if unit == "percent":
            return ("percent", float(v))
        if unit == "rows":
            return ("rows", int(v))
        self.error("expected PERCENT or ROWS")

    # -- expressions (precedence climbing)
    def expr(self) -> Expr:
        return self.or_expr()

    def or_expr(self):
        e = self.and_expr()
        while self.accept_kw("or"):
            e = BinOp("or", e, self.and_expr())
        return e

    def and_expr(self):
        e = self.not_expr()
        while self.accept_kw("and") or self.accept_op("&&"):
            e = BinOp("and", e, self.not_expr())
        return e

    def not_expr(self):
        if self.accept_kw("not") or self.accept_op("!"):
            return UnOp("not", self.not_expr())
        return self.cmp_expr()

    def cmp_expr(self):
        e = self.concat_expr()
        while True:
            if self.t.is_op("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
                op = self.next().val
                op = {"==": "=", "<>": "!="}.get(op, op)
                e = BinOp(op, e, self.concat_expr())
                continue
            neg = False
            save = self.i
            if self.t.is_kw("not") and self.peek().is_kw("in", "between", "like", "rlike", "regexp"):
                self.next()
                neg = True
            if self.accept_kw("is"):
                n = self.accept_kw("not")
                self.expect_kw("null")
                e = IsNull(e, n)
                continue
            if self.accept_kw("in"):
                self.expect_op("(")
                if self.t.is_kw("select", "with"):
                    q = self.query()
                    self.expect_op(")")
                    e = InList(e, [SubqueryExpr(q)], neg)
                    continue
                items = [self.expr()]
                while self.accept_op(","):
                    items.append(self.expr())
                self.expect_op(")")
                e = InList(e, items, neg)
                continue
            if self.accept_kw("between"):
                lo = self.concat_expr()
                self.expect_kw("and")
                hi = self.concat_expr()
                e = Between(e, lo, hi, neg)
                continue
            if self.t.is_kw("like", "rlike", "regexp"):
                rx = self.next().val != "like"
                e = Like(e, self.concat_expr(), rx, neg)
                continue
            self.i = save
            return e

    def concat_expr(self):
        e = self.add_expr()
        while self.accept_op("||"):
            e = Func("concat", [e, self.add_expr()])
        return e

    def add_expr(self):
        e = self.mul_expr()
        while self.t.is_op("+", "-"):
            op = self.next().val
            e = BinOp(op, e, self.mul_expr())
        return e

    def mul_expr(self):
        e = self.bit_expr()
        while self.t.is_op("*", "/", "%") or self.t.is_kw("div"):
            op = self.next().val
            e = BinOp(op, e, self.bit_expr())
        return e

    def bit_expr(self):
        e = self.unary()
        while self.t.is_op("&", "|", "^"):
            op = self.next().val
            e = BinOp(op, e, self.unary())
        return e

    def unary(self):
        if self.accept_op("-"):
            return UnOp("-", self.unary())
        if self.accept_op("+"):
            return self.unary()
        if self.accept_op("~"):
            return UnOp("~", self.unary())
        return self.postfix()

    def postfix(self):
        e = self.primary()
        while True:
            if self.accept_op("["):
                idx = self.expr()
                self.expect_op("]")
                e = Index(e, idx)
            elif self.t.is_op(".") and not isinstance(e, Col):
                self.next()
                e = Field(e, self.ident())
            else:
                return e

    def primary(self) -> Expr:
        t = self.t
        if t.kind == "num":
            self.next()
            v = t.val
            if any(c in v for c in ".eE"):
                return Lit(float(v))
            return Lit(int(v))
        if t.kind == "str":
            self.next()
            s = t.val
            while self.t.kind == "str":   # adjacent literals concatenate
                s += self.next().val
            return Lit(s)
        if t.is_kw("null"):
            self.next()
            return Lit(None)
        if t.is_kw("true", "false"):
            self.next()
            return Lit(t.val == "true")
        if t.is_op("("):
            self.next()
            if self.t.is_kw("select", "with"):
                q = self.query()
                self.expect_op(")")
                return SubqueryExpr(q)
            e = self.expr()
            self.expect_op(")")
            return e
        if t.is_kw("exists") and self.peek().is_op("("):
            self.next()
            self.next()
            q = self.query()
            self.expect_op(")")
            return Exists(q)
        if t.is_kw("case"):
            self.next()
            base = None
            if not self.t.is_kw("when"):
                base = self.expr()
            whens = []
            while self.accept_kw("when"):
                c = self.expr()
                self.expect_kw("then")
                whens.append((c, self.expr()))
            d = None
            if self.accept_kw("else"):
                d = self.expr()
            self.expect_kw("end")
            return Case(base, whens, d)
        if t.is_kw("cast"):
            self.next()
            self.expect_op("(")
            e = self.expr()
            self.expect_kw("as")
            ty = self._type_name()
            self.expect_op(")")
            return Cast(e, ty)
        if t.is_kw("if") and self.peek().is_op("("):
            self.next()
            return self._call("if")
        if (t.kind == "ident" or (t.kind == "kw" and t.val not in RESERVED)) and self.peek().is_op("("):
            name = self.next().val
            return self._call(name)
        if t.kind == "ident" or (t.kind == "kw" and t.val not in RESERVED):
            name = self.next().val
            if self.t.is_op(".") and (self.peek().kind == "ident" or (self.peek().kind == "kw" and self.peek().val not in RESERVED)):
                self.next()
                col = self.next().val
                if self.t.is_op("("):   # db.func(...)
                    return self._call(col)
                return Col(col, name)
            return Col(name)
        self.error("unexpected token in expression")

    def _type_name(self) -> str:
        parts = [self.next().val]
        if self.t.is_op("<"):
            depth = 0
            while True:
                tk = self.next()
                parts.append(tk.val)
                if tk.is_op("<"):
                    depth += 1
                elif tk.is_op(">"):
                    depth -= 1
                    if depth == 0:
                        break
        elif self.t.is_op("("):
            while not self.t.is_op(")"):
                parts.append(self.next().val)
            parts.append(self.next().val)
        return "".join(parts).lower()

    def _grouping_sets(self, keys: list):
        """``WITH ROLLUP`` / ``WITH CUBE`` / ``GROUPING SETS ((a, b), a, ())`` after a GROUP BY
        list: the key subsets to aggregate over, as index lists into ``keys``."""
        n = len(keys)
        if self.t.is_kw("with") and self.peek().kind == "ident" and self.peek().val.lower() in ("rollup", "cube"):
            self.next()
            kind = self.next().val.lower()
            if kind == "rollup":
                return [list(range(k)) for k in range(n, -1, -1)]
            return [[i for i in range(n) if m >> (n - 1 - i) & 1] for m in range((1 << n) - 1, -1, -1)]
        if not (self.t.kind == "ident" and self.t.val.lower() == "grouping"):
            return None
        self.next()
        if not (self.t.kind == "ident" and self.t.val.lower() == "sets"):
            self.error("expected GROUPING SETS")
        self.next()
        self.expect_op("(")

        def key_index(e):
            for i, k in enumerate(keys):
                if k == e:
                    return i
            self.error("a grouping set may only name GROUP BY expressions")

        sets = []
        while True:
            if self.accept_op("("):
                cur = []
                if not self.t.is_op(")"):
                    cur.append(key_index(self.expr()))
                    while self.accept_op(","):
                        cur.append(key_index(self.expr()))
                self.expect_op(")")
            else:
                cur = [key_index(self.expr())]
            sets.append(sorted(set(cur)))
            if not self.accept_op(","):
                break
        self.expect_op(")")
        return sets

    def _frame_bound(self):
        if self.accept_kw("unbounded"):
            if not self.t.is_kw("preceding", "following"):
                self.error("expected PRECEDING or FOLLOWING")
            self.next()
            return None
        if self.accept_kw("current"):
            self.expect_kw("row")
            return 0
        if self.t.kind != "num":
            self.error("expected a window frame bound")
        n = int(self.next().val)
        if self.accept_kw("preceding"):
            return -n
        self.expect_kw("following")
        return n

    def _arg(self) -> Expr:
        """A call argument; ``*`` / ``t.*`` stand for every column of the source (Hive's
        ``amplify(3, *)``), expanded by the executor."""
        if self.t.is_op("*"):
            self.next()
            return Star()
        if self.is_ident() and self.peek().is_op(".") and self.peek(2).is_op("*"):
            tname = self.ident()
            self.next(); self.next()
            return Star(tname)
        return self.expr()

    def _call(self, name: str) -> Func:
        self.expect_op("(")
        distinct = self.accept_kw("distinct")
        args = []
        star = False
        if self.t.is_op("*"):
            self.next()
            star = True
        elif not self.t.is_op(")"):
            args.append(self._arg())
            while self.accept_op(","):
                args.append(self._arg())
        self.expect_op(")")
        f = Func(name.lower(), args, distinct, star)
        if self.accept_kw("over"):
            self.expect_op("(")
            part, order = [], []
            if self.accept_kw("partition"):
                self.expect_kw("by")
                part = [self.expr()]
                while self.accept_op(","):
                    part.append(self.expr())
            if self.t.is_kw("order", "sort"):
                self.next()
                self.expect_kw("by")
                order = self.order_list()
            frame = None
            if self.t.is_kw("rows", "range"):
                unit = self.next().val
                if self.accept_kw("between"):
                    lo = self._frame_bound()
                    self.expect_kw("and")
                    frame = (unit, lo, self._frame_bound())
                else:
                    frame = (unit, self._frame_bound(), 0)
            self.expect_op(")")
            f.window = Window(part, order, frame)
        return f


def parse(sql: str):
    return Parser(sql).statement()


def parse_expr(sql: str) -> Expr:
    p = Parser(sql)
    e = p.expr()
    if p.t.kind != "eof":
        p.error("trailing input after expression")
    return e
