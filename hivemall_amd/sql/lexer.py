"""HiveQL lexer (the subset used by Hivemall's documented scripts)."""
from __future__ import annotations

import re
from dataclasses import dataclass

KEYWORDS = {
    "select", "distinct", "all", "from", "where", "group", "by", "having", "order", "sort",
    "cluster", "distribute", "limit", "as", "on", "join", "inner", "left", "right", "full",
    "outer", "cross", "semi", "lateral", "view", "union", "with", "and", "or", "not", "in",
    "is", "null", "true", "false", "between", "like", "rlike", "regexp", "case", "when", "then",
    "else", "end", "cast", "asc", "desc", "create", "table", "temporary", "external", "if",
    "exists", "insert", "overwrite", "into", "drop", "function", "macro", "set", "add", "jar",
    "source", "use", "over", "partition", "rows", "range", "unbounded", "preceding",
    "following", "current", "row", "show", "functions", "describe", "values", "div", "array",
    "map", "struct", "stored", "location", "row", "format", "delimited", "fields", "terminated",
    "tblproperties", "comment", "partitioned", "clustered", "sorted", "buckets", "explain",
    "reload", "nulls", "first", "last", "file", "archive", "jars", "files",
}


@dataclass
class Tok:
    kind: str    # kw, ident, num, str, op, eof
    val: str
    pos: int

    def is_kw(self, *ws: str) -> bool:
        return self.kind == "kw" and self.val in ws

    def is_op(self, *ops: str) -> bool:
        return self.kind == "op" and self.val in ops


_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+)
  | (?P<comment>--[^\n]*|/\*.*?\*/)
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[LlDdFfSsYy]?(?![A-Za-z_]))
  | (?P<str>'(?:[^'\\]|\\.|'')*'|"(?:[^"\\]|\\.)*")
  | (?P<bq>`[^`]*`)
  | (?P<ident>[A-Za-z_$][A-Za-z0-9_$]*)
  | (?P<op><=>|<=|>=|<>|!=|==|\|\||&&|[=<>+\-*/%(),.;\[\]:!~&|^])
""", re.VERBOSE | re.DOTALL)

_ESC = {"n": "\n", "t": "\t", "r": "\r", "0": "\0", "\\": "\\", "'": "'", '"': '"'}


def _unescape(s: str) -> str:
    q = s[0]
    body = s[1:-1]
    if q == "'":
        body = body.replace("''", "'")
    out = []
    i = 0
    while i < len(body):
        c = body[i]
        if c == "\\" and i + 1 < len(body):
            m = re.match(r"[0-7]{1,3}", body[i + 1:i + 4])
            if m:                                   # Hive's octal escapes: '\001', '\t' = '\011'
                out.append(chr(int(m.group(0), 8)))
                i += 1 + len(m.group(0))
                continue
            m = re.match(r"u[0-9a-fA-F]{4}", body[i + 1:i + 6])
            if m:
                out.append(chr(int(m.group(0)[1:], 16)))
                i += 6
                continue
            out.append(_ESC.get(body[i + 1], body[i + 1]))
            i += 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


def tokenize(sql: str) -> list[Tok]:
    toks: list[Tok] = []
    pos = 0
    n = len(sql)
    while pos < n:
        m = _TOKEN_RE.match(sql, pos)
        if not m:
            raise SyntaxError(f"unexpected character {sql[pos]!r} at {pos}: ...{sql[max(0, pos - 20):pos + 20]}...")
        kind = m.lastgroup
        text = m.group(kind)
        if kind in ("ws", "comment"):
            pass
        elif kind == "num":
            t = text.rstrip("LlDdFfSsYy") if text[-1] in "LlDdFfSsYy" else text
            toks.append(Tok("num", t, pos))
        elif kind == "str":
            toks.append(Tok("str", _unescape(text), pos))
        elif kind == "bq":
            toks.append(Tok("ident", text[1:-1], pos))
        elif kind == "ident":
            low = text.lower()
            toks.append(Tok("kw", low, pos) if low in KEYWORDS else Tok("ident", text, pos))
        else:
            toks.append(Tok("op", text, pos))
        pos = m.end()
    toks.append(Tok("eof", "", n))
    return toks


def split_statements(sql: str) -> list[str]:
    """Split a script on ``;`` outside quotes / comments."""
    out = []
    buf = []
    i = 0
    n = len(sql)
    q = None
    while i < n:
        c = sql[i]
        if q:
            buf.append(c)
            if c == "\\" and i + 1 < n:
                buf.append(sql[i + 1])
                i += 2
                continue
            if c == q:
                q = None
        elif c in ("'", '"', "`"):
            q = c
            buf.append(c)
        elif c == "-" and sql.startswith("--", i):
            j = sql.find("\n", i)
            j = n if j < 0 else j
            i = j
            continue
        elif c == "/" and sql.startswith("/*", i):
            j = sql.find("*/", i + 2)
            i = n if j < 0 else j + 2
            continue
        elif c == ";":
            s = "".join(buf).strip()
            if s:
                out.append(s)
            buf = []
        else:
            buf.append(c)
        i += 1
    s = "".join(buf).strip()
    if s:
        out.append(s)
    return out
