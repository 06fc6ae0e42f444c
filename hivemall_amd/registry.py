"""Function registry: Hivemall SQL function names -> implementations (the N6 layer).

Upstream registers ~200 functions with ``CREATE TEMPORARY FUNCTION <name> AS '<class>'``
in ``resources/ddl/define-all.hive``.  Here every implementation is
registered with a decorator that records its SQL kind:

* ``udf``   scalar, called per row (``impl(*args)``) or vectorised (``impl(*columns)``);
* ``udaf``  aggregate, called once per group with the group's argument columns as lists
            (``impl(*columns) -> value``);
* ``udtf``  table function.  ``per_row=True``: ``impl(*args) -> iterable of tuples`` per input
            row (explode-like, usable in ``LATERAL VIEW``).  ``per_row=False``: called once with
            every input row's arguments (``impl(*columns) -> DataFrame``) — the learners.

``hivemall_amd.functions()`` imports every module that registers functions; the SQL
frontend resolves names through :func:`lookup`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable

UDF, UDAF, UDTF = "udf", "udaf", "udtf"


@dataclass
class FunctionDef:
    name: str
    kind: str
    impl: Callable
    vectorized: bool = False
    per_row: bool = True
    cols: tuple = ()
    doc: str = ""
    aliases: tuple = field(default_factory=tuple)
    const_args: tuple = ()      # positions that must be constant (option strings)


REGISTRY: dict[str, FunctionDef] = {}


def _register(fd: FunctionDef) -> None:
    for n in (fd.name,) + tuple(fd.aliases):
        REGISTRY[n.lower()] = fd


def udf(name: str, *aliases: str, vectorized: bool = False):
    def deco(fn):
        _register(FunctionDef(name, UDF, fn, vectorized=vectorized, doc=(fn.__doc__ or "").strip(),
                              aliases=aliases))
        return fn
    return deco


def udaf(name: str, *aliases: str):
    def deco(fn):
        _register(FunctionDef(name, UDAF, fn, doc=(fn.__doc__ or "").strip(), aliases=aliases))
        return fn
    return deco


def udtf(name: str, *aliases: str, cols: tuple = (), per_row: bool = True):
    def deco(fn):
        _register(FunctionDef(name, UDTF, fn, per_row=per_row, cols=tuple(cols),
                              doc=(fn.__doc__ or "").strip(), aliases=aliases))
        return fn
    return deco


_LOADED = False


def load_all() -> dict[str, FunctionDef]:
    """Import every function module (idempotent)."""
    global _LOADED
    if not _LOADED:
        _LOADED = True
        from . import functions  # noqa: F401
    return REGISTRY


def lookup(name: str) -> FunctionDef | None:
    load_all()
    return REGISTRY.get(name.lower())


def names(kind: str | None = None) -> list[str]:
    load_all()
    return sorted(n for n, fd in REGISTRY.items() if kind is None or fd.kind == kind)
