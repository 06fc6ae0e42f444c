"""Command-line HiveQL runner — the ``hive -f script.hql`` / ``hive -e`` of this engine.

    python -m hivemall_amd.sql -f train.sql [--device cuda] [--table a9a=a9a.libsvm]
        [--hivevar k=v ...] [--out model.parquet] [--show 20]
    python -m hivemall_amd.sql -e "SELECT hivemall_version()"
    python -m hivemall_amd.sql < script.sql          # statements from stdin; a terminal gets
                                                      # an interactive ``hivemall>`` prompt

Scripts run statement by statement in one :class:`Session`: ``CREATE TABLE ... LOCATION``,
``LOAD DATA`` and ``INSERT OVERWRITE DIRECTORY`` move files in and out (io/tables.py);
``--table name=path[:format]`` registers a file before the script runs.  The last statement's
result is printed (``--show`` rows) or written to ``--out``.  Under ``torchrun`` every rank runs
the script and the learner UDTFs train data-parallel over RCCL (Session docstring); rank 0
prints / writes.
"""
from __future__ import annotations

import argparse
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m hivemall_amd.sql", description=__doc__.split("\n\n")[0])
    ap.add_argument("-f", "--file", action="append", default=[], help="HiveQL script (repeatable)")
    ap.add_argument("-e", "--execute", action="append", default=[], help="HiveQL text (repeatable)")
    ap.add_argument("--device", default=None, help="cpu | cuda (default: cuda when available)")
    ap.add_argument("--table", action="append", default=[], metavar="NAME=PATH[:FORMAT]",
                    help="register a file (parquet, text, libsvm, jsonl) as a table")
    ap.add_argument("--hivevar", action="append", default=[], metavar="K=V",
                    help="${hivevar:K} / ${K} substitution")
    ap.add_argument("--out", default=None, help="write the last result (parquet / tsv / csv / jsonl)")
    ap.add_argument("--show", type=int, default=20, help="rows of the last result to print")
    a = ap.parse_args(argv)

    rank = 0
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from ..parallel.dist import init_distributed

        ctx = init_distributed(device=a.device)
        rank = ctx.rank
    from ..io.tables import read_table, write_table
    from . import Session

    s = Session(device=a.device)
    for kv in a.hivevar:
        k, _, v = kv.partition("=")
        s.vars[k.strip()] = v
    for spec in a.table:
        name, _, path = spec.partition("=")
        fmt = None
        if ":" in path and not os.path.exists(path):
            path, _, fmt = path.rpartition(":")
        s.register(name.strip(), read_table(path, fmt))

    def show(df):
        import pandas as pd

        with pd.option_context("display.max_columns", 50, "display.width", 160):
            print(df.head(a.show).to_string(index=False))
            if len(df) > a.show:
                print(f"... ({len(df)} rows)")

    out = None
    for path in a.file:
        out = s.run_script(path)
    for text in a.execute:
        out = s.sql(text)
    if not a.file and not a.execute:
        if sys.stdin.isatty():
            return _repl(s, show)
        out = s.sql(sys.stdin.read())
    if rank == 0 and out is not None:
        if a.out:
            print(f"wrote {len(out)} rows to {write_table(out, a.out)}")
        else:
            show(out)
    return 0


def _repl(session, show) -> int:
    """``hivemall>`` prompt: statements end at ``;``; errors are printed, not fatal."""
    from .lexer import split_statements

    buf = ""
    while True:
        try:
            line = input("hivemall> " if not buf.strip() else "    ...> ")
        except EOFError:
            print()
            return 0
        if not buf.strip() and line.strip().lower() in ("quit", "exit", "quit;", "exit;"):
            return 0
        buf += line + "\n"
        if not line.rstrip().endswith(";"):
            continue
        for stmt in split_statements(buf):
            try:
                r = session.sql(stmt)
                if r is not None:
                    show(r)
            except Exception as e:          # the session stays usable after a bad statement
                print(f"FAILED: {type(e).__name__}: {e}")
        buf = ""


if __name__ == "__main__":
    sys.exit(main())
