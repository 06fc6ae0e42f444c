"""Data tables from files — what Hive's storage layer did for Hivemall scripts (SURVEY.md §3.1:
``CREATE EXTERNAL TABLE ... ROW FORMAT DELIMITED ... LOCATION``, ``LOAD DATA INPATH``, ``INSERT
OVERWRITE DIRECTORY``).

Formats (``fmt`` or the file extension):

* ``parquet`` (``.parquet`` / ``.pq``): read through pyarrow with Arrow-backed columns, so a
  ``list<string>`` feature column reaches the learners' ingest as its buffers;
* ``text`` (Hive ``TEXTFILE``; ``.tsv`` / ``.txt`` / ``.csv`` / anything else): one row per
  line, fields split by ``field_delim`` (Hive's default ``\\001``; ``.tsv`` tab, ``.csv``
  comma), ``array<...>`` columns split by ``collection_delim`` (default ``\\002``, or ``,``
  when the field delimiter is not a comma), ``\\N`` = NULL.  Field and array splitting run in
  Arrow's C++ kernels (no Python object per feature);
* ``libsvm`` (``.libsvm`` / ``.svm``): ``label idx:val idx:val ...`` -> ``(label double,
  features array<string>)``, Hivemall's a9a / news20 tutorial input;
* ``jsonl`` (``.jsonl`` / ``.json``): one JSON object per line.

A directory location reads every non-hidden file in it, in name order.
"""
from __future__ import annotations

import os
import re

import numpy as np
import pandas as pd

_EXT_FMT = {".parquet": "parquet", ".pq": "parquet", ".libsvm": "libsvm", ".svm": "libsvm",
            ".jsonl": "jsonl", ".json": "jsonl"}
_NUMERIC = {"tinyint": "int64", "smallint": "int64", "int": "int64", "integer": "int64",
            "bigint": "int64", "float": "float64", "double": "float64", "decimal": "float64"}


def _files(path: str) -> list[str]:
    if os.path.isdir(path):
        fs = sorted(os.path.join(path, f) for f in os.listdir(path)
                    if not f.startswith((".", "_")) and os.path.isfile(os.path.join(path, f)))
        if not fs:
            raise FileNotFoundError(f"no data files under {path}")
        return fs
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return [path]


def table_format(path: str, fmt: str | None = None) -> str:
    if fmt:
        f = fmt.lower()
        return {"textfile": "text", "sequencefile": "text", "orc": "parquet", "tsv": "text",
                "csv": "text", "json": "jsonl"}.get(f, f)
    p = _files(path)[0] if os.path.isdir(path) else path
    return _EXT_FMT.get(os.path.splitext(p)[1].lower(), "text")


def _default_delims(path: str, field_delim: str | None, collection_delim: str | None):
    ext = os.path.splitext(path)[1].lower()
    fd = field_delim if field_delim is not None else {".tsv": "\t", ".txt": "\t", ".csv": ","}.get(ext, "\x01")
    cd = collection_delim if collection_delim is not None else ("\x02" if fd in ("\x01", ",") else ",")
    return fd, cd


def _base_type(t: str) -> str:
    return re.split(r"[<(\s]", t.strip().lower(), maxsplit=1)[0]


def _read_text(path, columns, types, field_delim, collection_delim) -> pd.DataFrame:
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.csv as pcsv

    fd, cd = _default_delims(path, field_delim, collection_delim)
    if len(fd) != 1:
        raise ValueError(f"field delimiter must be one character, got {fd!r}")
    tabs = []
    for f in _files(path):
        ncol = len(columns) if columns else None
        ro = pcsv.ReadOptions(column_names=list(columns) if columns else None,
                              autogenerate_column_names=not columns, block_size=1 << 26)
        po = pcsv.ParseOptions(delimiter=fd, quote_char=False, escape_char=False)
        co = pcsv.ConvertOptions(column_types={c: pa.string() for c in (columns or [])} or None,
                                 null_values=["\\N"], strings_can_be_null=True)
        t = pcsv.read_csv(f, read_options=ro, parse_options=po, convert_options=co)
        if ncol is not None and t.num_columns != ncol:
            raise ValueError(f"{f}: {t.num_columns} fields per row, table declares {ncol}")
        tabs.append(t)
    t = pa.concat_tables(tabs) if len(tabs) > 1 else tabs[0]
    out = {}
    for i, name in enumerate(t.column_names):
        col = t.column(i).combine_chunks()
        ty = _base_type(types[i]) if types and i < len(types) and types[i] else ""
        if ty == "array":
            inner = _base_type(re.sub(r"^array\s*<", "", types[i].strip().lower()))
            lst = pc.split_pattern(col.cast(pa.string()), cd)
            if inner in _NUMERIC:
                lst = lst.cast(pa.list_(pa.float64() if _NUMERIC[inner] == "float64" else pa.int64()))
            out[name] = pd.Series(pd.arrays.ArrowExtensionArray(lst))
        elif ty in _NUMERIC:
            out[name] = col.cast(pa.float64() if _NUMERIC[ty] == "float64" else pa.int64()).to_pandas()
        elif ty == "boolean":
            out[name] = pc.equal(pc.utf8_lower(col.cast(pa.string())), "true").to_pandas()
        elif ty in ("string", "varchar", "char") or types:
            out[name] = col.cast(pa.string()).to_pandas()
        else:
            out[name] = col.to_pandas()          # no declared types: Arrow's inference
    return pd.DataFrame(out)


def _read_libsvm(path: str, columns) -> pd.DataFrame:
    import pyarrow as pa
    import pyarrow.compute as pc

    lines = []
    for f in _files(path):
        with open(f, "rb") as fh:
            lines.append(fh.read().decode("utf-8"))
    text = pa.array([ln for part in lines for ln in part.splitlines() if ln.strip()], type=pa.string())
    toks = pc.split_pattern_regex(pc.utf8_trim_whitespace(text), r"\s+")
    label = pc.list_element(toks, 0).cast(pa.float64())
    feats = pc.list_slice(toks, 1)
    names = list(columns) if columns else ["label", "features"]
    return pd.DataFrame({names[0]: label.to_pandas(),
                         names[1]: pd.Series(pd.arrays.ArrowExtensionArray(feats.cast(pa.list_(pa.string()))))})


def read_table(path: str, fmt: str | None = None, columns=None, types=None,
               field_delim: str | None = None, collection_delim: str | None = None) -> pd.DataFrame:
    """A data table from ``path`` (file or directory); ``columns`` / ``types`` as declared by
    ``CREATE TABLE`` (Hive type names; ``array<...>`` columns are split)."""
    f = table_format(path, fmt)
    if f == "parquet":
        import pyarrow.parquet as pq

        df = pd.concat([pq.read_table(p).to_pandas(types_mapper=pd.ArrowDtype) for p in _files(path)],
                       ignore_index=True)
        if columns:
            if len(columns) != df.shape[1]:
                raise ValueError(f"{path}: {df.shape[1]} columns, table declares {len(columns)}")
            df.columns = list(columns)
        return df
    if f == "libsvm":
        return _read_libsvm(path, columns)
    if f == "jsonl":
        df = pd.concat([pd.read_json(p, lines=True) for p in _files(path)], ignore_index=True)
        return df[list(columns)] if columns else df
    if f != "text":
        raise ValueError(f"unsupported table format {fmt!r}")
    return _read_text(path, columns, types, field_delim, collection_delim)


def _text_scalar(v) -> str:
    if v is None or v is pd.NA or (isinstance(v, float) and np.isnan(v)):
        return "\\N"
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"           # Hive's boolean text
    return str(v)


def _text_cell(v, cd: str) -> str:
    if isinstance(v, (list, tuple, np.ndarray)):
        return cd.join(_text_scalar(x) for x in v)
    return _text_scalar(v)


def write_table(df: pd.DataFrame, path: str, fmt: str | None = None, field_delim: str | None = None,
                collection_delim: str | None = None, overwrite_dir: bool = False) -> str:
    """Write a query result as Hive would for ``INSERT OVERWRITE DIRECTORY``: parquet, jsonl or
    delimited text (``\\N`` for NULL, arrays joined by the collection delimiter).  A path
    without an extension is a directory; the data goes to ``000000_0`` in it."""
    f = (fmt or "").lower() or _EXT_FMT.get(os.path.splitext(path)[1].lower(), "text")
    f = table_format(path, f) if fmt else f
    target = path
    if not os.path.splitext(path)[1]:
        os.makedirs(path, exist_ok=True)
        # INSERT OVERWRITE DIRECTORY (``overwrite_dir``) replaces the directory's data as Hive
        # does: every data file (any regular file not hidden by a leading '.' or '_', the files
        # a directory read picks up) goes first, so a stale 000000_0 of another format is never
        # read back
        for name in (os.listdir(path) if overwrite_dir else ()):
            fp = os.path.join(path, name)
            if not name.startswith((".", "_")) and os.path.isfile(fp):
                os.remove(fp)
        target = os.path.join(path, "000000_0" + (".parquet" if f == "parquet" else ""))
    else:
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    if f == "parquet":
        import pyarrow as pa
        import pyarrow.parquet as pq

        pq.write_table(pa.Table.from_pandas(df, preserve_index=False), target)
        return target
    if f == "jsonl":
        df.to_json(target, orient="records", lines=True)
        return target
    fd, cd = _default_delims(target, field_delim, collection_delim)
    with open(target, "w") as fh:
        cols = [df[c].tolist() for c in df.columns]
        for row in zip(*cols):
            fh.write(fd.join(_text_cell(v, cd) for v in row))
            fh.write("\n")
    return target
