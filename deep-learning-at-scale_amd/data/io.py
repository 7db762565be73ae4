"""Dataset ingest (replaces ``spark.read.csv(path, header=False, schema=schema)``, cnn.py:65).

Headerless CSV by default (as the reference), explicit schema from the submission strings
(data/schema.py). Parsing is done by the framework's own multithreaded C++ reader
(csrc/runtime/csv.cpp via data/native.py), or by Arrow's (pyarrow) when the native runtime
is not built: columns come back typed per the schema (int -> int32 = Spark IntegerType, float ->
float32 = FloatType, string -> utf8). Rows whose numeric cells fail to parse become nulls
in Spark; here they are dropped (and counted) because the regression models cannot use
them. Multi-rank jobs read the file once per rank and take a deterministic shard of the
rows AFTER the seeded split, so every rank agrees on the split (call site C5).
"""
from __future__ import annotations

import numpy as np

from .schema import FLOAT, INT, Schema
from .synth import TABLE_COLUMNS, TABLE_TYPES, well_log_table


def read_csv(path: str, schema: Schema, header: bool = False, block_size: int = 1 << 24) -> dict:
    """Native multithreaded C++ parser (csrc/runtime/csv.cpp) when built; Arrow otherwise."""
    from . import native

    if native.wanted():
        return native.read_csv(path, schema, header=header)
    return read_csv_arrow(path, schema, header=header, block_size=block_size)


def read_csv_arrow(path: str, schema: Schema, header: bool = False, block_size: int = 1 << 24) -> dict:
    import pyarrow as pa
    import pyarrow.csv as pacsv

    types = {f.name: (pa.int32() if f.kind == INT else pa.float32() if f.kind == FLOAT else pa.string())
             for f in schema.fields}
    read_opts = pacsv.ReadOptions(
        column_names=None if header else schema.names, autogenerate_column_names=False,
        skip_rows=0, block_size=block_size, use_threads=True)
    conv = pacsv.ConvertOptions(column_types=types, include_columns=schema.names,
                                strings_can_be_null=False, quoted_strings_can_be_null=False)
    parse = pacsv.ParseOptions(invalid_row_handler=lambda row: "skip")
    try:  # fast path: typed columnar parse
        tbl = pacsv.read_csv(path, read_options=read_opts, parse_options=parse, convert_options=conv)
        tolerant = False
    except pa.ArrowInvalid:  # a cell failed its type: parse as text, coerce per column
        conv = pacsv.ConvertOptions(column_types={n: pa.string() for n in schema.names},
                                    include_columns=schema.names, strings_can_be_null=False)
        tbl = pacsv.read_csv(path, read_options=read_opts, parse_options=parse, convert_options=conv)
        tolerant = True
    out = {}
    valid = np.ones(tbl.num_rows, dtype=bool)
    for f in schema.fields:
        col = tbl.column(f.name)
        if f.is_numeric:
            if tolerant:
                import pandas as pd

                num = pd.to_numeric(pd.Series(col.to_pylist()), errors="coerce").to_numpy()
                if f.kind == INT:
                    num = np.where(np.floor(num) == num, num, np.nan)
                bad = np.isnan(num)
                valid &= ~bad
                out[f.name] = np.where(bad, 0, num).astype(np.int64 if f.kind == INT else np.float32)
                continue
            valid &= ~np.asarray(col.is_null().to_numpy(zero_copy_only=False))
            arr = col.to_numpy(zero_copy_only=False)
            out[f.name] = np.asarray(arr, dtype=np.int64 if f.kind == INT else np.float32)
        else:
            out[f.name] = np.asarray(col.to_pylist(), dtype=object)
    if not valid.all():
        out = {k: v[valid] for k, v in out.items()}
    return out


def write_csv(table: dict, path: str, columns=None, header: bool = False) -> None:
    import pyarrow as pa
    import pyarrow.csv as pacsv

    cols = columns or list(table.keys())
    tbl = pa.table({c: np.asarray(table[c]) if table[c].dtype != object else list(table[c]) for c in cols})
    pacsv.write_csv(tbl, path, write_options=pacsv.WriteOptions(include_header=header))


def load_table(data: str, schema: Schema, header: bool = False, synth_wells: int = 16,
               synth_steps: int = 600, seed: int = 0) -> dict:
    """CSV path, or 'synth' for the Gilbert well-log generator (columns must exist there)."""
    if data in ("synth", "synthetic", ""):
        full = well_log_table(synth_wells, synth_steps, seed=seed)
        missing = [n for n in schema.names if n not in full]
        if missing:
            raise ValueError(
                f"synthetic data has columns {TABLE_COLUMNS} ({','.join(TABLE_TYPES)}); "
                f"unknown column(s) {missing}")
        out = {}
        for f in schema.fields:
            v = full[f.name]
            if f.kind == INT:
                v = np.asarray(v).astype(np.int64)
            elif f.kind == FLOAT:
                v = np.asarray(v).astype(np.float32)
            else:
                v = np.asarray([str(x) for x in v], dtype=object)
            out[f.name] = v
        return out
    return read_csv(data, schema, header=header)
