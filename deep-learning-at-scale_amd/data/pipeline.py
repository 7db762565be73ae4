"""Per-model dataset preparation: table -> (train, val, test) tensors.

* ``mlp`` / ``mlp_online``: one row = one sample, X [n, F] (one-hot categoricals +
  standardised continuous columns), y [n].
* ``lstm``: sliding windows of ``seq_len`` rows inside each series (group column), X
  [n, T, F]; y = target at the window's last row (nowcasting the flow from the log
  history, BASELINE.json:11 "time-series regression").
* ``cnn``: the reference's shapes (cnn.py:111-114 imply input (48, 1), 12 outputs): the
  past ``cnn_input_len`` target values of a series -> the next ``cnn_outputs`` values.
* ``gilbert``: the raw physical columns (whp, choke, glr) and the raw target.

The split (0.64/0.16/0.20, cnn.py:68) is drawn per row with a fixed seed for the row
models; the windowed models (lstm, cnn) split each series into contiguous time blocks with
a one-window gap (``window_split="time"``, data/features.py time_block_split), so
overlapping windows cannot leak val/test rows into training. The feature pipeline is
fitted on the training split only.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .features import (FeaturePipeline, SeriesWindows, make_windows, random_split, take, time_block_split,
                       window_rows, window_starts)
from .io import load_table
from .schema import parse_schema


@dataclasses.dataclass
class Prepared:
    train: tuple
    val: tuple
    test: tuple
    n_features: int
    pipeline: FeaturePipeline | None
    n_outputs: int = 1
    info: dict = dataclasses.field(default_factory=dict)


def _group_ids(table, schema, group_col):
    col = group_col or next((c for c in schema.categorical() if c in table), "")
    if not col:
        return None, ""
    vals = np.asarray(table[col])
    _, ids = np.unique(vals.astype(str), return_inverse=True)
    return ids, col


def _sort_by_group(table, ids, schema):
    if ids is None:
        return table, ids
    # stable sort keeps file (time) order within each series
    order = np.argsort(ids, kind="stable")
    return take(table, order), ids[order]


def prepare(cfg) -> Prepared:
    schema = parse_schema(cfg.column_names, cfg.column_types)
    table = load_table(cfg.data, schema, header=cfg.header, synth_wells=cfg.synth_wells,
                       synth_steps=cfg.synth_steps, seed=cfg.seed)
    n = len(table[schema.names[0]])
    if cfg.model == "gilbert":
        idx = random_split(n, cfg.split, cfg.seed)
        parts = []
        for ix in idx:
            t = take(table, ix)
            parts.append(({k: np.asarray(t[k], np.float64) for k in ("whp", "choke", "glr") if k in t},
                          np.asarray(t[cfg.target], np.float64)))
        return Prepared(parts[0], parts[1], parts[2], 3, None)

    if cfg.model in ("mlp", "mlp_online"):
        idx = random_split(n, cfg.split, cfg.seed)
        pipe = FeaturePipeline(schema, cfg.target, standardize_target=True).fit(take(table, idx[0]))
        parts = [pipe.transform(take(table, ix)) for ix in idx]
        return Prepared(*parts, n_features=pipe.n_features, pipeline=pipe)

    ids, gcol = _group_ids(table, schema, cfg.group_col)
    table, ids = _sort_by_group(table, ids, schema)
    def split_windows(starts, span):
        if getattr(cfg, "window_split", "time") == "random":
            return random_split(len(starts), cfg.split, cfg.seed)
        return time_block_split(starts, span, ids, cfg.split, cfg.seed)

    if cfg.model == "lstm":
        # leak-free time-block split of the windows; the feature pipeline is fitted ONLY on
        # the rows that training windows cover
        T = cfg.seq_len
        starts = window_starts(n, T, ids)
        idx = split_windows(starts, T)
        pipe = FeaturePipeline(schema, cfg.target, standardize_target=True)
        pipe.fit(take(table, window_rows(starts[idx[0]], T)))
        X, y = pipe.transform(table)
        # lazy windows: rows + start indices, gathered per batch (on the GPU once resident)
        yw = y[starts + T - 1].astype(np.float32)
        parts = [(SeriesWindows(X, starts[ix], T), yw[ix]) for ix in idx]
        return Prepared(*parts, n_features=pipe.n_features, pipeline=pipe,
                        info={"group_col": gcol, "windows": len(starts)})
    if cfg.model == "cnn":
        L, O = cfg.cnn_input_len, cfg.cnn_outputs
        starts = window_starts(n, L + O, ids)
        idx = split_windows(starts, L + O)
        pipe = FeaturePipeline(schema, cfg.target, standardize_target=True)
        pipe.fit(take(table, window_rows(starts[idx[0]], L + O)))
        y = pipe.target_values(table)
        seq = y[:, None]  # univariate (reference input_dim=1)
        Xw, _ = make_windows(seq, y, L + O, starts=starts)
        X, Y = Xw[:, :L, :], Xw[:, L:, 0]
        parts = [(X[ix], Y[ix]) for ix in idx]
        return Prepared(*parts, n_features=1, pipeline=pipe, n_outputs=O,
                        info={"group_col": gcol, "windows": len(X)})
    raise ValueError(f"unknown model {cfg.model!r}")
