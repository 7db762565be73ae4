"""Feature engineering that replaces the reference's Spark ML pipeline (cnn.py:68-107).

Reference stages and their semantics kept here:

* ``randomSplit([0.64, 0.16, 0.2])`` (cnn.py:68) — per-row uniform draw against the
  normalised cumulative weights; now SEEDED (defect A.1#10).
* ``StringIndexer`` per categorical column (cnn.py:75) — labels ordered by frequency,
  descending, ties alphabetical (Spark >= 3 ``frequencyDesc``).
* multi-column ``OneHotEncoder`` (cnn.py:77-80) — ``dropLast=True``: the last category
  index encodes to the all-zero vector.
* ``VectorAssembler`` (cnn.py:82-85, 96-103) — ``[one-hot blocks in indexer order,
  continuous columns in schema order]``.

Fixes of reference defects: the pipeline is fitted on the
TRAINING split only and applied to all three (#3 — the reference refits per split, so
category indices disagree between splits); the target is excluded from the features
(#4); unseen labels at transform time map to an extra "unknown" index (handleInvalid
``keep``) instead of aborting the job. Continuous columns are standardised with train
statistics (the reference fed raw magnitudes; standardisation is optional).
"""
from __future__ import annotations

import dataclasses
from collections import Counter

import numpy as np

from .schema import Schema


def random_split(n: int, weights=(0.64, 0.16, 0.2), seed: int = 42):
    """Row indices of each split (Spark randomSplit semantics, seeded)."""
    w = np.asarray(weights, dtype=np.float64)
    if np.any(w < 0) or w.sum() <= 0:
        raise ValueError("split weights must be non-negative with a positive sum")
    bounds = np.cumsum(w / w.sum())
    u = np.random.default_rng(seed).random(n)
    which = np.searchsorted(bounds, u, side="right")
    which = np.minimum(which, len(w) - 1)
    return [np.nonzero(which == k)[0] for k in range(len(w))]


@dataclasses.dataclass
class StringIndexer:
    column: str
    labels: list = dataclasses.field(default_factory=list)
    handle_invalid: str = "keep"  # 'keep' | 'error' | 'skip'(treated as keep for arrays)

    def fit(self, values) -> "StringIndexer":
        cnt = Counter(str(v) for v in values)
        self.labels = [k for k, _ in sorted(cnt.items(), key=lambda kv: (-kv[1], kv[0]))]
        return self

    def transform(self, values) -> np.ndarray:
        lut = {k: i for i, k in enumerate(self.labels)}
        out = np.empty(len(values), dtype=np.int64)
        unk = len(self.labels)
        for i, v in enumerate(values):
            j = lut.get(str(v))
            if j is None:
                if self.handle_invalid == "error":
                    raise ValueError(f"unseen label {v!r} in column {self.column!r}")
                j = unk
            out[i] = j
        return out

    @property
    def num_categories(self) -> int:
        return len(self.labels) + (1 if self.handle_invalid != "error" else 0)


def one_hot(idx: np.ndarray, num_categories: int, drop_last: bool = True) -> np.ndarray:
    size = num_categories - 1 if drop_last else num_categories
    out = np.zeros((len(idx), max(size, 0)), dtype=np.float32)
    ok = idx < size
    out[np.nonzero(ok)[0], idx[ok]] = 1.0
    return out


@dataclasses.dataclass
class FeaturePipeline:
    """Fit on train, transform any split: table (dict of columns) -> (X [n, F], y [n])."""

    schema: Schema
    target: str
    standardize: bool = True
    drop_last: bool = True
    indexers: list = dataclasses.field(default_factory=list)
    mean: np.ndarray | None = None
    std: np.ndarray | None = None
    y_mean: float = 0.0
    y_std: float = 1.0
    standardize_target: bool = False

    @property
    def categorical(self):
        return self.schema.categorical(exclude=(self.target,))

    @property
    def continuous(self):
        return self.schema.continuous(exclude=(self.target,))

    def fit(self, table: dict) -> "FeaturePipeline":
        if self.target not in self.schema.names:
            raise ValueError(f"target column {self.target!r} not in schema {self.schema.names}")
        self.indexers = [StringIndexer(c).fit(table[c]) for c in self.categorical]
        X = self._assemble(table)
        if self.standardize and X.shape[1]:
            self.mean = X.mean(axis=0)
            self.std = X.std(axis=0)
            self.std[self.std < 1e-8] = 1.0
        y = self.target_values(table, raw=True)
        if self.standardize_target and len(y):
            self.y_mean, self.y_std = float(y.mean()), float(y.std() or 1.0)
        return self

    def _assemble(self, table: dict) -> np.ndarray:
        n = len(table[self.schema.names[0]])
        blocks = [one_hot(ix.transform(table[ix.column]), ix.num_categories, self.drop_last)
                  for ix in self.indexers]
        for c in self.continuous:
            blocks.append(np.asarray(table[c], dtype=np.float32).reshape(n, 1))
        return np.concatenate(blocks, axis=1) if blocks else np.zeros((n, 0), np.float32)

    def target_values(self, table: dict, raw: bool = False) -> np.ndarray:
        f = self.schema[self.target]
        if not f.is_numeric:
            # regression target must be numeric (defect A.1#5: the reference built a
            # StringIndexer for it and never used it); try a float parse.
            y = np.asarray([float(v) for v in table[self.target]], dtype=np.float32)
        else:
            y = np.asarray(table[self.target], dtype=np.float32)
        if raw or not self.standardize_target:
            return y
        return ((y - self.y_mean) / self.y_std).astype(np.float32)

    def transform(self, table: dict):
        X = self._assemble(table)
        if self.standardize and self.mean is not None:
            nc = len(self.continuous)
            # one-hot blocks are left as 0/1; only continuous columns are scaled
            if nc:
                X[:, -nc:] = (X[:, -nc:] - self.mean[-nc:]) / self.std[-nc:]
        return X.astype(np.float32), self.target_values(table)

    def inverse_target(self, y):
        return y * self.y_std + self.y_mean if self.standardize_target else y

    @property
    def n_features(self) -> int:
        return sum(max(ix.num_categories - (1 if self.drop_last else 0), 0) for ix in self.indexers) + len(
            self.continuous)

    def state(self) -> dict:
        return {
            "target": self.target,
            "categorical": {ix.column: ix.labels for ix in self.indexers},
            "mean": None if self.mean is None else self.mean.tolist(),
            "std": None if self.std is None else self.std.tolist(),
            "y_mean": self.y_mean,
            "y_std": self.y_std,
            "standardize_target": self.standardize_target,
            "drop_last": self.drop_last,
        }


def time_block_split(starts: np.ndarray, span: int, groups=None, weights=(0.64, 0.16, 0.2), seed: int = 42):
    """Leak-free split of overlapping windows (window k covers rows starts[k] .. +span-1).

    Inside every series the windows are cut, in time order, into contiguous train / val /
    test blocks of the given proportions, and the ``span - 1`` windows after each cut are
    dropped, so no row that a val or test window reads (inputs or targets) lies inside any
    training window, and none of a test window's rows inside a val window. Series too short
    to be cut that way (fewer than 3 windows per block after the gaps) are assigned WHOLE,
    seeded, in the same proportions (disjoint series cannot share rows). The reference split
    ROWS at random (cnn.py:68); a random split of stride-1 windows would put 63 of a test
    window's 64 rows into training windows. Returns index arrays into ``starts``.
    """
    w = np.asarray(weights, dtype=np.float64)
    w = w / w.sum()
    starts = np.asarray(starts, np.int64)
    gid = np.zeros(len(starts), np.int64) if groups is None else np.asarray(groups)[starts]
    out = [[] for _ in w]
    gap = max(span - 1, 0)
    short = []
    # windows of one series are consecutive in `starts` (window_starts enumerates per series)
    bounds = np.flatnonzero(np.diff(gid)) + 1
    for seg in np.split(np.arange(len(starts)), bounds):
        usable = len(seg) - gap * (len(w) - 1)
        sizes = np.floor(w * max(usable, 0)).astype(np.int64)
        if usable <= 0 or sizes.min() < 3:
            short.append(seg)
            continue
        sizes[0] += usable - sizes.sum()
        pos = 0
        for k, sz in enumerate(sizes):
            out[k].append(seg[pos: pos + sz])
            pos += sz + gap
    if short:
        order = np.random.default_rng(seed).permutation(len(short))
        cuts = np.round(np.cumsum(w) * len(short)).astype(np.int64)
        if len(short) >= len(w):  # every split gets at least one whole series
            for k in range(len(w) - 1):
                cuts[k] = min(max(cuts[k], (cuts[k - 1] if k else 0) + 1), len(short) - (len(w) - 1 - k))
        lo = 0
        for k, hi in enumerate(cuts):
            out[k].extend(short[j] for j in order[lo:hi])
            lo = hi
    return [np.concatenate(o) if o else np.zeros(0, np.int64) for o in out]


def take(table: dict, idx) -> dict:
    return {k: np.asarray(v)[idx] for k, v in table.items()}


def window_starts(n: int, T: int, groups=None, stride: int = 1) -> np.ndarray:
    """First row of every length-``T`` window that stays inside one series (``groups`` =
    per-row series id, rows in time order inside a group)."""
    from . import native

    if native.wanted():  # C++ scan (csrc/runtime/windows.cpp); the loop below is its oracle
        return native.window_starts(n, T, groups, stride)
    return window_starts_py(n, T, groups, stride)


def window_starts_py(n: int, T: int, groups=None, stride: int = 1) -> np.ndarray:
    g = np.zeros(n, dtype=np.int64) if groups is None else np.asarray(groups)
    starts = []
    i = 0
    while i < n:
        j = i
        while j < n and g[j] == g[i]:
            j += 1
        starts.extend(range(i, j - T + 1, stride))
        i = j
    return np.asarray(starts, dtype=np.int64)


def window_rows(starts: np.ndarray, T: int) -> np.ndarray:
    """Sorted unique row indices covered by the windows starting at ``starts``."""
    if len(starts) == 0:
        return np.zeros((0,), np.int64)
    return np.unique((starts[:, None] + np.arange(T)[None, :]).ravel())


def make_windows(X: np.ndarray, y: np.ndarray, T: int, groups=None, stride: int = 1, starts=None):
    """Sliding windows for sequence models: (X_w [n, T, F], y_w [n]) with y at the last step.

    ``groups`` (per-row series id, rows already in time order inside a group) keeps
    windows from crossing series boundaries; ``starts`` (from :func:`window_starts`)
    overrides the enumeration.
    """
    if starts is None:
        starts = window_starts(len(X), T, groups, stride)
    if len(starts) == 0:
        return np.zeros((0, T, X.shape[1]), np.float32), np.zeros((0,), np.float32)
    idx = starts[:, None] + np.arange(T)[None, :]
    return X[idx].astype(np.float32), y[starts + T - 1].astype(np.float32)


class SeriesWindows:
    """Length-``T`` windows over a per-row feature matrix WITHOUT materialising them.

    ``rows`` [n_rows, F] (numpy or a device tensor) + ``starts`` [n_windows]. Indexing
    returns the gathered batch [len(idx), T, F] (numpy for numpy storage; a device tensor
    gathered on the GPU for tensor storage), so a dataset costs n_rows x F instead of
    n_windows x T x F (64x less for the LSTM config) — in host RAM and, after :meth:`to`,
    resident in HBM.
    """

    def __init__(self, rows, starts, T: int):
        self.rows, self.starts, self.T = rows, starts, int(T)

    def __len__(self) -> int:
        return len(self.starts)

    @property
    def shape(self):
        return (len(self.starts), self.T, self.rows.shape[1])

    @property
    def device(self):
        return getattr(self.rows, "device", None)

    def __getitem__(self, idx):
        st = self.starts[idx]
        if hasattr(st, "unsqueeze"):  # torch
            import torch

            ar = torch.arange(self.T, device=st.device)
            return self.rows[st.reshape(-1, 1) + ar]
        st = np.asarray(st).reshape(-1)
        from . import native

        if (isinstance(self.rows, np.ndarray) and self.rows.dtype == np.float32 and self.rows.flags.c_contiguous
                and native.wanted()):  # one memcpy per window, threaded
            return native.gather_windows(self.rows, st, self.T)
        return self.rows[st[:, None] + np.arange(self.T)[None, :]]

    def to(self, device):
        import torch

        rows = torch.as_tensor(self.rows, dtype=torch.float32).to(device)
        starts = torch.as_tensor(np.asarray(self.starts, np.int64) if not hasattr(self.starts, "to") else self.starts)
        return SeriesWindows(rows, starts.to(device), self.T)

    def materialize(self):
        return self[np.arange(len(self.starts))] if not hasattr(self.starts, "to") else self[:]
