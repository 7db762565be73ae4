"""Synthetic well-log data with a known physical ground truth.

The reference ships no data ("the features were changing at each learning job
submission", Readme.md:23-25); BASELINE.json:5 asks for synthetic well-log data. Every
generator here draws wellhead pressure, choke size and gas-liquid ratio (plus nuisance
channels: temperature, water cut, downstream pressure and a categorical well / field
id) and sets the oil rate from the Gilbert correlation (models/gilbert.py) passed
through a first-order lag (the well responds to choke changes over several steps, so a
sequence model has history to exploit) times log-normal measurement noise.

* :func:`well_log_table` — a tabular dataset (one row per well per timestep) in the
  column/type contract of the submission scripts (cnn.py:41-60 argv strings).
* :func:`synth_lstm_batch` / :func:`synth_tabular_batch` — vectorised on-the-fly
  mini-batches (standardised features, standardised log-rate target) for benchmarks.
"""
from __future__ import annotations

import numpy as np

from ..models.gilbert import GilbertModel

TABLE_COLUMNS = ["well", "field", "t", "whp", "choke", "glr", "temp", "water_cut", "dsp", "flow"]
TABLE_TYPES = ["string", "string", "int", "float", "float", "float", "float", "float", "float", "float"]
LAG = 0.7  # flow(t) = LAG * flow(t-1) + (1 - LAG) * gilbert(t)


def _series(rng, n, T):
    """Physical channels [n, T] for n independent wells."""
    whp0 = rng.uniform(300.0, 2500.0, size=(n, 1))
    decline = rng.uniform(0.0, 2e-3, size=(n, 1))
    t = np.arange(T)[None, :]
    whp = whp0 * np.exp(-decline * t) * np.exp(np.cumsum(rng.normal(0, 0.01, size=(n, T)), axis=1))
    # choke: piecewise constant with ~3 changes per 64 steps
    choke_levels = rng.uniform(12.0, 64.0, size=(n, T))
    change = rng.random((n, T)) < 0.05
    change[:, 0] = True
    idx = np.maximum.accumulate(np.where(change, np.arange(T)[None, :], 0), axis=1)
    choke = np.take_along_axis(choke_levels, idx, axis=1)
    glr = rng.uniform(0.3, 3.0, size=(n, 1)) * np.exp(np.cumsum(rng.normal(0, 0.005, size=(n, T)), axis=1))
    temp = rng.uniform(60.0, 180.0, size=(n, 1)) + rng.normal(0, 1.0, size=(n, T))
    wc = np.clip(rng.uniform(0.0, 0.6, size=(n, 1)) + np.cumsum(rng.normal(0, 0.002, size=(n, T)), axis=1), 0, 0.98)
    dsp = whp * rng.uniform(0.2, 0.5, size=(n, 1))
    return whp, choke, glr, temp, wc, dsp


def _flow(rng, whp, choke, glr, wc, noise=0.05):
    g = GilbertModel().flow_rate(whp, choke, glr) * (1.0 - 0.5 * wc)
    q = np.empty_like(g)
    q[:, 0] = g[:, 0]
    for k in range(1, g.shape[1]):
        q[:, k] = LAG * q[:, k - 1] + (1.0 - LAG) * g[:, k]
    return q * np.exp(rng.normal(0.0, noise, size=q.shape))


def well_log_table(n_wells: int = 8, steps: int = 500, seed: int = 0, n_fields: int = 3):
    """Columnar table (dict name -> np.ndarray) with TABLE_COLUMNS / TABLE_TYPES."""
    rng = np.random.default_rng(seed)
    whp, choke, glr, temp, wc, dsp = _series(rng, n_wells, steps)
    flow = _flow(rng, whp, choke, glr, wc)
    wells = np.array([f"W{i:03d}" for i in range(n_wells)])
    fields = np.array([f"F{i % n_fields}" for i in range(n_wells)])
    rep = lambda a: np.repeat(a, steps)  # noqa: E731
    return {
        "well": rep(wells),
        "field": rep(fields),
        "t": np.tile(np.arange(steps, dtype=np.int64), n_wells),
        "whp": whp.reshape(-1).astype(np.float32),
        "choke": choke.reshape(-1).astype(np.float32),
        "glr": glr.reshape(-1).astype(np.float32),
        "temp": temp.reshape(-1).astype(np.float32),
        "water_cut": wc.reshape(-1).astype(np.float32),
        "dsp": dsp.reshape(-1).astype(np.float32),
        "flow": flow.reshape(-1).astype(np.float32),
    }


def _feature_stack(whp, choke, glr, temp, wc, dsp, F, rng):
    base = [
        (whp - 1200.0) / 600.0,
        (choke - 38.0) / 15.0,
        (glr - 1.5) / 0.8,
        (temp - 120.0) / 35.0,
        (wc - 0.3) / 0.2,
        np.log(whp) - 7.0,
        np.log(choke) - 3.5,
        np.log(glr),
        (dsp - 400.0) / 250.0,
    ]
    feats = base[:F]
    n, T = whp.shape
    k = 0
    while len(feats) < F:  # nuisance channels: periodic + noise
        feats.append(np.sin(2 * np.pi * (np.arange(T)[None, :] / (8.0 + 3 * k)) + rng.uniform(0, 6.28, (n, 1)))
                     + 0.1 * rng.normal(size=(n, T)))
        k += 1
    return np.stack(feats, axis=-1).astype(np.float32)


def _target(q):
    return ((np.log(q) - 6.0) / 1.5).astype(np.float32)


def synth_lstm_batch(B: int, T: int, F: int, seed: int = 0, torch_out: bool = True):
    """(x [B, T, F], y [B]) — y is the standardised log-rate at the window's last step."""
    rng = np.random.default_rng(seed)
    whp, choke, glr, temp, wc, dsp = _series(rng, B, T)
    q = _flow(rng, whp, choke, glr, wc)
    x = _feature_stack(whp, choke, glr, temp, wc, dsp, F, rng)
    y = _target(q[:, -1])
    if torch_out:
        import torch

        return torch.from_numpy(x), torch.from_numpy(y)
    return x, y


def synth_tabular_batch(B: int, F: int, seed: int = 0, torch_out: bool = True):
    """(x [B, F], y [B]) single-timestep rows for the static / dynamic MLP."""
    rng = np.random.default_rng(seed)
    whp, choke, glr, temp, wc, dsp = _series(rng, B, 1)
    q = _flow(rng, whp, choke, glr, wc)
    x = _feature_stack(whp, choke, glr, temp, wc, dsp, F, rng)[:, 0, :]
    y = _target(q[:, 0])
    if torch_out:
        import torch

        return torch.from_numpy(x), torch.from_numpy(y)
    return x, y
