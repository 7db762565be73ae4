"""Saved-model and training-state formats.

``.mdl`` — best-model weights (cnn.py:122 ``ModelCheckpoint(storagePath + "models/%s.mdl",
save_best_only=True)``). Keras-0.x wrote an HDF5 file with attribute ``nb_layers`` and one
group ``layer_{k}`` per layer holding ``param_{n}`` datasets. h5py is not
available here, so the same *layout* is written as a safetensors file: tensor names
``layer_{k}/param_{n}`` in Keras-0.x shapes and order, metadata ``nb_layers``,
``layer_{k}/nb_params``, ``layer_{k}/class`` plus ``model`` and ``format``. Path, name and
best-only semantics are unchanged; only the container differs (documented in README).

``.ckpt`` — full training state for resume (the reference had none: no ``load_weights``
anywhere): flat fp32 parameters, optimizer state, epoch / step counters, early-stopping
state, feature-pipeline state and RNG. Written with ``torch.save`` of tensors, numbers,
strings, lists and dicts only, so it loads with ``torch.load(weights_only=True)``.

Writes are atomic (tmp file + rename) and done by rank 0 only (call site C4 adds the
barrier).
"""
from __future__ import annotations

import json
import os

import torch
from safetensors.torch import load_file, save_file
from safetensors import safe_open

MDL_FORMAT = "wellflow-mdl-1 (keras-0.x layer_k/param_n layout in safetensors)"


def save_mdl(path: str, model: str, layers: list, extra: dict | None = None) -> None:
    """``layers``: list of (class_name, [param tensors]) in Keras-0.x order."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tensors, meta = {}, {"model": model, "format": MDL_FORMAT, "nb_layers": str(len(layers))}
    for k, (cls, params) in enumerate(layers):
        meta[f"layer_{k}/class"] = cls
        meta[f"layer_{k}/nb_params"] = str(len(params))
        for n, p in enumerate(params):
            tensors[f"layer_{k}/param_{n}"] = p.detach().float().cpu().contiguous()
    if extra:
        meta["extra"] = json.dumps(extra)
    tmp = path + ".tmp"
    save_file(tensors, tmp, metadata=meta)
    os.replace(tmp, path)


def load_mdl(path: str):
    """-> (model name, [(class, [params])], extra dict)."""
    with safe_open(path, framework="pt") as f:
        meta = f.metadata() or {}
    tensors = load_file(path)
    n = int(meta.get("nb_layers", "0"))
    layers = []
    for k in range(n):
        cnt = int(meta.get(f"layer_{k}/nb_params", "0"))
        layers.append((meta.get(f"layer_{k}/class", ""), [tensors[f"layer_{k}/param_{i}"] for i in range(cnt)]))
    extra = json.loads(meta["extra"]) if "extra" in meta else {}
    return meta.get("model", ""), layers, extra


def save_state(path: str, state: dict) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_state(path: str) -> dict:
    return torch.load(path, map_location="cpu", weights_only=True)
