"""Saved-model and training-state formats.

``.mdl`` — best-model weights (cnn.py:122 ``ModelCheckpoint(storagePath + "models/%s.mdl",
save_best_only=True)``). Keras-0.x ``save_weights`` wrote an HDF5 file with attribute
``nb_layers`` and one group ``layer_{k}`` per layer holding attribute ``nb_params`` and
float32 datasets ``param_{n}``. That exact file is written here by the
pure-Python HDF5 writer in :mod:`.h5` (h5py is not installed), so a Keras-0.x
``model.load_weights(path)`` reads it; extra attributes (``model``, ``format``, ``extra``,
``layer_{k}/class``) are ignored by Keras. Round-1 files (safetensors with the same
``layer_{k}/param_{n}`` names) still load.

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
import numpy as np
from safetensors.torch import load_file
from safetensors import safe_open

from . import h5

MDL_FORMAT = "wellflow-mdl-2 (keras-0.x save_weights HDF5)"


def save_mdl(path: str, model: str, layers: list, extra: dict | None = None) -> None:
    """``layers``: list of (class_name, [param tensors]) in Keras-0.x order."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    root = h5.Group({"nb_layers": np.int64(len(layers)), "model": model, "format": MDL_FORMAT})
    if extra:
        root.attrs["extra"] = json.dumps(extra)
    for k, (cls, params) in enumerate(layers):
        g = root.group(f"layer_{k}", {"nb_params": np.int64(len(params)), "class": cls})
        for n, p in enumerate(params):
            g.children[f"param_{n}"] = p.detach().float().cpu().contiguous().numpy()
    tmp = path + ".tmp"
    h5.write(tmp, root)
    os.replace(tmp, path)


def _str(v) -> str:
    return v.decode("utf-8") if isinstance(v, (bytes, np.bytes_)) else str(v)


def load_mdl(path: str):
    """-> (model name, [(class, [params])], extra dict). Reads the HDF5 weight file (ours
    or one Keras 0.x wrote) and round-1 safetensors files."""
    if not h5.is_hdf5(path):
        return _load_mdl_safetensors(path)
    root = h5.read(path)
    layers = []
    for k in range(int(root.attrs["nb_layers"])):
        g = root[f"layer_{k}"]
        params = [torch.from_numpy(np.asarray(g[f"param_{i}"], np.float32)) for i in range(int(g.attrs["nb_params"]))]
        layers.append((_str(g.attrs.get("class", "")), params))
    extra = json.loads(_str(root.attrs["extra"])) if "extra" in root.attrs else {}
    return _str(root.attrs.get("model", "")), layers, extra


def _load_mdl_safetensors(path: str):
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
