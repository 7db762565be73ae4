"""The .mdl weight file is a real Keras-0.x HDF5 file (cnn.py:122 ModelCheckpoint ->
Sequential.save_weights). No h5py here, so the writer is checked against
the HDF5 C library's own tools when the image has them (/opt/conda/bin/h5dump, h5repack):
h5dump must parse our file and print the same numbers, and our reader must load a file
the library itself wrote (h5repack output)."""
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from wellflow.utils import h5

TOOLS = [d for d in ("/opt/conda/bin", *os.environ.get("PATH", "").split(":")) if d]


def _tool(name):
    for d in TOOLS:
        p = os.path.join(d, name)
        if os.access(p, os.X_OK):
            return p
    return shutil.which(name)


def _keras_like_tree(seed=0):
    rng = np.random.default_rng(seed)
    root = h5.Group({"nb_layers": np.int64(3), "model": "lstm"})
    g = root.group("layer_0", {"nb_params": np.int64(12), "class": "LSTM"})
    for i in range(12):  # > 8 links: two symbol-table nodes under the group B-tree
        g.children[f"param_{i}"] = rng.standard_normal((5, 7) if i % 3 != 2 else (7,)).astype(np.float32)
    root.group("layer_1", {"nb_params": np.int64(0), "class": "Dropout"})
    d = root.group("layer_2", {"nb_params": np.int64(2), "class": "Dense"})
    d.children["param_0"] = rng.standard_normal((7, 1)).astype(np.float32)
    d.children["param_1"] = np.zeros((1,), np.float32)
    return root


def _same(a: h5.Group, b: h5.Group):
    assert set(a.attrs) == set(b.attrs)
    for k, v in a.attrs.items():
        w = b.attrs[k]
        if isinstance(v, str):
            v = v.encode()
        assert np.array_equal(np.asarray(v), np.asarray(w)), k
    assert sorted(a.children) == sorted(b.children)
    for k, v in a.children.items():
        if isinstance(v, h5.Group):
            _same(v, b.children[k])
        else:
            assert b.children[k].dtype == v.dtype and np.array_equal(b.children[k], v), k


def test_roundtrip_own_reader(tmp_path):
    root = _keras_like_tree()
    p = tmp_path / "w.h5"
    h5.write(str(p), root)
    assert h5.is_hdf5(str(p))
    _same(root, h5.read(str(p)))


def test_value_types_roundtrip():
    root = h5.Group({"f64": np.float64(1.5), "i32v": np.arange(3, dtype=np.int32), "s": "héllo"})
    for dt in ("float16", "float32", "float64", "int8", "int16", "int64", "uint8", "uint32"):
        root.children[dt] = (np.arange(24) % 7).astype(dt).reshape(2, 3, 4)
    root.children["scalar"] = np.float32(3.25)
    back = h5.loads(h5.dumps(root))
    assert back.attrs["s"].decode() == "héllo" and back.attrs["f64"] == 1.5
    for dt in ("float16", "float32", "float64", "int8", "int16", "int64", "uint8", "uint32"):
        assert back[dt].dtype == np.dtype(dt) and np.array_equal(back[dt], root[dt])
    assert back["scalar"].shape == () and back["scalar"] == np.float32(3.25)


@pytest.mark.skipif(_tool("h5dump") is None, reason="HDF5 command-line tools not in this image")
def test_hdf5_library_parses_our_file(tmp_path):
    root = _keras_like_tree(1)
    p = tmp_path / "w.h5"
    h5.write(str(p), root)
    out = subprocess.run([_tool("h5dump"), "-p", str(p)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert 'ATTRIBUTE "nb_layers"' in out.stdout and "H5T_STD_I64LE" in out.stdout
    assert out.stdout.count("DATASET") == 14 and "H5T_IEEE_F32LE" in out.stdout
    assert "CONTIGUOUS" in out.stdout
    # the library reads the same numbers
    dd = subprocess.run([_tool("h5dump"), "-m", "%.9g", "-d", "/layer_2/param_0", "-y", "-w", "0", str(p)],
                        capture_output=True, text=True, timeout=60)
    assert dd.returncode == 0, dd.stderr
    body = dd.stdout.split("DATA {", 1)[1].split("}", 1)[0]
    vals = np.array([float(t) for t in body.replace(",", " ").split()], np.float32)
    assert np.array_equal(vals, root["layer_2"]["param_0"].ravel())


@pytest.mark.skipif(_tool("h5repack") is None, reason="HDF5 command-line tools not in this image")
def test_reader_loads_a_file_the_hdf5_library_wrote(tmp_path):
    root = _keras_like_tree(2)
    src, dst = tmp_path / "a.h5", tmp_path / "b.h5"
    h5.write(str(src), root)
    r = subprocess.run([_tool("h5repack"), str(src), str(dst)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert dst.read_bytes() != src.read_bytes()  # the library's own layout, not ours
    _same(root, h5.read(str(dst)))


def test_mdl_is_keras_save_weights_layout(tmp_path):
    """What Keras 0.x load_weights reads: f.attrs['nb_layers'], f['layer_k'].attrs['nb_params'],
    f['layer_k']['param_n'] float32."""
    from wellflow.utils.checkpoint import load_mdl, save_mdl

    layers = [("Dense", [torch.randn(6, 4), torch.randn(4)]), ("Activation", []),
              ("Dense", [torch.randn(4, 1), torch.randn(1)])]
    p = tmp_path / "mlp.mdl"
    save_mdl(str(p), "mlp", layers, {"epoch": 3})
    f = h5.read(str(p))
    assert int(f.attrs["nb_layers"]) == 3
    for k, (_, params) in enumerate(layers):
        g = f[f"layer_{k}"]
        assert int(g.attrs["nb_params"]) == len(params)
        for n, t in enumerate(params):
            assert g[f"param_{n}"].dtype == np.float32 and np.array_equal(g[f"param_{n}"], t.numpy())
    name, back, extra = load_mdl(str(p))
    assert name == "mlp" and extra == {"epoch": 3} and [c for c, _ in back] == ["Dense", "Activation", "Dense"]


def test_round1_safetensors_mdl_still_loads(tmp_path):
    from safetensors.torch import save_file
    from wellflow.utils.checkpoint import load_mdl

    p = tmp_path / "old.mdl"
    save_file({"layer_0/param_0": torch.ones(2, 3), "layer_0/param_1": torch.zeros(3)}, str(p),
              metadata={"model": "mlp", "nb_layers": "1", "layer_0/nb_params": "2", "layer_0/class": "Dense"})
    name, layers, extra = load_mdl(str(p))
    assert name == "mlp" and layers[0][0] == "Dense" and layers[0][1][0].shape == (2, 3) and extra == {}
