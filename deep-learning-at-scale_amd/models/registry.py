"""Model registry: name -> (fp32 reference module, native MI355X engine, Keras-0.x export).

Names follow the reference's taxonomy (Readme.md:11-21; MDL_NAME, cnn.py:39): ``cnn``
(implemented in the reference), ``mlp`` (ANN static), ``mlp_online`` (ANN dynamic),
``lstm`` and ``gilbert`` (physical, CPU only).
"""
from __future__ import annotations

import torch

from .base import TorchEngine
from .cnn import CNN1DRegressor, CnnLayout, NativeCNN
from .lstm import LSTMRegressor, LstmLayout, NativeLSTM
from .mlp import MLPRegressor, MlpLayout, NativeMLP

LEARNED = ("cnn", "mlp", "mlp_online", "lstm")


def build_reference(name: str, cfg, n_features: int, n_outputs: int = 1, seed: int = 0):
    torch.manual_seed(seed)
    if name in ("mlp", "mlp_online"):
        return MLPRegressor(n_features, tuple(cfg.mlp_hidden))
    if name == "lstm":
        return LSTMRegressor(n_features, cfg.hidden)
    if name == "cnn":
        return CNN1DRegressor(cfg.cnn_input_len, n_features, cfg.cnn_filters, cfg.cnn_kernel,
                              n_outputs, cfg.dropout).init_keras(seed)
    raise ValueError(f"no learned model named {name!r}")


def build_engine(name: str, cfg, n_features: int, n_outputs: int, batch: int, device,
                 native: bool, seed: int = 0):
    """Engine whose flat params start from the reference module's init (same seed)."""
    ref = build_reference(name, cfg, n_features, n_outputs, seed)
    if not native:
        return TorchEngine(ref, loss=cfg.loss, clip=cfg.clip, device=device), ref
    flat = ref.to_flat().to(device)
    if name in ("mlp", "mlp_online"):
        eng = NativeMLP(n_features, tuple(cfg.mlp_hidden), batch, device, loss=cfg.loss, clip=cfg.clip)
    elif name == "lstm":
        eng = NativeLSTM(n_features, cfg.hidden, cfg.seq_len, batch, device, loss=cfg.loss, clip=cfg.clip)
    elif name == "cnn":
        lay = CnnLayout(cfg.cnn_input_len, n_features, cfg.cnn_filters, cfg.cnn_kernel, n_outputs)
        eng = NativeCNN(lay, batch, device, dropout=cfg.dropout, loss=cfg.loss, clip=cfg.clip, seed=seed)
    else:
        raise ValueError(name)
    eng.params.copy_(flat)
    eng.sync_weights()
    return eng, ref


def engine_to_reference(eng, ref):
    """Copy the engine's current weights into the reference module (CPU)."""
    if getattr(eng, "native", False):
        ref.load_flat(eng.params.detach().cpu())
        return ref
    return eng.module


def reference_to_engine(ref, eng) -> None:
    if getattr(eng, "native", False):
        eng.params.copy_(ref.to_flat().to(eng.params.device))
        eng.sync_weights()
    else:
        eng.params.copy_(torch.nn.utils.parameters_to_vector(ref.parameters()).to(eng.params.device))


# ------------------------------------------------------------------ Keras-0.x layout
def keras_layers(name: str, ref) -> list:
    """Weights in Keras-0.x order/shapes: Dense W is (in, out); Conv W is
    (nb_filter, input_dim, filter_length, 1) with the taps flipped (Theano true
    convolution); LSTM params are [W_i, U_i, b_i, W_c, U_c, b_c, W_f, U_f, b_f, W_o, U_o, b_o]."""
    if name in ("mlp", "mlp_online"):
        out = []
        for lin in ref.linears():
            out.append(("Dense", [lin.weight.t(), lin.bias]))
            out.append(("Activation", []))
        out.append(("Dense", [ref.head.weight.t(), ref.head.bias]))
        return out
    if name == "cnn":
        w = ref.conv.weight.flip(-1).unsqueeze(-1)  # (F, C, k, 1)
        return [("Convolution1D", [w, ref.conv.bias]), ("Dropout", []), ("Flatten", []),
                ("Dense", [ref.dense.weight.t(), ref.dense.bias])]
    if name == "lstm":
        H = ref.hidden
        Wih, Whh = ref.lstm.weight_ih_l0, ref.lstm.weight_hh_l0
        b = ref.lstm.bias_ih_l0 + ref.lstm.bias_hh_l0
        sl = lambda g: slice(g * H, (g + 1) * H)  # noqa: E731  torch gate order i, f, g, o
        params = []
        for g in (0, 2, 1, 3):  # keras order i, c(=g), f, o
            params += [Wih[sl(g)].t(), Whh[sl(g)].t(), b[sl(g)]]
        return [("LSTM", params), ("Dense", [ref.head.weight.t(), ref.head.bias])]
    raise ValueError(name)


def load_keras_layers(name: str, ref, layers: list) -> None:
    with torch.no_grad():
        if name in ("mlp", "mlp_online"):
            dense = [p for cls, p in layers if cls == "Dense"]
            for lin, (W, b) in zip(ref.linears() + [ref.head], dense):
                lin.weight.copy_(W.t())
                lin.bias.copy_(b.view_as(lin.bias))
        elif name == "cnn":
            (W, b), (Wd, bd) = layers[0][1], layers[3][1]
            ref.conv.weight.copy_(W.squeeze(-1).flip(-1))
            ref.conv.bias.copy_(b)
            ref.dense.weight.copy_(Wd.t())
            ref.dense.bias.copy_(bd)
        elif name == "lstm":
            p = layers[0][1]
            H = ref.hidden
            for j, g in enumerate((0, 2, 1, 3)):
                ref.lstm.weight_ih_l0[g * H:(g + 1) * H].copy_(p[3 * j].t())
                ref.lstm.weight_hh_l0[g * H:(g + 1) * H].copy_(p[3 * j + 1].t())
                ref.lstm.bias_ih_l0[g * H:(g + 1) * H].copy_(p[3 * j + 2])
            ref.lstm.bias_hh_l0.zero_()
            W, b = layers[1][1]
            ref.head.weight.copy_(W.t())
            ref.head.bias.copy_(b.view_as(ref.head.bias))
        else:
            raise ValueError(name)


__all__ = ["LEARNED", "build_reference", "build_engine", "keras_layers", "load_keras_layers",
           "engine_to_reference", "reference_to_engine", "CnnLayout", "LstmLayout", "MlpLayout"]
