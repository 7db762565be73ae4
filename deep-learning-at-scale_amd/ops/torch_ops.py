"""torch.library custom ops over the HIP kernels, with autograd (SURVEY.md §1 design L6:
"ops/ torch.library custom-op bindings + autograd.Functions over kernels/").

The training engines (models/*.py Native*) drive the kernels imperatively for the fused,
graph-captured step. These ops expose the same kernels to plain PyTorch code, so an
``nn.Module`` built from them trains with ``loss.backward()`` and any ``torch.optim``
optimizer — the reference's "compile a model from layers and fit it" usage (cnn.py:110-118):

* ``wellflow::linear_act(x, W, b, act)``        y = act(x W^T + b), bf16 MFMA GEMM with the
  bias/ReLU/bf16 epilogue fused; backward: ReLU mask, dX GEMM, split-K dW GEMM (fp32 atomics),
  bias column sums.
* ``wellflow::lstm_regressor(x, flat, H, KX)``  seq-to-one LSTM regression (persistent
  forward over all timesteps + linear head); backward: persistent BPTT + the dW GEMM into the
  flat gradient of the models/lstm.py LstmLayout.
* ``wellflow::regression_loss(pred, y, kind, clip)``  sum of MSE / clipped-MAE (cnn.py:29-32)
  per-element losses and its gradient from the same kernel.

Inputs are cast to bf16 for the MFMA operands; parameters and gradients stay fp32. Every op
has a fake (meta) implementation, so it traces under torch.compile / FakeTensor. The ops run
on the GPU only (the CPU oracle is plain PyTorch: models/*.py reference modules).
"""
from __future__ import annotations

import torch
from torch import nn

from ..models.lstm import PSTAT_WORDS, decode_pstat, persistent_sync_buffer, pstat_error
from .native import gemm, lib

_BF = torch.bfloat16


def _r8(n: int) -> int:
    return (n + 7) // 8 * 8


# ----------------------------------------------------------------------------- linear_act
@torch.library.custom_op("wellflow::linear_act", mutates_args=())
def linear_act(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor, act: int) -> torch.Tensor:
    """x [M, K], W [N, K] (torch Linear layout), b [N] -> bf16 [M, N]; act 0 = linear, 1 = ReLU."""
    M, K = x.shape
    N = W.shape[0]
    Kp = _r8(K)
    xb = torch.zeros(M, Kp, dtype=_BF, device=x.device) if Kp != K else None
    if xb is not None:
        xb[:, :K] = x
        wb = torch.zeros(N, Kp, dtype=_BF, device=x.device)
        wb[:, :K] = W
    else:
        xb, wb = x.to(_BF).contiguous(), W.to(_BF).contiguous()
    y = torch.empty(M, N, dtype=_BF, device=x.device)
    gemm(xb, wb, M, N, Kp, outH=y, bias=b.float().contiguous(), act=int(act))
    return y


@linear_act.register_fake
def _(x, W, b, act):
    return x.new_empty((x.shape[0], W.shape[0]), dtype=_BF)


def _linear_act_setup(ctx, inputs, output):
    x, W, b, act = inputs
    ctx.save_for_backward(x, W, output)
    ctx.act = act


def _linear_act_bwd(ctx, dy):
    x, W, y = ctx.saved_tensors
    M, K = x.shape
    N = W.shape[0]
    dz = dy.to(_BF)
    if ctx.act == 1:
        dz = dz * (y > 0)
    dz = dz.contiguous()
    Np, Kp = _r8(N), _r8(K)
    # dX = dZ W  (A = dZ [M][N] K-contiguous, B(k, n) = W[n][k]: MN-contiguous, ld = K)
    dx = None
    if ctx.needs_input_grad[0]:
        dzp = dz if Np == N else torch.nn.functional.pad(dz, (0, Np - N))
        wt = W.to(_BF)
        if Np != N or Kp != K:
            wt = torch.nn.functional.pad(wt, (0, Kp - K, 0, Np - N))
        dxp = torch.empty(M, Kp, dtype=torch.float32, device=x.device)
        gemm(dzp.contiguous(), wt.contiguous(), M, Kp, Np, b_mn=True, ldb=Kp, outF=dxp)
        dx = dxp[:, :K].to(x.dtype)
    # dW = dZ^T X over the batch (split-K, fp32 atomics): A(n, m) = dZ[m][n], B(k, m) = X[m][k]
    dW = None
    if ctx.needs_input_grad[1]:
        xb = x.to(_BF)
        dzp = dz
        if Np != N or Kp != K:
            xb = torch.nn.functional.pad(xb, (0, Kp - K))
            dzp = torch.nn.functional.pad(dz, (0, Np - N))
        dWp = torch.zeros(Np, Kp, dtype=torch.float32, device=x.device)
        ks = max(1, min(32, M // 256))
        gemm(dzp.contiguous(), xb.contiguous(), Np, Kp, M, a_mn=True, lda=Np, b_mn=True, ldb=Kp,
             outF=dWp, atomic=True, ksplit=ks)
        dW = dWp[:N, :K].to(W.dtype)
    db = dz.float().sum(0).to(ctx.saved_tensors[1].dtype) if ctx.needs_input_grad[2] else None
    return dx, dW, db, None


linear_act.register_autograd(_linear_act_bwd, setup_context=_linear_act_setup)


# ----------------------------------------------------------------------------- regression_loss
@torch.library.custom_op("wellflow::regression_loss_fwd", mutates_args=())
def _loss_fwd(pred: torch.Tensor, y: torch.Tensor, kind: int, clip: float) -> tuple[torch.Tensor, torch.Tensor]:
    """-> (sum of per-element losses [1], d sum / d pred [same shape as pred], fp32)."""
    p = pred.float().contiguous().view(-1)
    t = y.float().contiguous().view(-1)
    n = p.numel()
    ls = torch.zeros(1, device=p.device)
    d = torch.empty(n, device=p.device)
    lib().loss(int(kind), p, t, n, 1, float(clip), 1.0, ls, None, d, None)
    return ls, d.view(pred.shape)


@_loss_fwd.register_fake
def _(pred, y, kind, clip):
    return pred.new_empty((1,), dtype=torch.float32), pred.new_empty(pred.shape, dtype=torch.float32)


def regression_loss(pred: torch.Tensor, y: torch.Tensor, kind: str = "mse", clip: float = 6.0) -> torch.Tensor:
    """Sum over elements of (pred - y)^2 ("mse") or clip(|y - pred|, 0, clip) ("mae_clip")."""
    return _RegressionLoss.apply(pred, y, {"mse": 0, "mae_clip": 1}[kind], float(clip))


class _RegressionLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, y, kind, clip):
        ls, d = torch.ops.wellflow.regression_loss_fwd(pred, y, kind, clip)
        ctx.save_for_backward(d)
        return ls[0]

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return (d * g).to(d.dtype), None, None, None


# ----------------------------------------------------------------------------- lstm_regressor
def _lstm_dims(B, T, F, KX, H):
    return (B, T, F, KX, H)


@torch.library.custom_op("wellflow::lstm_regressor_fwd", mutates_args=())
def _lstm_fwd(x: torch.Tensor, flat: torch.Tensor, H: int, KX: int) -> tuple[torch.Tensor, torch.Tensor,
                                                                            torch.Tensor, torch.Tensor,
                                                                            torch.Tensor]:
    """-> (pred [B], XH, Cst, S, Wpack) — the saved state of the persistent forward."""
    from ..models.lstm import LstmLayout

    B, T, F = x.shape
    lay = LstmLayout(F, H)
    assert lay.KX == KX
    C = lib()
    dev = x.device
    Bp = (B + 15) // 16 * 16
    XH = torch.zeros((T + 1) * B * lay.KA, dtype=_BF, device=dev)
    Cst = torch.zeros((T + 1) * Bp * H, dtype=torch.bfloat16, device=dev)  # bf16 c history
    S = torch.empty(T * Bp * lay.G, dtype=_BF, device=dev)
    Wp = torch.empty(lay.G * lay.KA + H * lay.G, dtype=_BF, device=dev)  # [Wp | WhhT]
    W, w_out, b_out = lay.views(flat)
    C.lstm_pack_weights(W.contiguous(), Wp[: lay.G * lay.KA], Wp[lay.G * lay.KA:], H, KX)
    dims = _lstm_dims(B, T, F, KX, H)
    C.lstm_pack_x(x.float().contiguous(), XH, *dims, True)
    sync = persistent_sync_buffer(B, 32, dev)
    if not C.lstm_forward_persistent(XH, Wp[: lay.G * lay.KA], Cst, S, sync, *dims):
        C.lstm_forward(XH, Wp[: lay.G * lay.KA], Cst, S, torch.empty(Bp * H, device=dev), *dims, 6)
    pred = torch.empty(B, device=dev)
    base = T * B * lay.KA
    hT = XH[base + KX: base + KX + (B - 1) * lay.KA + H]
    C.head_fwd(hT, lay.KA, B, H, w_out.contiguous(), b_out.contiguous(), None, pred, None, None, 0.0)
    if pstat_error(decode_pstat(sync[-PSTAT_WORDS:].tolist())):
        raise RuntimeError("wellflow::lstm_regressor: persistent forward left work undone "
                           f"{decode_pstat(sync[-PSTAT_WORDS:].tolist())}")
    return pred, XH, Cst, S, Wp


@_lstm_fwd.register_fake
def _(x, flat, H, KX):
    from ..models.lstm import LstmLayout

    B, T, F = x.shape
    lay = LstmLayout(F, H)
    Bp = (B + 15) // 16 * 16
    return (x.new_empty((B,), dtype=torch.float32), x.new_empty(((T + 1) * B * lay.KA,), dtype=_BF),
            x.new_empty(((T + 1) * Bp * H,), dtype=torch.float32), x.new_empty((T * Bp * lay.G,), dtype=_BF),
            x.new_empty((lay.G * lay.KA + H * lay.G,), dtype=_BF))


@torch.library.custom_op("wellflow::lstm_regressor_bwd", mutates_args=())
def _lstm_bwd(dpred: torch.Tensor, XH: torch.Tensor, Cst: torch.Tensor, S: torch.Tensor, Wp: torch.Tensor,
              flat: torch.Tensor, B: int, T: int, F: int, H: int, KX: int) -> torch.Tensor:
    """-> d flat (fp32, LstmLayout)."""
    from ..models.lstm import LstmLayout

    lay = LstmLayout(F, H)
    C = lib()
    dev = flat.device
    g = torch.zeros(lay.numel, device=dev)
    gW, gw_out, gb_out = lay.views(g)
    _, w_out, _ = lay.views(flat)
    dims = _lstm_dims(B, T, F, KX, H)
    base = T * B * lay.KA
    hT = XH[base + KX: base + KX + (B - 1) * lay.KA + H]
    dy = dpred.float().contiguous()
    C.head_bwd_w(hT, lay.KA, B, H, dy, gw_out, gb_out)
    Bp = (B + 15) // 16 * 16
    DG = torch.empty(T * B * lay.G, dtype=_BF, device=dev)
    dcarry = torch.empty(Bp * H, device=dev)
    sync = persistent_sync_buffer(B, 64, dev)
    ksplit = max(1, min(32, T * B // 16384))
    C.lstm_backward_dw(Wp[lay.G * lay.KA:], XH, Cst, S, DG, dcarry, dy, w_out.contiguous(), gW, *dims, 8, 0,
                       ksplit, sync, None)
    if pstat_error(decode_pstat(sync[-PSTAT_WORDS:].tolist())):
        raise RuntimeError("wellflow::lstm_regressor: persistent backward left work undone "
                           f"{decode_pstat(sync[-PSTAT_WORDS:].tolist())}")
    return g


@_lstm_bwd.register_fake
def _(dpred, XH, Cst, S, Wp, flat, B, T, F, H, KX):
    return flat.new_empty(flat.shape, dtype=torch.float32)


class _LSTMRegressorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, flat, H, KX):
        if x.requires_grad:
            raise NotImplementedError("wellflow::lstm_regressor does not produce input gradients "
                                      "(the features are data); detach x")
        pred, XH, Cst, S, Wp = torch.ops.wellflow.lstm_regressor_fwd(x, flat, H, KX)
        ctx.save_for_backward(XH, Cst, S, Wp, flat)
        ctx.dims = (x.shape[0], x.shape[1], x.shape[2], H, KX)
        return pred

    @staticmethod
    def backward(ctx, dpred):
        XH, Cst, S, Wp, flat = ctx.saved_tensors
        B, T, F, H, KX = ctx.dims
        return None, torch.ops.wellflow.lstm_regressor_bwd(dpred, XH, Cst, S, Wp, flat, B, T, F, H, KX), None, None


def lstm_regressor(x: torch.Tensor, flat: torch.Tensor, hidden: int) -> torch.Tensor:
    from ..models.lstm import LstmLayout

    return _LSTMRegressorFn.apply(x, flat, int(hidden), LstmLayout(x.shape[-1], hidden).KX)


# ----------------------------------------------------------------------------- modules
class NativeLinear(nn.Module):
    """``nn.Linear`` (+ optional ReLU) on the MFMA GEMM op; output bf16."""

    def __init__(self, in_features: int, out_features: int, relu: bool = False):
        super().__init__()
        ref = nn.Linear(in_features, out_features)
        self.weight = nn.Parameter(ref.weight.detach().clone())
        self.bias = nn.Parameter(ref.bias.detach().clone())
        self.relu = relu

    def forward(self, x):
        return torch.ops.wellflow.linear_act(x, self.weight, self.bias, 1 if self.relu else 0)


class NativeMLPModule(nn.Module):
    """F -> hidden... -> 1 regression MLP from NativeLinear layers (head in fp32 torch)."""

    def __init__(self, n_features: int, hidden=(256, 256)):
        super().__init__()
        layers, prev = [], n_features
        for h in hidden:
            layers.append(NativeLinear(prev, h, relu=True))
            prev = h
        self.body = nn.ModuleList(layers)
        self.head = nn.Linear(prev, 1)

    def forward(self, x):
        for layer in self.body:
            x = layer(x)
        return self.head(x.float()).squeeze(-1)


class NativeLSTMModule(nn.Module):
    """Seq-to-one LSTM regressor whose parameters are ONE flat fp32 tensor (LstmLayout)."""

    def __init__(self, n_features: int, hidden: int = 512, seed: int = 0):
        super().__init__()
        from ..models.lstm import init_lstm_flat

        self.hidden = hidden
        self.flat = nn.Parameter(init_lstm_flat(n_features, hidden, seed=seed))

    def forward(self, x):
        return lstm_regressor(x, self.flat, self.hidden)
