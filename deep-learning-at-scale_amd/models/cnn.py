"""The reference's only implemented model: 1-D CNN regression (cnn.py:110-114).

Keras-0.x ``Sequential``: ``Convolution1D(1, 100, 13, activation="relu")`` ->
``Dropout(0.5)`` -> ``Flatten()`` -> ``Dense(3600, 12)`` on input (B, 48, 1): 100 filters of
width 13 (valid), 36 output steps, flatten in (step, filter) order, 12 linear outputs,
44,612 parameters. Loss ``mae_clip`` (cnn.py:29-32), optimizer Keras SGD
lr 1e-3 / momentum 0.99 / decay 1e-6 / Nesterov (cnn.py:117), batch 20 (cnn.py:128).

* :class:`CNN1DRegressor` — PyTorch fp32 reference (CPU oracle, channels-last input).
* :class:`NativeCNN` — MI355X engine. For the reference shape (one input channel, 48-step
  windows, width 13, 97-112 filters, <= 16 outputs, dropout 0 or 0.5) the step is three
  fused kernels (csrc/cnn_fused.hip): a forward that keeps the 36 x 112 activation of every
  window on chip (conv MFMA -> ReLU -> hashed dropout -> dense MFMA -> loss, writing only
  dOut), a backward that recomputes the activation and accumulates dWd / dWc in registers,
  and a reduce of the per-workgroup partials. Other shapes (the job path's multi-channel
  windows) run im2col -> conv-as-GEMM with a fused ReLU + dropout epilogue -> dense GEMM ->
  loss kernel -> split-K weight-gradient GEMMs (csrc/gemm.hip).
  Internally filters are padded 100 -> 112 and outputs 12 -> 16 (zero rows; multiples of 16
  for the MFMA tiles); the padding stays exactly zero.

Theano's conv is a true convolution (kernel flipped); the exported reference layout
(``to_reference``) therefore flips the taps, so a Keras-0.x consumer of the .mdl sees the
same function.
"""
from __future__ import annotations

import dataclasses
import math
import os

import torch
from torch import nn

from .base import note_slow_path


def _r8(x: int) -> int:
    return (x + 7) // 8 * 8


def _r16(x: int) -> int:
    return (x + 15) // 16 * 16


_M32 = 0xFFFFFFFF


def _lowbias32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 integer hash on int64 tensors holding uint32 values (csrc/cnn_fused.hip)."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def cnn_dropout_mask(seed: int, step: int, B: int, T: int, Fp: int, device="cpu") -> torch.Tensor:
    """Keep mask [B, T, Fp] (bool) of the fused CNN kernels' dropout at p = 0.5, bit for bit:
    bit 2*(f >> 4) + ((f & 3) >> 1) + 16*(f & 1) of lowbias32(((w*T + t)*4 + ((f >> 2) & 3)) ^
    smix) (the two bits of a packed bf16 pair 16 apart: csrc/cnn_fused.hip), smix =
    lowbias32(seed ^ lowbias32(step + 0x9E3779B9)); ``step`` is the device step counter the
    forward and backward of one training step read (NativeCNN.rng)."""
    seed_t = torch.tensor(seed & _M32, dtype=torch.int64)
    smix = _lowbias32(seed_t ^ _lowbias32(torch.tensor((step + 0x9E3779B9) & _M32, dtype=torch.int64)))
    w = torch.arange(B, dtype=torch.int64, device=device).view(B, 1, 1)
    t = torch.arange(T, dtype=torch.int64, device=device).view(1, T, 1)
    f = torch.arange(Fp, dtype=torch.int64, device=device).view(1, 1, Fp)
    idx = (((w * T + t) & _M32) * 4 + ((f >> 2) & 3)) & _M32
    h = _lowbias32(idx ^ smix.to(device))
    bit = 2 * (f >> 4) + ((f & 3) >> 1) + 16 * (f & 1)
    return ((h >> bit) & 1).bool()


class CNN1DRegressor(nn.Module):
    def __init__(self, input_len: int = 48, in_ch: int = 1, filters: int = 100, kernel: int = 13,
                 outputs: int = 12, dropout: float = 0.5):
        super().__init__()
        self.input_len, self.in_ch, self.filters = input_len, in_ch, filters
        self.kernel, self.outputs, self.p = kernel, outputs, dropout
        self.lout = input_len - kernel + 1
        self.conv = nn.Conv1d(in_ch, filters, kernel)
        self.drop = nn.Dropout(dropout)
        self.dense = nn.Linear(filters * self.lout, outputs)

    def forward(self, x):  # x [B, L, C] (Keras channels-last)
        if x.dim() == 2:
            x = x.unsqueeze(-1)
        h = torch.relu(self.conv(x.transpose(1, 2)))  # [B, F, Lout]
        h = self.drop(h.transpose(1, 2).reshape(x.shape[0], -1))  # (step, filter) order
        out = self.dense(h)
        return out.squeeze(-1) if self.outputs == 1 else out

    def init_keras(self, seed: int = 0):
        """Keras-0.x defaults: conv 'uniform' (+-0.05), dense glorot_uniform, zero biases."""
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            self.conv.weight.uniform_(-0.05, 0.05, generator=g)
            self.conv.bias.zero_()
            lim = math.sqrt(6.0 / (self.dense.in_features + self.dense.out_features))
            self.dense.weight.uniform_(-lim, lim, generator=g)
            self.dense.bias.zero_()
        return self

    @property
    def layout(self) -> "CnnLayout":
        return CnnLayout(self.input_len, self.in_ch, self.filters, self.kernel, self.outputs)

    def to_flat(self) -> torch.Tensor:
        lay = self.layout
        flat = torch.zeros(lay.numel)
        Wc, Wd, bd = lay.views(flat)
        with torch.no_grad():
            w = self.conv.weight.float().cpu()  # [F, C, k]
            # column index of tap (k, c) = k*C + c (im2col order); bias column = k*C
            Wc[: self.filters, : lay.taps] = w.permute(0, 2, 1).reshape(self.filters, -1)
            Wc[: self.filters, lay.taps] = self.conv.bias.float().cpu()
            d = self.dense.weight.float().cpu().view(self.outputs, self.lout, self.filters)
            Wd.view(lay.Op, self.lout, lay.Fp)[: self.outputs, :, : self.filters] = d
            bd[: self.outputs] = self.dense.bias.float().cpu()
        return flat

    def load_flat(self, flat: torch.Tensor) -> None:
        lay = self.layout
        Wc, Wd, bd = lay.views(flat.detach().float().cpu())
        with torch.no_grad():
            w = Wc[: self.filters, : lay.taps].reshape(self.filters, self.kernel, self.in_ch)
            self.conv.weight.copy_(w.permute(0, 2, 1))
            self.conv.bias.copy_(Wc[: self.filters, lay.taps])
            d = Wd.view(lay.Op, self.lout, lay.Fp)[: self.outputs, :, : self.filters]
            self.dense.weight.copy_(d.reshape(self.outputs, -1))
            self.dense.bias.copy_(bd[: self.outputs])


@dataclasses.dataclass(frozen=True)
class CnnLayout:
    input_len: int = 48
    in_ch: int = 1
    filters: int = 100
    kernel: int = 13
    outputs: int = 12

    @property
    def lout(self):
        return self.input_len - self.kernel + 1

    @property
    def taps(self):
        return self.kernel * self.in_ch

    @property
    def Kc(self):  # im2col width: taps + bias column, padded to 8
        return _r8(self.taps + 1)

    @property
    def Fp(self):  # 16-filter MFMA blocks
        return _r16(self.filters)

    @property
    def Op(self):  # one 16-row MFMA tile of outputs
        return _r16(self.outputs)

    @property
    def fused_dims(self) -> list:
        """[L, C, taps, T, Fp, Kc, O] of the fused kernels (csrc/kernels.h CnnDims)."""
        return [self.input_len, self.in_ch, self.taps, self.lout, self.Fp, self.Kc, self.outputs]

    @property
    def flat_width(self):
        return self.lout * self.Fp

    @property
    def numel(self):
        return self.Fp * self.Kc + self.Op * self.flat_width + self.Op

    def views(self, flat):
        a = self.Fp * self.Kc
        b = a + self.Op * self.flat_width
        return (flat[:a].view(self.Fp, self.Kc), flat[a:b].view(self.Op, self.flat_width),
                flat[b : b + self.Op])


def cnn_fast_path_reason(layout: "CnnLayout", dropout: float) -> str | None:
    """None when the fused CNN kernels cover this layout (a Python mirror of
    csrc/cnn_fused.hip cnn_fused_supported), else why not: the step then runs im2col + the
    generic split-K GEMMs (7 launches; NativeCNN announces it once: note_slow_path)."""
    L = layout
    if L.in_ch != 1:
        return f"{L.in_ch} input channels (the fused kernels take the reference's single-channel series)"
    if L.lout != 36 or L.Fp != 112:
        return f"{L.lout} output steps x {L.Fp} padded filters (fused: 36 x 112, the reference's 48-step window, 100 filters)"
    if L.taps > 15 or L.Kc != 16:
        return f"{L.taps} taps (fused: <= 15, one 16-wide K slot with the bias)"
    if not 1 <= L.outputs <= 16:
        return f"{L.outputs} outputs (fused: 1 .. 16)"
    if L.input_len % 4 != 0:
        return f"window length {L.input_len} not a multiple of 4"
    if dropout not in (0.0, 0.5):
        return f"dropout {dropout} (fused: 0 or 0.5)"
    return None


class NativeCNN:
    """HIP/MFMA engine for the reference CNN (any batch up to ``batch``).

    ``fused`` (default where the shape allows, see module doc): three kernel launches per
    training step with the activation on chip; else the im2col + GEMM path."""

    native = True

    def __init__(self, layout: CnnLayout = CnnLayout(), batch: int = 1024, device="cuda",
                 dropout: float = 0.5, loss: str = "mae_clip", clip: float = 6.0, seed: int = 0,
                 params: torch.Tensor | None = None, grads: torch.Tensor | None = None,
                 fused: bool | None = None):
        from ..ops.native import lib

        self._C = lib()
        self.lay, self.B, self.p = layout, batch, dropout
        self.loss_kind, self.clip, self.seed = loss, clip, seed
        dev = torch.device(device)
        self.device = dev
        n = layout.numel
        self.params = params if params is not None else torch.zeros(n, device=dev)
        self.grads = grads if grads is not None else torch.zeros(n, device=dev)
        self.loss_sum = torch.zeros(1, device=dev)
        # dropout step counter on the device: the mask differs every training step, eager or
        # replayed from a captured hipGraph (a host-side step would be baked into the graph)
        self.rng = torch.zeros(1, dtype=torch.int64, device=dev)
        L = layout
        ok = self._C.cnn_fused_ok(L.fused_dims, float(dropout))
        why = cnn_fast_path_reason(L, float(dropout))
        assert (why is None) == bool(ok), (why, ok)  # the Python mirror must agree with the kernels
        if fused is None:
            fused = ok and os.environ.get("WELLFLOW_CNN_FUSED", "1") != "0"
        if not fused:
            note_slow_path("CNN", "training step runs im2col + generic GEMMs",
                           why or "fused kernels disabled (WELLFLOW_CNN_FUSED=0)",
                           f"window {L.input_len}x{L.in_ch} filters {L.filters} k {L.kernel} out {L.outputs} B={batch}")
        if fused and not ok:
            raise ValueError(f"fused CNN kernels do not cover {L} with dropout {dropout}")
        self.fused = bool(fused)
        bf = torch.bfloat16
        if self.fused:
            nfr = L.lout * (L.Fp // 16) * 64 * 4
            self.WcA = torch.empty(L.Fp * L.Kc, dtype=bf, device=dev)
            self.WdF = torch.empty(nfr, dtype=bf, device=dev)
            self.WdB = torch.empty(nfr, dtype=bf, device=dev)
            rows = _r16(batch)
            self.dout = torch.zeros(rows * 16, device=dev)
            self.pred = torch.zeros(rows * 16, device=dev)
            wd, wc, f = self._C.cnn_part_sizes(batch, L.fused_dims)
            self.part_wd = torch.zeros(wd, device=dev)
            self.part_wc = torch.zeros(wc, device=dev)
            self.part_f = torch.zeros(f, device=dev)
        else:
            self.shadow = torch.empty(n, dtype=bf, device=dev)
            self.Xcol = torch.empty(batch * L.lout * L.Kc, dtype=bf, device=dev)
            self.Hc = torch.empty(batch * L.flat_width, dtype=bf, device=dev)
            self.dZc = torch.empty(batch * L.flat_width, dtype=bf, device=dev)
            self.pred = torch.empty(batch * L.Op, device=dev)
            self.ypad = torch.zeros(batch * L.Op, device=dev)
            self.dpred = torch.zeros(batch * L.Op, dtype=bf, device=dev)
        self.sync_weights()

    @property
    def seed32(self) -> int:
        return (self.seed * 1000003) & 0x7FFFFFFF

    # ------------------------------------------------------------------ small batches
    SMALL_MAX_B = 64  # csrc/cnn_small.hip: every worker holds the whole batch's activations

    def small_steps_reason(self, B: int, opt=None, X=None) -> str | None:
        """None when K training steps of batch ``B`` can run as ONE persistent launch
        (csrc/cnn_small.hip: forward, backward and the Keras SGD update; 25 workgroups of 4
        filters, one exchange per step); else why not."""
        if self.device.type != "cuda":
            return "not on a GPU"
        if not self.fused:
            return "layout not covered by the fused kernels"
        L = self.lay
        if L.input_len != 48 or L.kernel != 13 or L.in_ch != 1:
            return f"window {L.input_len}x{L.in_ch}, kernel {L.kernel} (needs the reference's 48 x 1, 13)"
        if not 4 <= B <= self.SMALL_MAX_B or B % 4:
            return f"batch {B} (needs 4 <= B <= {self.SMALL_MAX_B}, B % 4 == 0)"
        G = -(-L.filters // 4)  # workgroups of 4 filters; each sums <= 48 of the B x outputs
        if G > 28 or -(-B * L.outputs // G) > 48:
            return f"{L.filters} filters x batch {B} x {L.outputs} outputs (needs <= 112 filters, <= 48 outputs per 4 filters)"
        if opt is not None:
            from ..optim.flat import FlatSGD

            if not isinstance(opt, FlatSGD) or opt.params is not self.params or opt.step_dev is None:
                return "optimizer is not a device FlatSGD over this engine's parameters"
        if X is not None and not (torch.is_tensor(X) and X.dtype == torch.float32 and X.is_cuda):
            return "data not a resident fp32 tensor"
        return None

    def fused_steps(self, X: torch.Tensor, Y: torch.Tensor, B: int, K: int, opt, grad_scale: float,
                    rows: torch.Tensor | None = None, loss_into: torch.Tensor | None = None,
                    stamps: torch.Tensor | None = None) -> None:
        """K complete training steps (forward with the engine's dropout stream, backward, the
        Keras SGD update of ``opt``) in ONE launch. Step k reads windows ``rows[k B : (k + 1) B]``
        of ``X`` ([N][48] fp32) / ``Y`` ([N][outputs]), or windows k B .. when ``rows`` is None.
        ``loss_into`` += each step's loss sum. The gradient bucket is not written; the bf16
        operand images are refreshed after the launch. Equals K single steps of this path bit for
        bit (tests/test_small_gpu.py)."""
        why = self.small_steps_reason(B, opt, X)
        if why is not None:
            raise RuntimeError(f"NativeCNN.fused_steps: {why}")
        if getattr(self, "_small_scr", None) is None:
            self._small_scr = torch.zeros(self._C.cnn_small_scratch_floats(), device=self.device)
            self._small_sync = torch.zeros(4, dtype=torch.int32, device=self.device)
        kind = 0 if self.loss_kind == "mse" else 1
        ok = self._C.cnn_small_steps(X.reshape(-1), Y.reshape(-1).float(), rows, B, K, self.lay.fused_dims,
                                     float(self.p), kind, float(self.clip), float(grad_scale), self.seed32, self.rng,
                                     self.params, opt.vel, opt.step_dev, opt.lr, opt.decay, opt.momentum,
                                     bool(opt.nesterov), 1.0, loss_into, self._small_scr, self._small_sync,
                                     self.lay.filters, stamps)
        if not ok:
            raise RuntimeError("NativeCNN.fused_steps: the launcher refused the shape")
        opt.iterations += K
        self.sync_weights()  # the bf16 operand images of the regular kernels (evaluation)

    def check_device_errors(self) -> None:
        """Raise if a small-batch launch's hand-off timed out (sticky word; the buffer is reset)."""
        sync = getattr(self, "_small_sync", None)
        if sync is None:
            return
        if int(sync[2].item()):
            sync.zero_()
            raise RuntimeError("NativeCNN: a small-batch persistent launch timed out in a hand-off "
                               "(results of that launch are invalid)")

    def fused_sgd_ok(self, opt) -> bool:
        """Whether :meth:`fused_sgd` covers ``opt`` (train/step.py's sync_weights decision)."""
        return bool(self.fused)

    def fused_sgd(self, opt, grad_scale: float) -> bool:
        """The optimizer's update and this engine's operand images in ONE launch (optim/flat.py
        FlatSGD ``writeback``; csrc/cnn_fused.hip cnn_sgd_pack_kernel); False = not covered (the
        caller runs the plain update and sync_weights)."""
        if not self.fused_sgd_ok(opt):
            return False
        self._C.cnn_sgd_pack(self.params, self.grads, opt.vel, opt.step_dev, opt.lr, opt.decay, opt.momentum,
                             opt.nesterov, grad_scale, opt.zero_grads, self.lay.fused_dims, self.WcA, self.WdF,
                             self.WdB)
        return True

    def sync_weights(self):
        if self.fused:
            Wc, Wd, _ = self.lay.views(self.params)
            self._C.cnn_pack(Wc, Wd, self.lay.fused_dims, self.WcA, self.WdF, self.WdB)
        else:
            self._C.cast_bf16(self.params, self.shadow)

    def _x2d(self, x):
        L = self.lay
        B = x.shape[0]
        if x.dim() == 3:
            assert x.shape[1] == L.input_len and x.shape[2] == L.in_ch
        return x.reshape(B, L.input_len * L.in_ch).contiguous().float()

    # ------------------------------------------------------------------ unfused GEMM path
    def _fwd(self, x, B, drop_p, seed, seed_dev=None):
        from ..ops.native import gemm

        L = self.lay
        if x.dim() == 2:
            x = x.unsqueeze(-1)
        assert x.shape[1] == L.input_len and x.shape[2] == L.in_ch and B <= self.B
        self._C.im2col1d(x.contiguous().float(), B, L.input_len, L.in_ch, L.kernel, L.Kc, self.Xcol)
        Wc, Wd, _ = L.views(self.shadow)
        _, _, bd = L.views(self.params)
        gemm(self.Xcol, Wc, B * L.lout, L.Fp, L.Kc, outH=self.Hc, act=1, drop_p=drop_p, seed=seed,
             seed_dev=seed_dev)
        gemm(self.Hc, Wd, B, L.Op, L.flat_width, outF=self.pred, bias=bd)

    def forward(self, x):
        L = self.lay
        B = x.shape[0]
        assert B <= self.B
        if self.fused:
            _, _, bd = L.views(self.params)
            self._C.cnn_forward(self._x2d(x), B, L.fused_dims, float(self.p), self.WcA, self.WdF, bd, None, None,
                                self.pred, None, False, 0, self.clip, 1.0, self.seed32, None)
            out = self.pred[: B * 16].view(B, 16)[:, : L.outputs]
        else:
            self._fwd(x, B, 0.0, 0)
            out = self.pred[: B * L.Op].view(B, L.Op)[:, : L.outputs]
        return out.squeeze(-1) if L.outputs == 1 else out

    def forward_backward(self, x, y, grad_scale: float, zero_grads: bool = True, step: int = 0,
                         loss_into: torch.Tensor | None = None):
        """Gradient of grad_scale * sum of per-element losses into ``grads`` (models/base.py);
        returns the device loss sum (``loss_into`` when given: added straight into it)."""
        L = self.lay
        B = x.shape[0]
        assert B <= self.B
        if zero_grads:
            self.grads.zero_()
        gWc, gWd, gbd = L.views(self.grads)
        kind = 0 if self.loss_kind == "mse" else 1
        if self.fused:
            ls = loss_into if loss_into is not None else self.loss_sum
            if loss_into is None:
                self.loss_sum.zero_()
            _, _, bd = L.views(self.params)
            xf = self._x2d(x)
            dims, p = L.fused_dims, float(self.p)
            self._C.cnn_forward(xf, B, dims, p, self.WcA, self.WdF, bd, y.reshape(B, -1).contiguous().float(),
                                self.dout, None, self.part_f, True, kind, self.clip, float(grad_scale), self.seed32,
                                self.rng)
            self._C.cnn_backward(xf, B, dims, p, self.WcA, self.WdB, self.dout, self.seed32, self.rng,
                                 self.part_wd, self.part_wc)
            self._C.cnn_reduce(self.part_wd, self.part_wc, self.part_f, B, dims, gWc, gWd, gbd, ls, self.rng)
            return ls
        from ..ops.native import gemm

        self.loss_sum.zero_()
        self._fwd(x, B, self.p, self.seed32, self.rng)
        self.rng += 1
        yv = self.ypad[: B * L.Op].view(B, L.Op)
        yv[:, : L.outputs].copy_(y.view(B, -1))
        _, Wd, _ = L.views(self.shadow)
        self._C.loss(kind, self.pred, self.ypad, B, L.Op, self.clip, float(grad_scale),
                     self.loss_sum, self.dpred, None, gbd)
        # dWd = dpred^T Hc   (reduce over batch)
        ks = int(os.environ.get("WELLFLOW_CNN_KS1", "0")) or max(1, min(16, B // 256))
        gemm(self.dpred, self.Hc, L.Op, L.flat_width, B, a_mn=True, lda=L.Op, b_mn=True,
             ldb=L.flat_width, outF=gWd, atomic=True, ksplit=ks)
        # dHc = dpred Wd, masked by the stored post-dropout activation, x 1/(1-p)
        gemm(self.dpred, Wd, B, L.flat_width, L.Op, b_mn=True, ldb=L.flat_width, outH=self.dZc,
             mask=self.Hc, mask_scale=1.0 / (1.0 - self.p) if self.p > 0 else 1.0)
        # dWc = dZc^T Xcol   (reduce over batch x steps); K = B x steps is huge and M x N =
        # filters x taps tiny: split K deep (WELLFLOW_CNN_KS2 overrides)
        ks2 = int(os.environ.get("WELLFLOW_CNN_KS2", "0")) or max(1, min(512, (B * L.lout) // 4096))
        gemm(self.dZc, self.Xcol, L.Fp, L.Kc, B * L.lout, a_mn=True, lda=L.Fp, b_mn=True,
             ldb=L.Kc, outF=gWc, atomic=True, ksplit=ks2)
        if loss_into is not None:
            loss_into += self.loss_sum
        return self.loss_sum
