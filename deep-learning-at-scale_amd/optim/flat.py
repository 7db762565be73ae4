"""Optimizers over ONE flat fp32 master buffer.

All parameters of a model are views into a single contiguous fp32 tensor and all
gradients into a second one, so an update is one kernel launch (``adam`` / ``sgd`` in
csrc/elementwise.hip) and the data-parallel reduction is one collective on one bucket.
On CPU tensors the same math runs in PyTorch (this is the fp32 oracle path used by the
CPU tests and the parity report — never a silent stand-in for a GPU op).
"""
from __future__ import annotations

import torch


class FlatAdam:
    """Adam / AdamW (decoupled weight decay) with PyTorch's bias-correction semantics."""

    def __init__(self, params: torch.Tensor, grads: torch.Tensor, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 shadow: torch.Tensor | None = None, zero_grads: bool = False, shadow_t=None,
                 writeback=None):
        """GPU fusions: ``shadow`` (bf16, same numel) receives the updated weights in the same
        launch (an engine whose compute copy is a plain cast, e.g. NativeMLP.shadow);
        ``shadow_t`` = (bf16 tensor, offset, rows, cols) receives one [rows][cols] block
        transposed in the same launch (NativeMLP.shadow_t: W2^T of the 128-row step kernel);
        ``zero_grads`` clears the gradient bucket after the update (the next
        forward_backward then runs with zero_grads=False); ``writeback``: an engine whose
        ``fused_adam(opt, grad_scale)`` runs this update AND refreshes its compute copies in one
        launch (NativeLSTM: Wp / WhhT), so no sync_weights launch follows (train/step.py)."""
        assert params.dtype == torch.float32 and params.shape == grads.shape
        self.params, self.grads = params, grads
        self.shadow, self.zero_grads = shadow, zero_grads
        self.shadow_t = shadow_t
        self.writeback = writeback
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.t = 0
        # device-side step counter: the GPU update is graph-capturable (bias corrections
        # are computed in-kernel from it, never baked in as launch constants)
        self.step_dev = torch.zeros(4, device=params.device) if params.is_cuda else None

    def step(self, grad_scale: float = 1.0) -> None:
        self.t += 1
        b1, b2 = self.betas
        if self.params.is_cuda:
            from ..ops.native import lib

            wb = self.writeback
            if wb is not None and wb.params is self.params and wb.fused_adam(self, grad_scale):
                return
            st = self.shadow_t or (None, 0, 0, 0)
            lib().adam_dev(self.params, self.grads, self.m, self.v, self.step_dev, self.lr, b1, b2,
                           self.eps, self.weight_decay, grad_scale, self.shadow, self.zero_grads, *st)
            return
        bc1, bc2 = 1.0 - b1**self.t, 1.0 - b2**self.t
        g = self.grads * grad_scale
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        upd = (self.m / bc1) / ((self.v / bc2).sqrt() + self.eps)
        if self.weight_decay:
            upd = upd + self.weight_decay * self.params
        self.params.sub_(self.lr * upd)
        if self.shadow is not None:
            self.shadow.copy_(self.params)
        if self.shadow_t is not None:
            t, off, r, c = self.shadow_t
            t.view(c, r).copy_(self.params[off : off + r * c].view(r, c).t())
        if self.zero_grads:
            self.grads.zero_()

    @property
    def steps_taken(self) -> int:
        """Updates applied so far. On the GPU the device counter is the truth: hipGraph
        replays (train/step.py) advance it without calling :meth:`step` on the host."""
        if self.step_dev is not None:
            return int(self.step_dev[0].item())
        return self.t

    def state_dict(self) -> dict:
        self.t = self.steps_taken
        return {"kind": "adam", "t": self.t, "m": self.m.detach().cpu(), "v": self.v.detach().cpu(),
                "lr": self.lr, "betas": list(self.betas), "eps": self.eps,
                "weight_decay": self.weight_decay}

    def load_state_dict(self, sd: dict) -> None:
        self.t = int(sd["t"])
        if self.step_dev is not None:
            self.step_dev.zero_()  # [1] is the kernel's completion ticket
            self.step_dev[0] = float(self.t)
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.lr, self.betas, self.eps = sd["lr"], tuple(sd["betas"]), sd["eps"]
        self.weight_decay = sd["weight_decay"]


class FlatSGD:
    """Keras-0.x SGD (cnn.py:117: lr=0.001, momentum=0.99, decay=1e-6, nesterov=True).

    lr_t = lr / (1 + decay * iterations); v = mu*v - lr_t*g;
    p += mu*v - lr_t*g (Nesterov) else p += v.
    """

    def __init__(self, params: torch.Tensor, grads: torch.Tensor, lr: float = 0.001,
                 momentum: float = 0.99, decay: float = 1e-6, nesterov: bool = True,
                 zero_grads: bool = False, writeback=None):
        """``writeback``: an engine whose ``fused_sgd(opt, grad_scale)`` runs this update AND
        refreshes its compute copies in one launch (NativeCNN: the bf16 operand images), so no
        separate sync_weights launch follows (train/step.py StepRunner)."""
        self.params, self.grads = params, grads
        self.writeback = writeback
        self.lr, self.momentum, self.decay, self.nesterov = lr, momentum, decay, nesterov
        self.zero_grads = zero_grads
        self.vel = torch.zeros_like(params)
        self.iterations = 0
        # device iteration counter ([1] = completion ticket): lr_t is computed in-kernel, so a
        # hipGraph-captured update decays the learning rate on every replay
        self.step_dev = torch.zeros(4, device=params.device) if params.is_cuda else None

    def step(self, grad_scale: float = 1.0) -> None:
        if self.params.is_cuda:
            from ..ops.native import lib

            self.iterations += 1
            wb = self.writeback
            if wb is not None and wb.params is self.params and wb.fused_sgd(self, grad_scale):
                return
            lib().sgd_dev(self.params, self.grads, self.vel, self.step_dev, self.lr, self.decay, self.momentum,
                          self.nesterov, grad_scale, self.zero_grads)
            return
        lr_t = self.lr / (1.0 + self.decay * self.iterations)
        self.iterations += 1
        g = self.grads * grad_scale
        self.vel.mul_(self.momentum).sub_(lr_t * g)
        if self.nesterov:
            self.params.add_(self.momentum * self.vel - lr_t * g)
        else:
            self.params.add_(self.vel)
        if self.zero_grads:
            self.grads.zero_()

    @property
    def steps_taken(self) -> int:
        if self.step_dev is not None:
            return int(self.step_dev[0].item())
        return self.iterations

    def state_dict(self) -> dict:
        self.iterations = self.steps_taken
        return {"kind": "sgd", "iterations": self.iterations, "vel": self.vel.detach().cpu(),
                "lr": self.lr, "momentum": self.momentum, "decay": self.decay,
                "nesterov": self.nesterov}

    def load_state_dict(self, sd: dict) -> None:
        self.iterations = int(sd["iterations"])
        if self.step_dev is not None:
            self.step_dev.zero_()
            self.step_dev[0] = float(self.iterations)
        self.vel.copy_(sd["vel"])
        self.lr, self.momentum, self.decay, self.nesterov = sd["lr"], sd["momentum"], sd["decay"], sd["nesterov"]


def make_optimizer(name: str, params, grads, **kw):
    name = name.lower()
    if name in ("adam", "adamw"):
        return FlatAdam(params, grads, **kw)
    if name in ("sgd", "sgd_nesterov"):
        return FlatSGD(params, grads, **kw)
    raise ValueError(f"unknown optimizer {name!r}")
