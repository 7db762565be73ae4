"""LSTM time-series regression (README "LSTM model", Readme.md:21; BASELINE.json:11 —
seq-len 64, hidden 512, DP, bf16).

Two implementations with one parameter layout:

* :class:`LSTMRegressor` — plain PyTorch fp32 module (``nn.LSTM`` + linear head). It is
  the CPU oracle for val-MSE parity and the reference for the kernel tests.
* :class:`NativeLSTM` — the MI355X engine: ONE persistent launch for the whole forward
  (all T steps; gate weights resident in registers, h handed between workgroups in-launch:
  csrc/lstm_persistent_fwd.inc.h), step T-1 of the backward plus ONE persistent launch for
  steps T-2..0 (csrc/lstm_persistent_bwd.inc.h), and a single split-K weight-gradient GEMM
  over all (t, b) (csrc/gemm_core.h). The per-timestep kernels of csrc/lstm.hip remain the
  fallback for shapes the persistent schedule cannot host (a one-time notice says so).
  Parameters live in a flat fp32 master buffer (so the optimizer and the DP all-reduce
  are one launch / one collective each); the fused Adam launch also writes the bf16 operand
  images the kernels read.

Flat layout (``LstmLayout``): ``[Wcat (4H x KA, unit-major rows 4u+g) | w_out (H) | b_out (1)]``
with ``Wcat = [W_ih | b_ih + b_hh | 0 ... | W_hh]`` (KA = KX + H, KX = 64-aligned, the
bias rides on a constant-1 input column).
"""
from __future__ import annotations

import dataclasses
import math
import os
import sys

import torch
from torch import nn


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclasses.dataclass(frozen=True)
class LstmLayout:
    n_features: int
    hidden: int

    @property
    def KX(self) -> int:
        return _round_up(self.n_features + 1, 64)

    @property
    def KA(self) -> int:
        return self.KX + self.hidden

    @property
    def G(self) -> int:
        return 4 * self.hidden

    @property
    def w_size(self) -> int:
        return self.G * self.KA

    @property
    def numel(self) -> int:
        return _round_up(self.w_size + self.hidden + 1, 4)

    def views(self, flat: torch.Tensor):
        W = flat[: self.w_size].view(self.G, self.KA)
        w_out = flat[self.w_size : self.w_size + self.hidden]
        b_out = flat[self.w_size + self.hidden : self.w_size + self.hidden + 1]
        return W, w_out, b_out

    def perm(self) -> torch.Tensor:
        """perm[p] = natural gate-row (gate*H + unit) stored at master row p = 4*unit + gate
        (csrc/lstm_layout.h dg_col: the backward's gate-gradient column order; the
        forward's bf16 weights are re-permuted by the pack kernel)."""
        p = torch.arange(self.G)
        return (p & 3) * self.hidden + (p >> 2)


class LSTMRegressor(nn.Module):
    """fp32 reference: x [B, T, F] -> y [B] from the last hidden state."""

    def __init__(self, n_features: int, hidden: int = 512):
        super().__init__()
        self.n_features = n_features
        self.hidden = hidden
        self.lstm = nn.LSTM(n_features, hidden, batch_first=True)
        self.head = nn.Linear(hidden, 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out, _ = self.lstm(x)
        return self.head(out[:, -1]).squeeze(-1)

    # ---- flat-layout conversion (shared with NativeLSTM / checkpoints) ----
    def to_flat(self) -> torch.Tensor:
        lay = LstmLayout(self.n_features, self.hidden)
        flat = torch.zeros(lay.numel, dtype=torch.float32)
        W, w_out, b_out = lay.views(flat)
        nat = torch.zeros(lay.G, lay.KA)
        F, H = self.n_features, self.hidden
        with torch.no_grad():
            nat[:, :F] = self.lstm.weight_ih_l0.float().cpu()
            nat[:, F] = (self.lstm.bias_ih_l0 + self.lstm.bias_hh_l0).float().cpu()
            nat[:, lay.KX :] = self.lstm.weight_hh_l0.float().cpu()
            W.copy_(nat[lay.perm()])
            w_out.copy_(self.head.weight.view(-1).float().cpu())
            b_out.copy_(self.head.bias.view(-1).float().cpu())
        return flat

    def load_flat(self, flat: torch.Tensor) -> None:
        lay = LstmLayout(self.n_features, self.hidden)
        W, w_out, b_out = lay.views(flat.detach().float().cpu())
        nat = torch.empty_like(W)
        nat[lay.perm()] = W
        F = self.n_features
        with torch.no_grad():
            self.lstm.weight_ih_l0.copy_(nat[:, :F])
            self.lstm.bias_ih_l0.copy_(nat[:, F])
            self.lstm.bias_hh_l0.zero_()
            self.lstm.weight_hh_l0.copy_(nat[:, lay.KX :])
            self.head.weight.copy_(w_out.view(1, -1))
            self.head.bias.copy_(b_out)


# completion STAT block at the end of every persistent sync buffer (csrc/persistent_guard.h)
PSTAT_WORDS = 64
_PST_STICKY, _PST_DONE, _PST_EXPECT, _PST_STARTED, _PST_EXPECT_WG, _PST_EXITS, _PST_LAUNCHES = range(7)
_PST_REC = 8
_EXIT_REASONS = {1: "the launch's error word was set while it polled (another workgroup's spin bound)",
                 2: "its own hand-off spin bound tripped",
                 3: "wave 0 read a hand-off flag != 1 from LDS although its own poll succeeded",
                 4: "a wave read a hand-off flag != 1 from LDS",
                 5: "the sync buffer was last used by a launch of another shape (row tiles, steps): "
                    "zero it (reset_device_errors) before changing the batch"}


def persistent_sync_buffer(B: int, row_quantum: int, device) -> torch.Tensor:
    """int32 sync buffer of a persistent LSTM kernel for batches <= B, zeroed here once: one
    64-B line of hand-off words per row block of ``row_quantum`` rows (launch epoch, group
    arrival counters, tagged error word; csrc/persistent_sync.h — they only count up, no
    launch resets them) and the STAT block of running completion totals at its end."""
    return torch.zeros(16 + 16 * (B // row_quantum + 1) + PSTAT_WORDS, dtype=torch.int32, device=device)


def decode_pstat(words) -> dict:
    """STAT block (list of 64 ints) -> named totals + the first early-exit record."""
    w = [int(v) & 0xFFFFFFFF for v in words]
    rec = None
    if w[_PST_REC - 1]:
        r = w[_PST_REC : _PST_REC + 8]
        rec = {"block": r[0], "step": r[1], "reason": r[2], "why": _EXIT_REASONS.get(r[2], "?"),
               "err_seen": r[3], "arrivals_seen": r[4], "target": r[5], "flag": r[6], "started_ordinal": r[7]}
    return {"sticky": w[_PST_STICKY], "done": w[_PST_DONE], "expect": w[_PST_EXPECT], "started": w[_PST_STARTED],
            "expect_wg": w[_PST_EXPECT_WG], "exits": w[_PST_EXITS], "launches": w[_PST_LAUNCHES], "first_exit": rec}


def pstat_error(st: dict) -> int:
    """0 = every launch since the reset completed; bit 0 spin bound tripped, bit 1 short
    step count, bit 2 workgroups that never started, bit 3 early exits recorded."""
    e = 1 if st["sticky"] else 0
    e |= 2 if st["done"] != st["expect"] else 0
    e |= 4 if st["started"] != st["expect_wg"] else 0
    e |= 8 if st["exits"] else 0
    return e


def init_lstm_flat(n_features: int, hidden: int, seed: int = 0) -> torch.Tensor:
    """PyTorch-default init (U(-1/sqrt(H), 1/sqrt(H))) in the flat layout."""
    g = torch.Generator().manual_seed(seed)
    lay = LstmLayout(n_features, hidden)
    k = 1.0 / math.sqrt(hidden)
    flat = torch.zeros(lay.numel)
    W, w_out, b_out = lay.views(flat)
    W[:, :n_features].uniform_(-k, k, generator=g)
    W[:, n_features].uniform_(-2 * k, 2 * k, generator=g)  # b_ih + b_hh
    W[:, lay.KX :].uniform_(-k, k, generator=g)
    w_out.uniform_(-k, k, generator=g)
    b_out.uniform_(-k, k, generator=g)
    return flat


class NativeLSTM:
    """HIP/MFMA LSTM regression engine for a fixed (max) batch size.

    ``params``/``grads`` are flat fp32 device buffers in :class:`LstmLayout` order;
    call :meth:`sync_weights` after every change to ``params``.
    """

    native = True
    window_indexed = True  # forward_backward(windows, y, ..., rows=) reads the windows in place

    def __init__(self, n_features: int, hidden: int, seq_len: int, batch: int,
                 device="cuda", params: torch.Tensor | None = None,
                 grads: torch.Tensor | None = None, loss: str = "mse", clip: float = 6.0):
        from ..ops.native import lib

        self._C = lib()
        self.loss_kind, self.clip = loss, clip
        self.lay = LstmLayout(n_features, hidden)
        self.F, self.H, self.T, self.B = n_features, hidden, seq_len, batch
        lay = self.lay
        dev = torch.device(device)
        self.device = dev
        self.params = params if params is not None else torch.zeros(lay.numel, device=dev)
        self.grads = grads if grads is not None else torch.zeros(lay.numel, device=dev)
        bf = torch.bfloat16
        T, B, H = seq_len, batch, hidden
        Bp = _round_up(B, 16)  # fragment-native state (C, S, dc carry) is 16-row padded
        self.XH = torch.zeros((T + 1) * B * lay.KA, dtype=bf, device=dev)
        # cell-state history c_t for the backward, bf16 (slab 0 = c_{-1} = 0 stays zero); the
        # forward carries c in fp32 (persistent: registers; per-step: dcarry as an fp32 slab)
        self.Cst = torch.zeros((T + 1) * Bp * H, dtype=bf, device=dev)
        self.S = torch.empty(T * Bp * lay.G, dtype=bf, device=dev)
        self.DG = torch.empty(T * B * lay.G, dtype=bf, device=dev)
        self.dcarry = torch.empty(Bp * H, dtype=torch.float32, device=dev)
        self.Wp = torch.empty(lay.G * lay.KA, dtype=bf, device=dev)
        self._xh_const = False  # XH's constant x-block columns written (_pack_x)
        self.WhhT = torch.empty(H * lay.G, dtype=bf, device=dev)
        self.pred = torch.empty(B, dtype=torch.float32, device=dev)
        self.dy = torch.empty(B, dtype=torch.float32, device=dev)
        self.loss_sum = torch.zeros(1, dtype=torch.float32, device=dev)
        # tile shapes (csrc/kernels.h LstmDims), A/B-tuned on MI355X with tools/tune_lstm.py
        # (profiles/r1_*): fwd 256x256 glds ring (v6), bwd 64x128 glds ring (v9); dW split-K 32.
        self.fwd_variant, self.bwd_variant = 6, 8
        # persistent forward (csrc/lstm_persistent.hip): all T steps in ONE cooperative
        # launch with the gate weights resident in registers; falls back to the per-step
        # kernels (fwd_variant) when the shape / device cannot host it
        self.persistent = os.environ.get("WELLFLOW_PERSISTENT", "1") != "0"
        self.sync = persistent_sync_buffer(B, 32, dev)
        self.last_forward_persistent = False
        # persistent backward (csrc/lstm_persistent_bwd.hip): steps T-2..0 in ONE launch,
        # W_hh^T in registers, dc carry in LDS; per-step kernels (bwd_variant) otherwise
        self.persistent_bwd = os.environ.get("WELLFLOW_PERSISTENT_BWD", "1") != "0"
        self.sync_bwd = persistent_sync_buffer(B, 64, dev)
        self.dw_ksplit = 0  # 0 = heuristic
        # timesteps per overlapped dW GEMM chunk; 0 = serial dW at the end (measured faster:
        # the BPTT chain already fills every CU, overlapping only adds contention)
        self.dw_chunk = 0
        # split-K partial slab of the dW GEMM (csrc/gemm.hip launch_dw_288w): each split's tile
        # plain-stored and one reduce, instead of fp32 atomics into gW (WELLFLOW_DW_SLAB=0: atomics)
        self.dw_slab = None
        if os.environ.get("WELLFLOW_DW_SLAB", "1") != "0":
            self.dw_slab = torch.empty(self._dw_slab_splits(lay.G, lay.KA, T * B, dev) * lay.G * lay.KA,
                                       dtype=torch.float32, device=dev)
        self._fallback_noted = set()
        self.last_backward_persistent = False
        self.sync_weights()

    @staticmethod
    def _dw_slab_splits(G: int, KA: int, K: int, device) -> int:
        """Split-K partials the dW GEMM will actually store (csrc/gemm.hip launch_dw_288w: the
        heuristic split min(32, K / 16384), clamped to one workgroup per CU, i.e. CUs / tiles =
        16 on 256 CUs), so the slab is no larger than what is written (round-4 ADVICE: 32 splits
        were allocated, 151 MB at the default shape, half never written). A larger explicit
        dw_ksplit than this falls back to atomics in the launcher (slab_cap check)."""
        ks = max(1, min(32, K // 16384))
        if G % 256 == 0 and KA % 288 == 0:
            tiles = (G // 256) * (KA // 288)
            cus = torch.cuda.get_device_properties(device).multi_processor_count
            if ks * tiles > cus and cus // tiles >= 1:
                ks = cus // tiles
        return ks

    @staticmethod
    def full_grid_batch(hidden: int, device) -> int:
        """Rows per step that fill ONE co-resident persistent grid on this device: 256 rows
        (8 chunks of 32) per workgroup, (4 hidden / 256) gate-column workgroups per row block,
        one workgroup per CU (csrc/lstm_persistent.hip persistent_split) — 8192 at H = 512 on
        a 256-CU MI355X. A job's default LSTM batch (config.py batch_size 0 = auto): the
        reference's small batches (cnn.py:128 uses 20) would run a 64-workgroup grid on 256 CUs."""
        props = torch.cuda.get_device_properties(device)
        nb = max(1, 4 * hidden // 256)
        return 256 * max(1, props.multi_processor_count // nb)

    # ------------------------------------------------------------------ weights
    def fused_adam_ok(self, opt) -> bool:
        """Whether :meth:`fused_adam` covers ``opt`` (train/step.py decides from the same
        predicate whether the step still needs its own sync_weights launch)."""
        # (the kernel transposes W_hh in 32 x 32 tiles)
        return opt.shadow is None and opt.shadow_t is None and self.H % 32 == 0 and self.lay.KX % 32 == 0

    def fused_adam(self, opt, grad_scale: float) -> bool:
        """The optimizer's Adam update and this engine's bf16 compute copies (Wp, WhhT) in ONE
        launch (optim/flat.py FlatAdam ``writeback``; csrc/elementwise.hip lstm_adam_pack_kernel)."""
        if not self.fused_adam_ok(opt):
            return False
        b1, b2 = opt.betas
        self._C.lstm_adam_pack(self.params, self.grads, opt.m, opt.v, opt.step_dev, opt.lr, b1, b2, opt.eps,
                               opt.weight_decay, grad_scale, opt.zero_grads, self.Wp, self.WhhT, self.H, self.lay.KX)
        return True

    def sync_weights(self) -> None:
        W, _, _ = self.lay.views(self.params)
        self._C.lstm_pack_weights(W, self.Wp, self.WhhT, self.H, self.lay.KX)

    def _dims(self, B):
        return (B, self.T, self.F, self.lay.KX, self.H)

    def _pack_x(self, x, B):
        """x -> the bf16 x block of XH. The block's constant part (the 1 column of the bias,
        the zero padding up to KX) is written by the first pack only: later packs write the
        feature chunks alone (csrc/lstm.hip lstm_pack_x_kernel)."""
        self._C.lstm_pack_x(x, self.XH, *self._dims(B), not self._xh_const)
        self._xh_const = True

    def _hT(self, B):
        lay = self.lay
        base = self.T * self.B * lay.KA  # XH[T] starts here (row stride KA)
        return self.XH[base + lay.KX : base + lay.KX + (B - 1) * lay.KA + self.H]

    def _note_fallback(self, which: str, enabled: bool) -> None:
        """Say ONCE per engine that a pass runs as per-step kernels (a silent fallback costs
        ~25 % of the step): either disabled by env or refused for this shape / device."""
        if which in self._fallback_noted:
            return
        self._fallback_noted.add(which)
        why = ("disabled (WELLFLOW_PERSISTENT%s=0)" % ("_BWD" if which == "backward" else "")
               if not enabled else "shape/device not supported by the persistent schedule")
        print(f"wellflow: LSTM {which} runs per-step kernels: {why} "
              f"(B={self.B} T={self.T} F={self.F} H={self.H})", file=sys.stderr, flush=True)

    def _forward_steps(self, B):
        C = self._C
        # raises if the launch itself fails; False = shape / device cannot host the schedule
        ok = self.persistent and C.lstm_forward_persistent(self.XH, self.Wp, self.Cst, self.S, self.sync,
                                                          *self._dims(B))
        if not ok:
            self._note_fallback("forward", self.persistent)
            C.lstm_forward(self.XH, self.Wp, self.Cst, self.S, self.dcarry, *self._dims(B), self.fwd_variant)
        self.last_forward_persistent = bool(ok)

    def persistent_stats(self) -> dict:
        """Running completion totals of the persistent forward / backward since the last
        :meth:`reset_device_errors` (csrc/persistent_guard.h; one host sync)."""
        w = torch.stack([self.sync[-PSTAT_WORDS:], self.sync_bwd[-PSTAT_WORDS:]]).cpu().tolist()
        return {"forward": decode_pstat(w[0]), "backward": decode_pstat(w[1])}

    def persistent_error(self) -> int:
        """Bits 0-3: forward, bits 4-7: backward (:func:`pstat_error`) — covers EVERY launch and
        sub-batch since the last :meth:`reset_device_errors`, not only the last one."""
        st = self.persistent_stats()
        return pstat_error(st["forward"]) | (pstat_error(st["backward"]) << 4)

    def reset_device_errors(self) -> None:
        """Zero both sync buffers WHOLE: the STAT totals and the monotonic hand-off words
        (csrc/persistent_sync.h: launch epochs and group arrival counters only count up, and
        no launch resets them, so they are cleared only together, between launches)."""
        self.sync.zero_()
        self.sync_bwd.zero_()

    def check_device_errors(self) -> None:
        """Raise if any persistent launch since the last reset left work undone (a tripped
        spin bound, an early exit, a short step count or workgroups that never started): the
        state of the affected steps is garbage."""
        st = self.persistent_stats()
        bad = {k: v for k, v in st.items() if pstat_error(v)}
        if not bad:
            return
        what = []
        for k, v in bad.items():
            e = pstat_error(v)
            parts = []
            if e & 1:
                parts.append("hit the hand-off spin bound (a workgroup never arrived: non-resident grid or a hung wave)")
            if e & 2:
                parts.append(f"completed {v['done']} of {v['expect']} workgroup-steps")
            if e & 4:
                parts.append(f"started {v['started']} of {v['expect_wg']} workgroups")
            if e & 8:
                parts.append(f"{v['exits']} waves exited early")
            if v["first_exit"]:
                parts.append(f"first exit: {v['first_exit']}")
            what.append(f"{k} ({v['launches']} launches): " + "; ".join(parts))
        raise RuntimeError("persistent LSTM " + " | ".join(what) + "; results of the affected steps are invalid")

    # ------------------------------------------------------------------ passes
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: [B, T, F] fp32 (B <= max batch) -> predictions [B] (view of an internal buffer)."""
        B = x.shape[0]
        assert x.shape[1] == self.T and x.shape[2] == self.F and B <= self.B
        x = x.contiguous().float()
        # XH is laid out for the max batch B; a smaller batch uses the leading rows of
        # every timestep slab only if B == self.B, so smaller batches run padded.
        if B != self.B:
            xp = torch.zeros(self.B, self.T, self.F, device=x.device)
            xp[:B] = x
            x = xp
        C = self._C
        self._pack_x(x, self.B)
        self._forward_steps(self.B)
        _, w_out, b_out = self.lay.views(self.params)
        C.head_fwd(self._hT(self.B), self.lay.KA, self.B, self.H, w_out, b_out, None, self.pred,
                   None, None, 0.0)
        return self.pred[:B]

    def forward_backward(self, x, y: torch.Tensor, grad_scale: float,
                         zero_grads: bool = True, step: int = 0,
                         loss_into: torch.Tensor | None = None, rows: torch.Tensor | None = None) -> torch.Tensor:
        """One training forward + backward on a full batch; grads land in ``self.grads``.

        Gradient of ``grad_scale * sum_i loss_i`` (models/base.py contract; use
        1 / global_batch for the mean over all data-parallel ranks). Returns the device
        scalar sum of per-sample losses of this batch (no host sync). ``rows`` (int64, device):
        ``x`` is a resident :class:`~wellflow.data.features.SeriesWindows` and ``y`` its
        targets; the batch is windows ``rows`` — read in place by the x-pack kernel
        (``window_indexed``: no per-step gather of the [B][T][F] windows).
        """
        B = self.B
        if rows is not None:
            assert rows.shape == (B,) and x.rows.shape[1] == self.F and x.T == self.T
            y = y.index_select(0, rows)
        else:
            assert x.shape == (B, self.T, self.F)
        assert y.shape == (B,)
        C = self._C
        lay = self.lay
        W, w_out, b_out = lay.views(self.params)
        gW, gw_out, gb_out = lay.views(self.grads)
        if zero_grads:
            self.grads.zero_()
        # loss_into: the head kernel adds this batch's loss straight into the caller's
        # accumulator (train/step.py StepRunner: no per-step zero fill and accumulate launch)
        ls = loss_into if loss_into is not None else self.loss_sum
        if loss_into is None:
            self.loss_sum.zero_()
        if rows is not None:
            self._C.lstm_pack_x_win(x.rows, x.starts, rows, self.XH, *self._dims(B), not self._xh_const)
            self._xh_const = True
        else:
            self._pack_x(x.contiguous(), B)
        self._forward_steps(B)
        hT = self._hT(B)
        y = y.contiguous().float()
        # head + MSE + dy + the head's weight gradient in ONE pass over h_T (elementwise.hip
        # head_fwd_bwd_kernel) when the shape allows, else the forward kernel + head_bwd_w
        fused_head = (self.loss_kind == "mse" and
                      C.head_fwd_bwd(hT, lay.KA, B, self.H, w_out, b_out, y, self.pred, self.dy, ls,
                                     2.0 * float(grad_scale), gw_out, gb_out))
        if not fused_head:
            if self.loss_kind == "mse":  # head + MSE + dy fused in one kernel
                C.head_fwd(hT, lay.KA, B, self.H, w_out, b_out, y, self.pred, self.dy,
                           ls, 2.0 * float(grad_scale))
            else:
                C.head_fwd(hT, lay.KA, B, self.H, w_out, b_out, None, self.pred, None, None, 0.0)
                C.loss(1, self.pred, y, B, 1, self.clip, float(grad_scale), ls, None,
                       self.dy, None)
            C.head_bwd_w(hT, lay.KA, B, self.H, self.dy, gw_out, gb_out)
        # BPTT chain (high-priority stream) + dWcat = sum_{t,b} dG_t[b]^T [x_t | 1 | h_{t-1}][b]
        # as split-K GEMM chunks on a low-priority stream, overlapped with the chain.
        K = self.T * B
        ksplit = self.dw_ksplit or max(1, min(32, K // 16384))
        if self.dw_chunk > 0:
            ksplit = max(1, ksplit * self.dw_chunk // self.T)
        pb = C.lstm_backward_dw(self.WhhT, self.XH, self.Cst, self.S, self.DG, self.dcarry, self.dy,
                                w_out, gW, *self._dims(B), self.bwd_variant, self.dw_chunk, ksplit,
                                self.sync_bwd if self.persistent_bwd and self.dw_chunk <= 0 else None,
                                self.dw_slab if self.dw_chunk <= 0 else None)
        self.last_backward_persistent = bool(pb)
        if not pb and self.dw_chunk <= 0:
            self._note_fallback("backward", self.persistent_bwd)
        return ls
