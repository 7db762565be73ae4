"""Decode the fused CNN forward's dropout keep bits exactly (round-5 probe): conv weights 0 and
bias 1 on one filter f0 make every pre-activation of f0 equal 1; dense weights 2^(t - 3j) on
(t, f0) make output j the binary number of the keep bits of steps 3j .. 3j + 2. Compared with
models/cnn.py cnn_dropout_mask per (window, step, filter)."""
import sys

import torch

sys.path.insert(0, ".")
from wellflow.models.cnn import CNN1DRegressor, NativeCNN, cnn_dropout_mask  # noqa: E402

DEV = "cuda:0"
B = 64
ref = CNN1DRegressor(dropout=0.5).init_keras(4).to(DEV)
eng = NativeCNN(ref.layout, batch=B, device=DEV, dropout=0.5, loss="mse", seed=7)
lay = eng.lay
x, y = torch.zeros(B, 48, 1, device=DEV), torch.zeros(B, 12, device=DEV)
want = cnn_dropout_mask(eng.seed32, 5, B, 36, lay.Fp, device=DEV)  # [B, T, Fp]
got = torch.zeros_like(want)
for f0 in range(100):
    flat = torch.zeros(lay.numel, device=DEV)
    Wc, Wd, bd = lay.views(flat)
    Wc[f0, lay.taps] = 1.0  # conv bias of f0 (column taps of the flat conv block)
    Wdv = Wd.view(lay.Op, 36, lay.Fp)
    for t in range(36):
        Wdv[t // 3, t, f0] = float(2 ** (t % 3))
    eng.params.copy_(flat)
    eng.sync_weights()
    eng.rng.fill_(5)
    eng.forward_backward(x, y, grad_scale=1.0)
    torch.cuda.synchronize()
    out = eng.dout[: B * 16].view(B, 16)[:, :12] / 2.0 / 2.0  # dout = 2 * out (mse), out = 2 * bits
    v = out.round().long()
    for t in range(36):
        got[:, t, f0] = ((v[:, t // 3] >> (t % 3)) & 1).bool()
diff = (got[:, :, :100] != want[:, :, :100])
print("mismatching bits:", int(diff.sum()), "of", diff.numel())
if diff.any():
    idx = diff.nonzero()
    print("by f % 16:", torch.bincount(idx[:, 2] % 16, minlength=16).tolist())
    print("by f // 16:", torch.bincount(idx[:, 2] // 16, minlength=7).tolist())
    print("by w % 16:", torch.bincount(idx[:, 0] % 16, minlength=16).tolist())
    print("by t % 4:", torch.bincount(idx[:, 1] % 4, minlength=4).tolist())
    print("first:", idx[:10].tolist())
