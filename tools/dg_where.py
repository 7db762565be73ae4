"""Localise persistent-backward mismatches (DG at the first persistent step) by row tile / unit."""
import sys, torch
sys.path.insert(0, ".")
from wellflow.data.synth import synth_lstm_batch
from wellflow.models.lstm import NativeLSTM, init_lstm_flat
B, H, T, F = 8192, 512, 8, 16
eng = NativeLSTM(F, H, T, B, device="cuda")
eng.params.copy_(init_lstm_flat(F, H, seed=4).cuda()); eng.sync_weights()
x, y = synth_lstm_batch(B, T, F, seed=5); x, y = x.cuda(), y.cuda()
res = {}
for pb in (False, True):
    eng.persistent_bwd = pb
    eng.forward_backward(x, y, grad_scale=1.0 / B); torch.cuda.synchronize()
    res[pb] = eng.DG.clone().float().view(T, B, 4 * H)
t = T - 2
d = (res[False][t] - res[True][t]).abs()
scale = res[False][t].abs().max()
bad = d > 1e-3 * scale
print("bad elems", int(bad.sum()), "of", d.numel())
rows = bad.any(1).nonzero().flatten()
print("bad rows (first 40)", rows[:40].tolist())
rt = (rows % 256) // 16
print("row tile within WG histogram", torch.bincount(rt, minlength=16).tolist())
print("row-in-tile histogram", torch.bincount(rows % 16, minlength=16).tolist())
cols = bad.any(0).nonzero().flatten()
u = cols // 4
print("unit blocks (64) histogram", torch.bincount(u // 64, minlength=8).tolist())
print("unit within 16 histogram", torch.bincount(u % 16, minlength=16).tolist())
print("gate histogram", torch.bincount(cols % 4, minlength=4).tolist())
