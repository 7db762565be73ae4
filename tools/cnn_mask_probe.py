"""Which keep-bit mapping does the fused CNN forward apply? Emulates the forward's dOut under
candidate mappings and reports the distance to the kernel's dOut (round-5 probe)."""
import sys

import torch

sys.path.insert(0, ".")
from wellflow.models.base import per_element_loss  # noqa: E402
from wellflow.models.cnn import CNN1DRegressor, NativeCNN, _lowbias32, _M32  # noqa: E402

DEV = "cuda:0"
bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731


def words(seed, step, B, T):
    smix = _lowbias32(torch.tensor(seed & _M32) ^ _lowbias32(torch.tensor((step + 0x9E3779B9) & _M32)))
    w = torch.arange(B).view(B, 1, 1)
    t = torch.arange(T).view(1, T, 1)
    q = torch.arange(4).view(1, 1, 4)
    return _lowbias32((((w * T + t) & _M32) * 4 + q) & _M32 ^ smix).to(DEV)  # [B, T, 4]


f = torch.arange(100, device=DEV)
maps = {
    "current": 2 * (f >> 4) + ((f & 3) >> 1) + 16 * (f & 1),
    "r4": 4 * (f >> 4) + (f & 3),
    "swap_hi_lo": 2 * (f >> 4) + ((f & 3) >> 1) + 16 * (1 - (f & 1)),
    "b_only": 2 * (f >> 4) + 16 * (f & 1),
    "h_as_q": 2 * (f >> 4) + ((f & 3) >> 1) + 16 * (f & 1),
}
torch.manual_seed(2)
B = 1000
ref = CNN1DRegressor(dropout=0.5).init_keras(4).to(DEV)
with torch.no_grad():
    ref.conv.bias.uniform_(-0.05, 0.05)
eng = NativeCNN(ref.layout, batch=4096, device=DEV, dropout=0.5, loss="mse", seed=7)
eng.params.copy_(ref.to_flat().to(DEV))
eng.sync_weights()
x, y = torch.randn(B, 48, 1, device=DEV), torch.randn(B, 12, device=DEV)
eng.rng.fill_(5)
eng.forward_backward(x, y, grad_scale=1.0 / (B * 12))
torch.cuda.synchronize()
dout_n = eng.dout[: B * 16].view(B, 16)[:, :12]
W = words(eng.seed32, 5, B, 36)  # [B, T, 4] hash words per q
Wc, bc = ref.conv.weight.detach().view(100, 13), ref.conv.bias.detach()
Wd, bd = ref.dense.weight.detach().view(12, 36, 100), ref.dense.bias.detach()
xw = bf(x.view(B, 48))
win = torch.stack([xw[:, t : t + 13] for t in range(36)], 1)
p = win @ bf(Wc).t() + bf(bc)
qf = (f >> 2) & 3
for name, bit in maps.items():
    mask = ((W[:, :, qf] >> bit) & 1).float()
    act = torch.relu(bf(p)) * mask
    o = (torch.einsum("btf,jtf->bj", act, bf(Wd)) * 2.0 + bd).requires_grad_(True)
    per_element_loss("mse", o, y).sum().mul(1.0 / (B * 12)).backward()
    print(f"{name:12s} dout rel distance {rel(dout_n, o.grad):.5f}")
# per-filter check: drop one filter block's contribution at a time is not observable; report
# the kept fraction per (f & 3) under the current mapping for sanity
bit = maps["current"]
mask = ((W[:, :, qf] >> bit) & 1).float()
act = torch.relu(bf(p)) * mask
o = (torch.einsum("btf,jtf->bj", act, bf(Wd)) * 2.0 + bd).requires_grad_(True)
per_element_loss("mse", o, y).sum().mul(1.0 / (B * 12)).backward()
err = (dout_n - o.grad).abs().sum(1) / o.grad.abs().sum(1).clamp_min(1e-12)
bad = (err > 1e-3).nonzero().flatten()
print("windows off:", bad.numel(), "of", B, "first", bad[:20].tolist())
print("by w % 16:", torch.bincount(bad % 16, minlength=16).tolist())
print("by group:", torch.bincount(bad // 16, minlength=(B + 15) // 16)[:64].tolist())
# the forward output itself: which (t, f) of a bad window would fix it? try flipping each bit
if bad.numel():
    w0 = int(bad[0])
    base = (o.grad[w0] - dout_n[w0]).norm().item()
    best = []
    for t in range(36):
        for ff in range(100):
            m2 = mask[w0].clone()
            m2[t, ff] = 1 - m2[t, ff]
            a2 = torch.relu(bf(p[w0])) * m2
            o2 = (torch.einsum("tf,jtf->j", a2, bf(Wd)) * 2.0 + bd)
            d2 = 2 * (o2 - y[w0]) / (B * 12)
            e = (d2 - dout_n[w0]).norm().item()
            if e < 0.5 * base:
                best.append((t, ff, e / base))
    print("window", w0, "single flips that halve the error:", best[:10])
