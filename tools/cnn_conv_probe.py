"""Conv-weight gradient of the fused CNN backward vs (a) the fp32 reference and (b) a torch
emulation of the kernels' bf16 roundings (round-5 probe: is a 5 % conv error numerics or a bug?)."""
import sys

import torch

sys.path.insert(0, ".")
from wellflow.models.base import per_element_loss  # noqa: E402
from wellflow.models.cnn import CNN1DRegressor, NativeCNN, cnn_dropout_mask  # noqa: E402

DEV = "cuda:0"
bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731

for loss, B, dp_ in (("mse", 1000, 0.5), ("mae_clip", 4096, 0.5), ("mse", 1000, 0.0), ("mse", 64, 0.5)):
    torch.manual_seed(2)
    ref = CNN1DRegressor(dropout=dp_).init_keras(4).to(DEV)
    with torch.no_grad():
        ref.conv.bias.uniform_(-0.05, 0.05)
        ref.dense.bias.uniform_(-0.1, 0.1)
    eng = NativeCNN(ref.layout, batch=max(4096, B), device=DEV, dropout=dp_, loss=loss, seed=7)
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()
    x, y = torch.randn(B, 48, 1, device=DEV), torch.randn(B, 12, device=DEV)
    eng.rng.fill_(5)
    eng.forward_backward(x, y, grad_scale=1.0 / (B * 12))
    torch.cuda.synchronize()
    gWc_n = eng.lay.views(eng.grads)[0][:100, :14]
    mask = cnn_dropout_mask(eng.seed32, 5, B, 36, eng.lay.Fp, device=DEV)[:, :, :100].float()
    ks = 2.0
    if dp_ == 0.0:
        mask, ks = torch.ones_like(mask), 1.0
    gWd_n = eng.lay.views(eng.grads)[1][:12].view(12, 36, 112)[:, :, :100]
    dout_n = eng.dout[: B * 16].view(B, 16)[:, :12]
    # fp32 reference
    xr = x.clone()
    h = torch.relu(ref.conv(xr.transpose(1, 2))).transpose(1, 2) * mask * ks
    out = ref.dense(h.reshape(B, -1))
    L = per_element_loss(loss, out, y).sum() / (B * 12)
    ref.zero_grad()
    L.backward()
    gWc_r = torch.cat([ref.conv.weight.grad.view(100, 13), ref.conv.bias.grad.view(100, 1)], 1)
    # bf16 emulation of the kernels
    Wc, bc = ref.conv.weight.detach().view(100, 13), ref.conv.bias.detach()
    Wd, bd = ref.dense.weight.detach().view(12, 36, 100), ref.dense.bias.detach()
    xw = bf(x.view(B, 48))
    win = torch.stack([xw[:, t : t + 13] for t in range(36)], 1)  # [B, T, 13]
    p = win @ bf(Wc).t() + bf(bc)  # [B, T, F]
    act = torch.relu(bf(p)) * mask
    o = torch.einsum("btf,jtf->bj", act, bf(Wd)) * ks + bd
    o = o.detach().requires_grad_(True)
    per_element_loss(loss, o, y).sum().mul(1.0 / (B * 12)).backward()
    dout = o.grad
    doA = bf(dout * ks)
    gWd_e = torch.einsum("btf,bj->jtf", act, doA)
    dA = torch.einsum("bj,jtf->btf", doA, bf(Wd))
    dp = bf(dA) * (act != 0).float()
    gW = torch.einsum("btf,btk->fk", dp, win)
    gb = dp.sum((0, 1))
    gWc_e = torch.cat([gW, gb[:, None]], 1)
    print(f"{loss} B={B} p={dp_}: dout vs emu {rel(dout_n, dout):.4f} dWd vs emu {rel(gWd_n, gWd_e):.4f}; "
          f"dWc: native vs fp32 {rel(gWc_n, gWc_r):.4f}  native vs bf16-emulation {rel(gWc_n, gWc_e):.4f}  "
          f"emulation vs fp32 {rel(gWc_e, gWc_r):.4f}")
