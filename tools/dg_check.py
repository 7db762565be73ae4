import sys, torch
sys.path.insert(0, ".")
from wellflow.data.synth import synth_lstm_batch
from wellflow.models.lstm import NativeLSTM, init_lstm_flat
for (B, H, T) in [(8192, 512, 8), (2048, 512, 64), (512, 256, 6)]:
    F = 16
    eng = NativeLSTM(F, H, T, B, device="cuda")
    eng.params.copy_(init_lstm_flat(F, H, seed=4).cuda()); eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F, seed=5); x, y = x.cuda(), y.cuda()
    res = {}
    for pb in (False, True):
        eng.persistent_bwd = pb
        eng.forward_backward(x, y, grad_scale=1.0 / B); torch.cuda.synchronize()
        res[pb] = (eng.DG.clone().float(), eng.grads.clone())
    (d0, g0), (d1, g1) = res[False], res[True]
    G = 4 * H
    d0 = d0.view(T, B, G); d1 = d1.view(T, B, G)
    for t in [T - 1, T - 2, T - 3, 0]:
        a, b = d0[t], d1[t]
        print(B, H, T, "t", t, "max", (a - b).abs().max().item(), "scale", a.abs().max().item(), "relF", ((a - b).norm() / a.norm()).item(), flush=True)
    print("  grad rel", ((g0 - g1).norm() / g0.norm()).item())
