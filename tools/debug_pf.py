"""Persistent-forward bring-up: compare against the per-step kernels and locate mismatches."""
import sys

import torch

sys.path.insert(0, ".")
from wellflow.data.synth import synth_lstm_batch  # noqa: E402
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402


VERBOSE = False


def run(B, H, T, F=16):
    eng = NativeLSTM(F, H, T, B, device="cuda")
    eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
    eng.sync_weights()
    x, _ = synth_lstm_batch(B, T, F, seed=2)
    x = x.cuda()
    C, dims, KA = eng._C, eng._dims(B), eng.lay.KA
    C.lstm_pack_x(x, eng.XH, *dims)
    C.lstm_forward(eng.XH, eng.Wp, eng.Cst, eng.S, *dims, 6)
    ref = (eng.XH.clone(), eng.Cst.clone(), eng.S.clone())
    eng.XH[B * KA:].zero_()
    C.lstm_pack_x(x, eng.XH, *dims)
    eng.Cst[B * H:].zero_()
    eng.S.zero_()
    ok = C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *dims)
    torch.cuda.synchronize()
    print(f"B={B} H={H} T={T} ok={ok} err={int(eng.sync[0].item())} cnt0={int(eng.sync[16].item())}")
    XH = eng.XH.view(T + 1, B, KA).float()
    R = ref[0].view(T + 1, B, KA).float()
    for t in range(1, T + 1):
        d = (XH[t, :, 64:] - R[t, :, 64:]).abs()
        bad = d > 1e-2
        nb = int(bad.sum())
        print(f"  h_{t - 1}: maxdiff {d.max().item():.4f} bad {nb}/{d.numel()}")
        if nb and t <= 2 and VERBOSE:
            idx = bad.nonzero()
            rows, cols = idx[:, 0], idx[:, 1]
            print("    rows%32 hist", torch.bincount(rows % 32, minlength=32).tolist())
            print("    unit%64 hist", torch.bincount(cols % 64, minlength=64).tolist())
            print("    rowblock(256) hist", torch.bincount(rows // 256).tolist()[:40])
            print("    unitblock(64) hist", torch.bincount(cols // 64).tolist())
            print("    sample", idx[:8].tolist(), XH[t, rows[:4], 64 + cols[:4]].tolist(), R[t, rows[:4], 64 + cols[:4]].tolist())
    dc = (eng.Cst - ref[1]).abs().view(T + 1, -1).amax(1)
    ds = (eng.S.float() - ref[2].float()).abs().view(T, -1).amax(1)
    print("  C maxdiff per t", [round(v, 4) for v in dc.tolist()])
    print("  S maxdiff per t", [round(v, 4) for v in ds.tolist()])


if __name__ == "__main__":
    cfgs = [(1024, 512, 1), (2048, 512, 1), (4096, 512, 1), (8192, 128, 1), (16384, 128, 1), (16384, 256, 1),
            (1024, 512, 3)]
    if len(sys.argv) > 1:
        cfgs = [tuple(map(int, a.split(","))) for a in sys.argv[1:]]
    for B, H, T in cfgs:
        run(B, H, T)
