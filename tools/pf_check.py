"""Persistent forward variants (WELLFLOW_PF_DBG values) against the per-step forward:
max |diff| and the count of differing elements of h (XH), C and S, per shape."""
import os
import sys

import torch

sys.path.insert(0, ".")
from wellflow.data.synth import synth_lstm_batch  # noqa: E402
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402

variants = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0"]  # WELLFLOW_PF_DBG values
for B, H, T in ((8192, 512, 8), (512, 256, 6), (256, 128, 5), (2048, 512, 64)):
    F = 16
    eng = NativeLSTM(F, H, T, B, device="cuda")
    eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
    eng.sync_weights()
    x, _ = synth_lstm_batch(B, T, F, seed=2)
    x = x.cuda()
    C, dims = eng._C, eng._dims(B)
    C.lstm_pack_x(x, eng.XH, *dims, True)
    C.lstm_forward(eng.XH, eng.Wp, eng.Cst, eng.S, eng.dcarry, *dims, 6)
    ref = (eng.XH.clone(), eng.Cst.clone(), eng.S.clone())
    for v in variants:
        if int(v) and H != 512:
            continue  # diagnostic variants exist at H = 512 only
        os.environ["WELLFLOW_PF_DBG"] = v
        eng.XH[B * eng.lay.KA:].zero_()
        C.lstm_pack_x(x, eng.XH, *dims, True)
        eng.Cst[B * H:].zero_()
        eng.S.zero_()
        C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *dims)
        torch.cuda.synchronize()
        out = []
        for name, a, b in zip(("XH", "C", "S"), (eng.XH, eng.Cst, eng.S), ref):
            d = (a.float() - b.float()).abs()
            out.append(f"{name} max {d.max().item():.4g} ndiff {(d > 0).sum().item()}/{d.numel()}")
        print(f"B={B} H={H} T={T} dbg={v}: " + "  ".join(out), flush=True)
    os.environ["WELLFLOW_PF_DBG"] = "0"
