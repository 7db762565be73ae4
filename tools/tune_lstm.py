#!/usr/bin/env python3
"""A/B the LSTM kernel tile variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24). Prints median/min ms per phase per variant."""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from wellflow.data.synth import synth_lstm_batch  # noqa: E402
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402
from wellflow.ops.native import gemm  # noqa: E402


def timeit(fn, reps=3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--fwd", default="0,1,2")
    ap.add_argument("--bwd", default="0,1,2,3")
    ap.add_argument("--ksplit", default="8,16,32,64")
    ap.add_argument("--tiles", default="1,2", help="dW GEMM tiles (1: 256x128, 2: 128x288)")
    a = ap.parse_args()
    B, T, F, H = a.batch, 64, 16, 512
    eng = NativeLSTM(F, H, T, B)
    eng.params.copy_(init_lstm_flat(F, H).cuda())
    eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F)
    x, y = x.cuda(), y.cuda()
    eng.forward_backward(x, y, 2.0 / B)
    C = eng._C
    dims = eng._dims(B)
    lay = eng.lay
    gW, _, _ = lay.views(eng.grads)
    # correctness: every variant must reproduce the v0 (register-staged) outputs exactly
    C.lstm_forward(eng.XH, eng.Wp, eng.Cst, eng.S, eng.dcarry, *dims, 0)
    ref_fwd = (eng.XH.clone(), eng.Cst.clone(), eng.S.clone())
    for v in map(int, a.fwd.split(",")):
        eng.Cst[B * H:].zero_(); eng.S.zero_()  # (XH keeps x_t; its h part is rewritten)
        C.lstm_forward(eng.XH, eng.Wp, eng.Cst, eng.S, eng.dcarry, *dims, v)
        torch.cuda.synchronize()
        errs = [(x.float() - y.float()).abs().max().item() for x, y in zip((eng.XH, eng.Cst, eng.S), ref_fwd)]
        print(f"check fwd v{v}: max|diff| XH {errs[0]:.3g} C {errs[1]:.3g} S {errs[2]:.3g}", flush=True)
    w_out = lay.views(eng.params)[1]
    C.lstm_backward(eng.WhhT, eng.XH, eng.Cst, eng.S, eng.DG, eng.dcarry, eng.dy, w_out, *dims, 0, None)
    ref_dg = eng.DG.clone()
    for v in map(int, a.bwd.split(",")):
        eng.DG.zero_()
        C.lstm_backward(eng.WhhT, eng.XH, eng.Cst, eng.S, eng.DG, eng.dcarry, eng.dy, w_out, *dims, v, None)
        torch.cuda.synchronize()
        print(f"check bwd v{v}: max|diff| DG {(eng.DG.float() - ref_dg.float()).abs().max().item():.3g}", flush=True)
    res = {}
    for r in range(a.rounds):
        for v in map(int, a.fwd.split(",")):
            ms = timeit(lambda: C.lstm_forward(eng.XH, eng.Wp, eng.Cst, eng.S, eng.dcarry, *dims, v))
            res.setdefault(f"fwd v{v}", []).append(ms)
        for v in map(int, a.bwd.split(",")):
            ms = timeit(lambda: C.lstm_backward(eng.WhhT, eng.XH, eng.Cst, eng.S, eng.DG, eng.dcarry,
                                                eng.dy, lay.views(eng.params)[1], *dims, v, None))
            res.setdefault(f"bwd v{v}", []).append(ms)
        for ks in map(int, a.ksplit.split(",")):
            for tile in map(int, a.tiles.split(",")):
                def dw():
                    gW.zero_()
                    gemm(eng.DG, eng.XH, lay.G, lay.KA, T * B, a_mn=True, lda=lay.G, b_mn=True, ldb=lay.KA,
                         outF=gW, ldo=lay.KA, atomic=True, ksplit=ks, tile=tile)
                res.setdefault(f"dW tile{tile} ks{ks}", []).append(timeit(dw))
        # decomposition of one backward step: same-shape GEMM alone, cell epilogue alone
        tmp = torch.empty(B * H, dtype=torch.bfloat16, device="cuda")
        A1 = eng.DG[B * lay.G : 2 * B * lay.G]
        res.setdefault("bwd-shape GEMM x63", []).append(
            63 * timeit(lambda: gemm(A1, eng.WhhT, B, H, lay.G, outH=tmp)))
        d1 = (B, 1, F, lay.KX, H)
        res.setdefault("bwd epilogue-only x63", []).append(63 * timeit(lambda: C.lstm_backward(
            eng.WhhT, eng.XH, eng.Cst, eng.S, eng.DG, eng.dcarry, eng.dy, lay.views(eng.params)[1], *d1, 0, None)))
        res.setdefault("fwd-shape GEMM x64", []).append(
            64 * timeit(lambda: gemm(eng.XH[: B * lay.KA], eng.Wp, B, lay.G, lay.KA, outH=eng.DG[: B * lay.G])))
    fl_fwd = 2.0 * B * lay.G * lay.KA * T
    fl_bwd = 2.0 * B * H * lay.G * (T - 1)
    fl_dw = 2.0 * B * T * lay.G * lay.KA
    for k, v in res.items():
        fl = fl_fwd if k.startswith("fwd") else fl_bwd if k.startswith("bwd") else fl_dw
        med = statistics.median(v)
        print(f"{k:16s} median {med:8.3f} ms  min {min(v):8.3f} ms  {fl / med / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
