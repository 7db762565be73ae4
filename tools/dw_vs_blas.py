#!/usr/bin/env python3
"""LSTM weight-gradient GEMM (M = 4H = 2048, N = KA = 576, K = T*B = 524288, bf16 -> fp32):
the hand-written split-K MFMA kernel (csrc/gemm.hip gemm_dw_kernel) against the library GEMM
(torch.mm with out_dtype=float32 -> hipBLASLt), same operands, and their agreement."""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from wellflow.ops.native import gemm  # noqa: E402

T, B, H, KA = 64, 8192, 512, 576
G = 4 * H
K = T * B
torch.manual_seed(0)
DG = (torch.randn(K, G, device="cuda") * 0.01).to(torch.bfloat16)
XH = torch.randn(K + B, KA, device="cuda").to(torch.bfloat16)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


out_k = torch.zeros(G, KA, device="cuda")


def native():
    out_k.zero_()
    gemm(DG, XH, G, KA, K, a_mn=True, lda=G, b_mn=True, ldb=KA, outF=out_k, atomic=True, ksplit=32, tile=3)


out_b = torch.empty(G, KA, device="cuda")


def blas():
    torch.mm(DG.t(), XH[:K], out_dtype=torch.float32, out=out_b)


tn = timeit(native)
try:
    tb = timeit(blas)
    err = ((out_k - out_b).norm() / out_b.norm()).item()
except Exception as e:  # noqa: BLE001
    tb, err = float("nan"), repr(e)
flop = 2.0 * G * KA * K
print(f"native split-K MFMA: {tn:.3f} ms ({flop / tn / 1e9:.0f} TFLOP/s) | hipBLASLt torch.mm: {tb:.3f} ms "
      f"({flop / tb / 1e9:.0f} TFLOP/s) | rel diff {err}", flush=True)
