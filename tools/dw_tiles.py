"""A/B of the LSTM weight-gradient tiles on the bench shape (M = 4H = 2048, N = KA = 576,
K = T*B = 524288, MN x MN operands, split-K fp32 atomics): time per call, interleaved over
rounds, and max |diff| against the default tile (3 = 256x192 64-deep 2-stage).

    python tools/dw_tiles.py [tiles ...]      (default: 1 2 3; 4 / 5 = 256x192 with the 5- / 4-slot
                                              32-deep half-step ring; 7 = the production 256x288,
                                              8 = 256x288 with global_load_lds instead of MUBUF
                                              LDS-DMA; 9 / 10 = diagnostics of 7, results wrong:
                                              DMA every other half step / DMA + barriers only, no
                                              fragment reads or MFMAs; 11 = 7 with the DMA pieces
                                              between the MFMAs; DW_KS=16,32 picks the
                                              split-K depths)
"""
import sys

import torch

sys.path.insert(0, ".")
from wellflow.ops.native import gemm  # noqa: E402

M, N, K, KA = 2048, 576, 64 * 8192, 640
tiles = [int(a) for a in sys.argv[1:]] or [1, 2, 3]
torch.manual_seed(0)
dG = (torch.randn(K, M, device="cuda") * 0.1).to(torch.bfloat16)
XH = torch.randn(K, KA, device="cuda").to(torch.bfloat16)
outs = {}


def run(tile, ks):
    out = outs.setdefault((tile, ks), torch.zeros(M, N, device="cuda"))
    out.zero_()
    gemm(dG, XH, M, N, K, a_mn=True, lda=M, b_mn=True, ldb=KA, outF=out, ldo=N, atomic=True,
         ksplit=ks, tile=tile)
    return out


def timeit(fn, n=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


ref = run(3, 32).clone()
torch.cuda.synchronize()
import os  # noqa: E402

cfgs = [(t, ks) for t in tiles for ks in (int(k) for k in os.environ.get("DW_KS", "16,32,64").split(","))]
for c in cfgs:  # warm-up + correctness
    d = (run(*c) - ref).abs().max().item()
    print(f"tile {c[0]} ks {c[1]}: max|diff| vs tile 3 = {d:.3e} (ref max {ref.abs().max().item():.2f})", flush=True)
best = {c: 1e9 for c in cfgs}
for r in range(4):
    for c in cfgs:
        best[c] = min(best[c], timeit(lambda: run(*c)))
for c in cfgs:
    t = best[c]
    print(f"tile {c[0]} ks {c[1]}: {t:.3f} ms  {2 * M * N * K / t / 1e9:.0f} TF/s", flush=True)
