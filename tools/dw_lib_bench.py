"""Time the LSTM dW GEMM shape (M = 4H = 2048, N = KA = 576, K = T*B = 524288, bf16 in, fp32
accumulate) on our MFMA kernels vs the vendor library (hipBLASLt via torch.mm)."""
import sys
import torch

sys.path.insert(0, ".")
from wellflow.ops.native import gemm  # noqa: E402

M, N, K, KA = 2048, 576, 64 * 8192, 640
dG = torch.randn(K, M, device="cuda").to(torch.bfloat16)    # MN-contiguous A: dG[k, m]
XH = torch.randn(K, KA, device="cuda").to(torch.bfloat16)   # MN-contiguous B: XH[k, n]
out = torch.zeros(M, N, device="cuda")


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


for tile in (1, 3):
    for ks in (16, 32, 64):
        t = timeit(lambda: gemm(dG, XH, M, N, K, a_mn=True, lda=M, b_mn=True, ldb=KA, outF=out,
                                ldo=N, atomic=True, ksplit=ks, tile=tile))
        print(f"ours tile {tile} ks {ks}: {t:.3f} ms  {2 * M * N * K / t / 1e9:.0f} TF/s", flush=True)
A = dG.t()
Bv = XH[:, :N]
t = timeit(lambda: torch.mm(A, Bv))
print(f"torch.mm bf16->bf16: {t:.3f} ms  {2 * M * N * K / t / 1e9:.0f} TF/s", flush=True)
try:
    t = timeit(lambda: torch.ops.aten.mm.dtype(A, Bv, torch.float32))
    print(f"torch.mm bf16->fp32: {t:.3f} ms  {2 * M * N * K / t / 1e9:.0f} TF/s", flush=True)
except Exception as ex:  # noqa: BLE001
    print("mm.dtype unavailable:", ex)
At = dG.t().contiguous()
t = timeit(lambda: torch.mm(At, XH[:, :N]))
print(f"torch.mm bf16 (A row-major): {t:.3f} ms  {2 * M * N * K / t / 1e9:.0f} TF/s", flush=True)

# calibration: a large square bf16 GEMM through the vendor library
S = 8192
a = torch.randn(S, S, device="cuda").to(torch.bfloat16)
b = torch.randn(S, S, device="cuda").to(torch.bfloat16)
t = timeit(lambda: torch.mm(a, b))
print(f"torch.mm 8192^3 bf16: {t:.3f} ms  {2 * S ** 3 / t / 1e9:.0f} TF/s", flush=True)
o = torch.empty(S, S, device="cuda")
t = timeit(lambda: gemm(a, b, S, S, S, outF=o))
print(f"ours 8192^3 (K-contig A, B^T): {t:.3f} ms  {2 * S ** 3 / t / 1e9:.0f} TF/s", flush=True)
