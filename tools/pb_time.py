"""Time the persistent LSTM backward (BPTT chain, steps T-1..0) against the per-step
kernels, with the timing-only diagnostic builds (WELLFLOW_PF_DBG, see
csrc/lstm_persistent_bwd.hip): 1 no hand-off wait, 2 no MFMA, 4 no DG stores,
8 no S/c loads, 16 no A loads."""
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
from wellflow.data.synth import synth_lstm_batch  # noqa: E402
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402


def timeit(fn, reps=5):
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


B, H, F, T = 8192, 512, 16, 64
eng = NativeLSTM(F, H, T, B, device="cuda")
eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
eng.sync_weights()
x, y = synth_lstm_batch(B, T, F, seed=2)
eng.forward_backward(x.cuda(), y.cuda(), 1.0 / B)
C, dims = eng._C, eng._dims(B)
w_out = eng.lay.views(eng.params)[1]
args = (eng.WhhT, eng.XH, eng.Cst, eng.S, eng.DG, eng.dcarry, eng.dy, w_out, *dims)
row = {"step v8": timeit(lambda: C.lstm_backward(*args, 8, None))}
ref = eng.DG.clone()
for dbg in os.environ.get("PB_CHECK", "0").split(","):  # correct builds must match the per-step kernels
    os.environ["WELLFLOW_PF_DBG"] = dbg
    eng.DG.zero_()
    C.lstm_backward(*args, 8, eng.sync_bwd)
    torch.cuda.synchronize()
    err = (eng.DG.float() - ref.float()).abs().max().item()
    print(f"check dbg{dbg}: max|dDG| {err:.3g} (scale {ref.float().abs().max().item():.3g}) "
          f"sticky word {int(eng.sync_bwd[-64].item())}", flush=True)
dbgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2", "4", "8", "16"]
# variants interleaved over several rounds (a fixed order biases toward the later ones:
# clocks and caches settle), median per variant
ts = {}
for rnd in range(int(os.environ.get("PB_ROUNDS", "3"))):
    for dbg in (dbgs if rnd % 2 == 0 else dbgs[::-1]):
        os.environ["WELLFLOW_PF_DBG"] = dbg
        ts.setdefault(f"pb dbg{dbg}", []).append(timeit(lambda: C.lstm_backward(*args, 8, eng.sync_bwd)))
os.environ["WELLFLOW_PF_DBG"] = "0"
for k, v in ts.items():
    row[k] = statistics.median(v)
print("bwd chain T=64 B=8192: " + "  ".join(f"{k} {v:.3f}ms" for k, v in row.items()), flush=True)
