"""Time the persistent forward against the per-step forward, with diagnostic knobs."""
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
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


B, H, F = 8192, 512, 16
for T in (64,):
    eng = NativeLSTM(F, H, T, B, device="cuda")
    eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
    eng.sync_weights()
    x = torch.randn(B, T, F, device="cuda")
    C, dims = eng._C, eng._dims(B)
    C.lstm_pack_x(x, eng.XH, *dims, True)
    row = {}
    row["step v6"] = timeit(lambda: C.lstm_forward(eng.XH, eng.Wp, eng.Cst, eng.S, eng.dcarry, *dims, 6))
    for dbg in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("0", "1", "2", "4", "14")):
        os.environ["WELLFLOW_PF_DBG"] = dbg
        row[f"pf dbg{dbg}"] = timeit(lambda: C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *dims))
    os.environ["WELLFLOW_PF_DBG"] = "0"
    print(f"T={T}: " + "  ".join(f"{k} {v:.3f}ms" for k, v in row.items()), flush=True)
