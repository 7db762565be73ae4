"""Per-term budget of the persistent LSTM forward (round-6 VERDICT item 1): time ONE
WELLFLOW_PF_DBG variant of lstm_fwd_persistent_kernel per process (a diagnostic build:
WELLFLOW_DIAG_BUILD=<set>), so a variant that faults is named by the process that ran it.

    python tools/pf_budget.py DBG [reps]      -> one line: "pf dbg<DBG> <median ms> <min ms>"

Variants (timing only, results garbage): 4 no C/S stores, 32 no A-fragment LDS reads,
8192 no cell math in the MFMA loop, 8224 = 8192 + 32, 131072 no LDS-DMA after step 0,
139296 = 131072 + 8224 (bare MFMAs + hand-off + stores), 139300 = that + no C/S stores.
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402

dbg = sys.argv[1] if len(sys.argv) > 1 else "0"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
os.environ["WELLFLOW_PF_DBG"] = dbg
B, H, F, T = 8192, 512, 16, 64
eng = NativeLSTM(F, H, T, B, device="cuda")
eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
eng.sync_weights()
x = torch.randn(B, T, F, device="cuda")
C, dims = eng._C, eng._dims(B)
C.lstm_pack_x(x, eng.XH, *dims, True)
print(f"pf dbg{dbg}: launching", flush=True)
assert C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *dims)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *dims)
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
st = eng.persistent_stats()["forward"]
print(f"pf dbg{dbg} {statistics.median(ts):.4f} {min(ts):.4f} ms  launches {st['launches']} "
      f"complete {st.get('complete')}", flush=True)
