"""Per-chunk timeline of the persistent forward (diagnostic build WELLFLOW_PF_DBG=16):
s_memrealtime stamps (100 MHz) of step 10 for every workgroup, averaged."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402

B, H, F, T = 8192, 512, 16, 64
eng = NativeLSTM(F, H, T, B, device="cuda")
eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
eng.sync_weights()
x = torch.randn(B, T, F, device="cuda")
C, dims = eng._C, eng._dims(B)
C.lstm_pack_x(x, eng.XH, *dims, True)
sync = torch.zeros(4096 + 2 * 64 * 256 + 64, dtype=torch.int32, device="cuda")  # + the STAT block
os.environ["WELLFLOW_PF_DBG"] = sys.argv[1] if len(sys.argv) > 1 else "16"
for _ in range(3):
    assert C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, sync, *dims)
torch.cuda.synchronize()
st = sync[4096:-64].view(torch.int64).view(256, 64).cpu().numpy().astype(np.float64) * 10.0  # ns
base = st[:, 0:1]
rel = (st - base) / 1000.0  # us from step start
names = ["sync_end"] + [f"c{c}_{k}" for c in range(8) for k in ("top", "after_wait", "mfma_done", "epi_done", "published")]
print("step 10, us since step start (mean / max over 256 workgroups)")
print(f"{'arrived':16s} {rel[:, 62].mean():8.2f} {rel[:, 62].max():8.2f}")
print(f"{'poll_matched':16s} {rel[:, 63].mean():8.2f} {rel[:, 63].max():8.2f}")
for i, nm in enumerate(names, start=1):
    print(f"{nm:16s} {rel[:, i].mean():8.2f} {rel[:, i].max():8.2f}")
d = np.diff(rel[:, 2:42].reshape(256, 8, 5)[:, 1:, :], axis=2).mean(axis=(0, 1))  # chunks >= 1
print("per chunk mean (c >= 1): wait %.2f  mfma %.2f  store %.2f  publish %.2f us" % tuple(d))
top = rel[:, 2:42:5]
print("chunk-to-chunk mean %.2f us" % np.diff(top, axis=1).mean())
kt = rel[:, 42:42 + 18]  # chunk 3: k-tile starts (after_wait .. mfma_done)
seg = np.diff(np.concatenate([kt, rel[:, 3 + 5 * 3 + 1:3 + 5 * 3 + 2]], axis=1), axis=1).mean(axis=0)
print("chunk 3 per k-tile (us):", " ".join("%.3f" % v for v in seg))
