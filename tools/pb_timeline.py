"""Per-row-tile timeline of the persistent backward (diagnostic build WELLFLOW_PF_DBG=32):
s_memrealtime stamps (100 MHz) of step 10, wave 0 of every workgroup, averaged."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from wellflow.data.synth import synth_lstm_batch  # noqa: E402
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402

B, H, F, T, NRT = 8192, 512, 16, 64, 16
eng = NativeLSTM(F, H, T, B, device="cuda")
eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
eng.sync_weights()
x, y = synth_lstm_batch(B, T, F, seed=2)
eng.forward_backward(x.cuda(), y.cuda(), 1.0 / B)
C, dims = eng._C, eng._dims(B)
w_out = eng.lay.views(eng.params)[1]
args = (eng.WhhT, eng.XH, eng.Cst, eng.S, eng.DG, eng.dcarry, eng.dy, w_out, *dims)
sync = torch.zeros(4096 + 2 * 128 * 256 + 64, dtype=torch.int32, device="cuda")  # + the STAT block
os.environ["WELLFLOW_PF_DBG"] = sys.argv[1] if len(sys.argv) > 1 else "32"
for _ in range(3):
    C.lstm_backward(*args, 8, sync)
torch.cuda.synchronize()
st = sync[4096:-64].view(torch.int64).view(256, 128).cpu().numpy().astype(np.float64) * 10.0  # ns
rel = (st - st[:, 0:1]) / 1000.0  # us from step start
print("step 10, us since step start (mean / max over 256 workgroups)")
print(f"{'handoff_done':16s} {rel[:, 1].mean():8.2f} {rel[:, 1].max():8.2f}")
t5 = rel[:, 2:2 + 5 * NRT].reshape(256, NRT, 5)
for k, nm in enumerate(("a_ready", "mfma_done", "barrier_done", "epi_start", "stored")):
    print(f"tile0 {nm:12s} {t5[:, 0, k].mean():8.2f}   tile15 {t5[:, NRT - 1, k].mean():8.2f}")
d = np.diff(t5[:, 1:, :], axis=2).mean(axis=(0, 1))
top = t5[:, :, 0]
print("per tile mean (t >= 1): mfma %.3f  exch+barrier %.3f  partial reads %.3f  epilogue+stores %.3f us" % tuple(d))
print("tile-to-tile (a_ready) mean %.3f us; stored -> next a_ready %.3f us" %
      (np.diff(top, axis=1).mean(), (t5[:, 1:, 0] - t5[:, :-1, 4]).mean()))
