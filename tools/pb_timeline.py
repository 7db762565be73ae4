"""Per-row-tile timeline of the persistent backward (diagnostic build WELLFLOW_PF_DBG=32):
s_memrealtime stamps (100 MHz) of step 10, wave 0 of every workgroup, averaged.
Slots (csrc/lstm_persistent_bwd.inc.h): 0 step top, 1 slow-path wait entered (a group's poll
missed; absent when every poll matched), 2 + 5 RT + {0 A(RT) landed, 1 MFMAs done, 2 partials
written, 3 (last tile) partials summed, 4 tile end}."""
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
    sync[4096:-64].zero_()
    C.lstm_backward(*args, 8, sync)
torch.cuda.synchronize()
raw = sync[4096:-64].view(torch.int64).view(256, 128).cpu().numpy().astype(np.float64)
st = np.where(raw > 0, raw * 10.0, np.nan)  # ns; unset slots -> NaN
rel = (st - st[:, 0:1]) / 1000.0  # us from step start
print("step 10, us since step start (mean / max over 256 workgroups)")
slow = np.isfinite(rel[:, 1]).sum()
print(f"slow-path waits at step 10: {slow} of 256 workgroups")
t5 = rel[:, 2:2 + 5 * NRT].reshape(256, NRT, 5)
for k, nm in enumerate(("a_ready", "mfma_done", "written", "summed", "end")):
    print(f"tile0 {nm:10s} {np.nanmean(t5[:, 0, k]):8.2f}   tile15 {np.nanmean(t5[:, NRT - 1, k]):8.2f}")
top = t5[:, :, 0]
print("per tile mean: a_ready->mfma_done %.3f  mfma_done->written %.3f  end->next a_ready %.3f us" %
      (np.nanmean(t5[:, :, 1] - t5[:, :, 0]), np.nanmean(t5[:, :, 2] - t5[:, :, 1]),
       np.nanmean(t5[:, 1:, 0] - t5[:, :-1, 4])))
print("tile-to-tile (a_ready) mean %.3f us; step span (tile 0 a_ready -> tile 15 end) %.2f us" %
      (np.nanmean(np.diff(top, axis=1)), np.nanmean(t5[:, NRT - 1, 4] - t5[:, 0, 0])))
