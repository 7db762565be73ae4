"""Phase timeline of the persistent small-batch MLP launch (csrc/mlp_small.hip): s_memrealtime
(100 MHz) stamps at 14 phase boundaries of every step, thread 0 of each of the 16 workers.

    python tools/small_timeline.py [B] [F]   -> median microseconds per phase (steps 8..63)
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from wellflow.data.synth import synth_tabular_batch  # noqa: E402
from wellflow.models.mlp import NativeMLP, init_mlp_flat  # noqa: E402
from wellflow.optim.flat import FlatAdam  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
F = int(sys.argv[2]) if len(sys.argv) > 2 else 16
K = 64
PH = ["W1 poll + stage X", "H1", "layer 2 + partials", "(no barrier)", "partial poll, pred, dy",
      "dZ2 + publish", "dW2, W2 Adam + image", "barrier rest", "dH1 + dZ1", "dW1", "W1/b1/b3 Adam",
      "W1 granules", "(no barrier)"]
dev = "cuda"
eng = NativeMLP(F, (256, 256), B, device=dev)
eng.params.copy_(init_mlp_flat(F, (256, 256), seed=1).to(dev))
eng.sync_weights()
opt = FlatAdam(eng.params, eng.grads, lr=1e-3, shadow=eng.shadow, zero_grads=True, shadow_t=eng.shadow_t)
X, Y = synth_tabular_batch(K * B, F, seed=2)
X, Y = X.to(dev).to(torch.bfloat16), Y.to(dev)
st = torch.zeros(16 * 64 * 16, dtype=torch.int64, device=dev)
for _ in range(3):
    eng.fused_steps(X, Y, B, K, opt, 1.0 / B)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
eng.fused_steps(X, Y, B, K, opt, 1.0 / B, stamps=st)
ev1.record()
torch.cuda.synchronize()
eng.check_device_errors()
s = st.view(16, 64, 16).cpu().double() / 100.0  # microseconds
print(f"B={B} F={F} K={K}: {ev0.elapsed_time(ev1) * 1000 / K:.2f} us per step (launch / K)")
steps = range(8, K)
per_step = [statistics.median(float(s[w, k + 1, 0] - s[w, k, 0]) for w in range(16)) for k in range(8, K - 1)]
print(f"step period (stamp 0 to next stamp 0, median over workers): {statistics.median(per_step):.2f} us")
for p in range(13):
    d = [float(s[w, k, p + 1] - s[w, k, p]) for w in range(16) for k in steps]
    print(f"  {PH[p]:<20} median {statistics.median(d):6.2f} us  max {max(d):6.2f}")
d = [float(s[w, k, 14] - s[w, k, 1]) for w in range(16) for k in steps]
print(f"  (of H1: the next batch's prefetch issue {statistics.median(d):.2f} us)")
