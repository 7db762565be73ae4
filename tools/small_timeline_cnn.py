"""Phase timeline of the persistent small-batch CNN launch (csrc/cnn_small.hip): s_memrealtime
(100 MHz) stamps at 11 phase boundaries of every step, thread 0 of each worker.

    python tools/small_timeline_cnn.py [B]   -> median microseconds per phase (steps 8..63)
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from wellflow.models.cnn import CNN1DRegressor, CnnLayout, NativeCNN  # noqa: E402
from wellflow.optim.flat import FlatSGD  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 20
K = 64
PH = ["stage x / y", "conv + ReLU + dropout", "dense share + publish", "poll, pred, dOut", "dWd", "dAct -> dP",
      "dWc", "SGD"]
dev = "cuda"
lay = CnnLayout()
eng = NativeCNN(lay, B, dev)
eng.params.copy_(CNN1DRegressor(lay.input_len, lay.in_ch, lay.filters, lay.kernel, lay.outputs).to_flat().to(dev))
eng.sync_weights()
opt = FlatSGD(eng.params, eng.grads, zero_grads=True, writeback=eng)
g = torch.Generator().manual_seed(1)
series = torch.randn(K * B, lay.input_len + lay.outputs, generator=g).cumsum(1) * 0.1
X, Y = series[:, : lay.input_len].contiguous().to(dev), series[:, lay.input_len:].contiguous().to(dev)
G = (lay.filters + 3) // 4
st = torch.zeros(28 * 64 * 16, dtype=torch.int64, device=dev)
for _ in range(3):
    eng.fused_steps(X, Y, B, K, opt, 1.0 / (B * 12))
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
eng.fused_steps(X, Y, B, K, opt, 1.0 / (B * 12), stamps=st)
ev1.record()
torch.cuda.synchronize()
eng.check_device_errors()
s = st.view(28, 64, 16)[:G].cpu().double() / 100.0
print(f"CNN B={B} K={K} G={G}: {ev0.elapsed_time(ev1) * 1000 / K:.2f} us per step (launch / K)")
per = [statistics.median(float(s[w, k + 1, 0] - s[w, k, 0]) for w in range(G)) for k in range(8, K - 1)]
print(f"step period (median over workers): {statistics.median(per):.2f} us")
for p in range(8):
    d = [float(s[w, k, p + 1] - s[w, k, p]) for w in range(G) for k in range(8, K)]
    print(f"  {PH[p]:<24} median {statistics.median(d):6.2f} us  max {max(d):6.2f}")
for name, a, b in (("hop 1 (own sums)", 3, 9), ("hop 2 poll", 9, 10), ("loss / dOut tail", 10, 4)):
    d = [float(s[w, k, b] - s[w, k, a]) for w in range(G) for k in range(8, K)]
    print(f"    of the poll: {name:<18} median {statistics.median(d):6.2f} us  max {max(d):6.2f}")
