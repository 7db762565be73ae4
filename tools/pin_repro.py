"""Does a pinned host allocation between persistent-LSTM launches make later launches exit
early? (Round-2 finding: pinned eval prefetch slots allocated between the epochs of a
graph-replayed job made the persistent kernels complete only part of their steps.)

Prints the running completion totals (csrc/persistent_guard.h) of the forward and backward for eager
launches and for hipGraph replays, before and after pinning host memory."""
import sys

import torch

sys.path.insert(0, ".")
from wellflow.data.synth import synth_lstm_batch  # noqa: E402
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402

B, T, F, H = 8192, 64, 16, 512
eng = NativeLSTM(F, H, T, B, device="cuda")
eng.params.copy_(init_lstm_flat(F, H, seed=0).cuda())
eng.sync_weights()
x, y = synth_lstm_batch(B, T, F, seed=0)
x, y = x.cuda(), y.cuda()


def counters(tag):
    torch.cuda.synchronize()
    st = eng.persistent_stats(); fw, bw = st["forward"], st["backward"]
    ok = fw["done"] == fw["expect"] and bw["done"] == bw["expect"]
    print(f"{tag:40s} fwd {fw['done']}/{fw['expect']} bwd {bw['done']}/{bw['expect']} sticky {fw['sticky']},{bw['sticky']} "
          f"-> {'ok' if ok else 'SHORT'} {fw['first_exit']} {bw['first_exit']}",
          flush=True)


eng.forward_backward(x, y, 1.0 / B)
counters("eager")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    eng.forward_backward(x, y, 1.0 / B)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    eng.forward_backward(x, y, 1.0 / B)
g.replay()
counters("graph replay")
pinned = [torch.empty(B * T * F, dtype=torch.float32).pin_memory() for _ in range(2)]
counters("after pinning (no launch)")
g.replay()
counters("graph replay after pinning")
eng.forward_backward(x, y, 1.0 / B)
counters("eager after pinning")
for p in pinned:
    p.cuda()  # a copy from the pinned buffers
g.replay()
counters("graph replay after pinned copies")
del pinned
g.replay()
counters("graph replay after freeing")

# the job's pattern: the native prefetcher filling pinned slots while the persistent forward
# (evaluation) runs, then the graph-replayed training step
import numpy as np  # noqa: E402

from wellflow.data import native  # noqa: E402

rows = np.random.default_rng(0).standard_normal((200000, F)).astype(np.float32)
starts = np.arange(0, 200000 - T, dtype=np.int64)
pf = native.Prefetcher(rows, starts, np.zeros(len(rows), np.float32), T, B, nslots=2, threads=2, pin=True)
rng = np.random.default_rng(1)
pf.submit(0, rng.integers(0, len(starts), B))
for k in range(4):
    pf.submit((k + 1) % 2, rng.integers(0, len(starts), B))
    xh, _ = pf.wait(k % 2)
    xb = xh.to("cuda")
    eng.forward(xb)
pf.wait(0)
pf.wait(1)
counters("eval forwards with the pinned prefetcher")
pf.close()
del pf
g.replay()
counters("graph replay after the pinned prefetcher")
g.replay()
counters("second replay")
eng.forward_backward(x, y, 1.0 / B)
counters("eager after the pinned prefetcher")
