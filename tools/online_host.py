#!/usr/bin/env python3
"""Host-side cost of one streamed (online) MLP step: time spent in DeviceStreamer.next() and
StepRunner.run() per step, against the device step time (is the online path host-bound?)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from wellflow.data.stream import DeviceStreamer, HostPool  # noqa: E402
from wellflow.data.synth import synth_tabular_batch  # noqa: E402
from wellflow.models.mlp import NativeMLP, init_mlp_flat  # noqa: E402
from wellflow.optim.flat import FlatAdam  # noqa: E402
from wellflow.parallel.dist import DistContext  # noqa: E402
from wellflow.train.step import StepRunner  # noqa: E402

B, F = 262144, 16
ctx = DistContext.from_env()
eng = NativeMLP(F, (256, 256), B, device=ctx.device)
eng.params.copy_(init_mlp_flat(F, (256, 256), seed=0).to(ctx.device))
eng.sync_weights()
opt = FlatAdam(eng.params, eng.grads, lr=1e-3, shadow=eng.shadow, zero_grads=True)
pool = HostPool(lambda k: synth_tabular_batch(B, F, seed=k), n=8, x_dtype=torch.bfloat16)
st = DeviceStreamer(pool, ctx.device, depth=4)
run = StepRunner(eng, opt, ctx, 1.0 / B, lambda k: tuple(st.slots[k][:2]))
for _ in range(10):
    st.next()
    run.run(st.last_slot)
torch.cuda.synchronize()
N = 50
tn = tr = 0.0
t0 = time.perf_counter()
for _ in range(N):
    a = time.perf_counter()
    st.next()
    b = time.perf_counter()
    run.run(st.last_slot)
    tr += time.perf_counter() - b
    tn += b - a
host = time.perf_counter() - t0
torch.cuda.synchronize()
wall = time.perf_counter() - t0
print(f"per step: next() {1e3 * tn / N:.3f} ms, run() {1e3 * tr / N:.3f} ms, host loop {1e3 * host / N:.3f} ms, "
      f"wall {1e3 * wall / N:.3f} ms")

# where next() spends its host time: the pieces of one refill, timed one by one
xd, yd, _ = st.slots[0]
xs, ys = pool.batches[0]
parts = {"wait_event": 0.0, "copy x": 0.0, "copy y": 0.0, "record": 0.0}
ev = torch.cuda.Event()
for _ in range(N):
    run.run(st.last_slot)
    done = torch.cuda.Event()
    done.record()
    t = time.perf_counter()
    st.copy_stream.wait_event(done)
    t1 = time.perf_counter()
    with torch.cuda.stream(st.copy_stream):
        xd.copy_(xs, non_blocking=True)
        t2 = time.perf_counter()
        yd.copy_(ys, non_blocking=True)
        t3 = time.perf_counter()
        ev.record(st.copy_stream)
    t4 = time.perf_counter()
    for k, v in zip(parts, (t1 - t, t2 - t1, t3 - t2, t4 - t3)):
        parts[k] += v
    torch.cuda.current_stream().wait_event(ev)
torch.cuda.synchronize()
print("refill pieces (us per step):", {k: round(1e6 * v / N, 1) for k, v in parts.items()})
