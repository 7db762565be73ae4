#!/usr/bin/env python3
"""Where does the round-2 H2D stall come from? (data/stream.py docstring)

The streamed online step used a copy stream whose refill of a ring slot WAITED on an event of
the compute stream (a cross-queue dependency) and 4-5 % of the 9.4 MB copies then took 3-6 ms.
This isolates the pattern: the compute stream runs a steady ~0.3 ms step (bf16 GEMMs), the copy
stream refills slot k after the compute of batch k-2. For every copy it records, on the GPU
timeline (events with timing):

  dep   = the compute event the copy depends on (recorded after batch k-2's compute)
  start = an event on the copy stream right after its wait (= the copy may start)
  end   = an event after the copy

and reports the distributions of start - dep (how late the copy queue notices its
dependency), end - start (the copy itself) and the host-side issue time. ``--mode host``
is the shipped ordering (the host syncs on dep, the copy has no queue dependency).

    python tools/h2d_stall.py --mode queue|host [--iters 300] [--mb 9.4] [--out file.json]
"""
import argparse
import json
import time

import torch


def pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(q * len(s)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["queue", "host"], default="queue")
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--mb", type=float, default=9.4)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    comp = torch.cuda.current_stream(dev)
    cstream = torch.cuda.Stream(device=dev)
    n = int(a.mb * 1e6 / 2)
    host = [torch.randn(n).to(torch.bfloat16).pin_memory() for _ in range(a.depth)]
    slots = [torch.empty(n, dtype=torch.bfloat16, device=dev) for _ in range(a.depth)]
    A = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    Bm = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    C = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)

    def step(k):  # ~0.3 ms of compute reading slot k
        torch.mm(A, Bm, out=C)
        C[:1, :1].add_(slots[k % a.depth][:1].view(1, 1))

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    consumed = [None] * a.depth
    ready = [None] * a.depth
    recs = []
    issue_us = []

    def refill(k, dep):
        s = k % a.depth
        t0 = time.perf_counter()
        if dep is not None:
            if a.mode == "host":
                dep.synchronize()
            else:
                cstream.wait_event(dep)
        st, en = ev(), ev()
        with torch.cuda.stream(cstream):
            st.record(cstream)
            slots[s].copy_(host[s], non_blocking=True)
            en.record(cstream)
            r = torch.cuda.Event()
            r.record(cstream)
        ready[s] = r
        issue_us.append((time.perf_counter() - t0) * 1e6)
        recs.append((dep, st, en))

    for k in range(a.depth):
        refill(k, None)
    for k in range(a.iters):
        s = k % a.depth
        comp.wait_event(ready[s])
        step(k)
        d = ev()
        d.record(comp)
        consumed[s] = d
        if k >= 1:  # refill the slot of batch k - 1 + depth... lag: the slot consumed by batch k-1
            kk = k - 1 + a.depth
            refill(kk, consumed[(k - 1) % a.depth])
    torch.cuda.synchronize()
    lag, dur = [], []
    for dep, st, en in recs:
        if dep is None:
            continue
        lag.append(dep.elapsed_time(st))
        dur.append(st.elapsed_time(en))
    out = {"mode": a.mode, "iters": a.iters, "mb": a.mb,
           "lag_ms": {"median": pct(lag, 0.5), "p95": pct(lag, 0.95), "max": max(lag), "over_1ms": sum(v > 1 for v in lag)},
           "copy_ms": {"median": pct(dur, 0.5), "p95": pct(dur, 0.95), "max": max(dur), "over_1ms": sum(v > 1 for v in dur)},
           "host_issue_us": {"median": pct(issue_us, 0.5), "max": max(issue_us)}}
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({**out, "lag_ms_all": lag, "copy_ms_all": dur}, f)


if __name__ == "__main__":
    main()
