#!/usr/bin/env python3
"""Host->device copy bandwidth for the streamed (online) model: pinned vs pageable, alone and
while the compute stream is busy, with and without NUMA binding (utils/numa.py).

    python tools/h2d_bw.py [--mb 9] [--bind]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def bw(d, h, reps=20, stream=None):
    s = stream or torch.cuda.current_stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(reps):
            d.copy_(h, non_blocking=True)
    s.synchronize()
    return d.numel() * d.element_size() / 1e9 / ((time.perf_counter() - t0) / reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=9)
    ap.add_argument("--bind", action="store_true", help="bind to the GPU's NUMA node first")
    a = ap.parse_args()
    if a.bind:
        from wellflow.utils.numa import bind_to_gpu_numa

        print("bound cpus:", len(bind_to_gpu_numa(0)))
    n = a.mb * 1024 * 1024 // 4
    d = torch.empty(n, device="cuda")
    h = torch.randn(n)
    print(f"H2D pageable {a.mb} MB: {bw(d, h):.1f} GB/s", flush=True)
    hp = h.pin_memory()
    print(f"H2D pinned   {a.mb} MB: {bw(d, hp):.1f} GB/s", flush=True)
    # the same copies on a side stream while the compute stream runs matmuls
    side = torch.cuda.Stream()
    x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    torch.cuda.synchronize()
    for _ in range(40):
        x @ x
    g = bw(d, hp, stream=side)
    torch.cuda.synchronize()
    print(f"H2D pinned   {a.mb} MB beside compute: {g:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
