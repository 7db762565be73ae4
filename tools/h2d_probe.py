#!/usr/bin/env python3
"""Host -> HBM copy rate of the online MLP's per-step payload (262,144 rows: 8.4 MB of bf16 x +
1 MB of fp32 y, pinned) issued on 1, 2 or 4 copy streams (the payload split evenly), to see
whether more than one DMA queue raises the PCIe rate the streamed bench is bound by.

    python tools/h2d_probe.py [--reps 200]
"""
import argparse

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda")
    nbytes = 262144 * 16 * 2 + 262144 * 4
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    for ns in (1, 2, 4, 1, 2, 4):
        streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
        cut = [nbytes * i // ns for i in range(ns + 1)]
        for _ in range(10):
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    dst[cut[i]:cut[i + 1]].copy_(src[cut[i]:cut[i + 1]], non_blocking=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            for i, s in enumerate(streams):
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    dst[cut[i]:cut[i + 1]].copy_(src[cut[i]:cut[i + 1]], non_blocking=True)
            for s in streams:
                torch.cuda.current_stream().wait_stream(s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print(f"streams {ns}: {ms * 1e3:.1f} us per {nbytes / 1e6:.2f} MB = {nbytes / ms / 1e6:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
