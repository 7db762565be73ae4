#!/usr/bin/env python3
"""Host->device copy bandwidth: pinned vs pageable, sync vs async (feeds the streaming design)."""
import time

import torch

for mb in (4, 16, 64):
    n = mb * 1024 * 1024 // 4
    d = torch.empty(n, device="cuda")
    for kind in ("pageable", "pinned"):
        h = torch.randn(n)
        if kind == "pinned":
            h = h.pin_memory()
        for _ in range(3):
            d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        print(f"H2D {kind:8s} {mb:3d} MB: {mb / 1024 / dt:.1f} GB/s", flush=True)
