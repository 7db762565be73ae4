#!/usr/bin/env python3
"""Is a pinned host->device copy asynchronous for the host? Host time of one issue call
(torch copy_ non_blocking, raw hipMemcpyAsync, and a captured hipGraph replay) vs its device time."""
import ctypes
import time

import torch

n = 9 * 1024 * 1024 // 4
d = torch.empty(n, device="cuda")
hp = torch.randn(n).pin_memory()
s = torch.cuda.Stream()
torch.cuda.synchronize()


def host_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = 0.0
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        t += time.perf_counter() - a
        torch.cuda.synchronize()
    return 1e6 * t / reps


def tcopy():
    with torch.cuda.stream(s):
        d.copy_(hp, non_blocking=True)


print(f"torch copy_ non_blocking: host {host_time(tcopy):.1f} us per call", flush=True)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]


def raw():
    hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(hp.data_ptr()), d.numel() * 4, 1,
                       ctypes.c_void_p(s.cuda_stream))


print(f"hipMemcpyAsync H2D:       host {host_time(raw):.1f} us per call", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    d.copy_(hp, non_blocking=True)
print(f"graph replay (memcpy node): host {host_time(g.replay):.1f} us per call", flush=True)
torch.cuda.synchronize()
a = time.perf_counter()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
print(f"graph replay device-inclusive: {1e6 * (time.perf_counter() - a) / 20:.1f} us per copy "
      f"({n * 4 / 1e3 / (1e6 * (time.perf_counter() - a) / 20):.1f} GB/s)", flush=True)
