"""Tracing / profiling hooks (SURVEY.md §5 "Tracing / profiling": the reference only had a
wall clock around fit, cnn.py:126-133).

* :func:`trace_range` — named ranges on the GPU timeline. On ROCm PyTorch builds the
  ``torch.cuda.nvtx`` entry points are backed by roctx, so the ranges show up in
  ``rocprofv3 --marker-trace`` / Perfetto next to the HIP kernels. Enabled by
  ``WELLFLOW_TRACE=1`` (zero cost otherwise).
* :class:`StepTimer` — device-event timing of named phases, aggregated per phase
  (used by tools and the trainer's ``--profile`` summaries).
* kernel-level evidence comes from ``rocprofv3 --kernel-trace --stats`` and ``--pmc``
  (tools/gpu.sh prof / pmc / pmcsets), summarised into profiles/.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict

import torch

_TRACE = os.environ.get("WELLFLOW_TRACE", "0") == "1"


@contextlib.contextmanager
def trace_range(name: str, device=None):
    if _TRACE and device is not None and torch.device(device).type == "cuda":
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


class StepTimer:
    """Accumulate per-phase device time with events (no host sync until ``summary``)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.events = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.cuda:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self.events[name].append((a, b))
        else:
            t0 = time.perf_counter()
            yield
            self.events[name].append(time.perf_counter() - t0)

    def summary(self) -> dict:
        if self.cuda:
            torch.cuda.synchronize(self.device)
        out = {}
        for k, v in self.events.items():
            ms = [a.elapsed_time(b) for a, b in v] if self.cuda else [1000.0 * x for x in v]
            out[k] = {"calls": len(ms), "total_ms": sum(ms), "mean_ms": sum(ms) / max(len(ms), 1)}
        return out
