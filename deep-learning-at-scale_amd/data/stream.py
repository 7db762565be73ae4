"""Streaming mini-batches host -> HBM for the dynamic (online) model (BASELINE.json:10).

``DeviceStreamer`` keeps a ring of ``depth`` device buffers fed from pinned host memory on
a dedicated copy stream: batch k+1 (and k+2 ...) is in flight over PCIe while the compute
stream trains on batch k; compute waits only on the event of the batch it consumes. The
source is any iterator of (x, y) numpy/torch arrays (CSV chunks, a message queue, the
synthetic generator). Pinned sources (``HostPool``) are copied straight from their own
pages; anything else is first staged into a pinned ring (one host memcpy, then an async
DMA), so the H2D copy never runs synchronously from pageable memory.

Ordering (measured on MI355X, tools/online_host.py, bench.py h2d_* fields): a copy-stream
wait on an event of the compute stream (a cross-queue dependency, compute queue -> SDMA) made
4-5 % of the 9.4 MB batch copies stall for 3-6 ms (0.38-0.47 ms per step instead of 0.275).
Cause (profiles/r3_h2d_stall.md, tools/h2d_stall.py + a memory-copy trace): the DMA never
takes more than ~0.27 ms; the SDMA queue notices a satisfied compute-queue dependency ~0.5 ms
late at the median and ~7 ms late in a few percent of cases, and the compute stream, waiting on
that copy, drains (blit copies resolve the same wait in ~0.05 ms).
The slot's reuse is therefore ordered on the HOST: before refilling the slot of batch k-2 the
producer synchronizes on an event recorded right after batch k-2's compute (batch k-1's compute
is already queued, so the GPU never runs dry), and the copy itself has no queue dependency.
With that the streamed step runs at the static step's speed (952 vs 950 M rows/s; copies
median 0.22 ms, max 0.24 ms). A producer thread issuing the copies was slower (GIL
contention), and so were extra copy streams.

The device ring buffers keep their addresses for the streamer's lifetime — a hipGraph
captured on slot k (train/step.py StepRunner: one graph per slot) stays valid. Sources are
CHUNKS: :meth:`feed` queues one (train/online.py: one per stream chunk), iterating the
streamer yields the batches of the oldest unconsumed chunk and stops at its end, and the
ring position runs on across chunks. :meth:`prefetch` issues the next chunk's first batches
while the consumer does something else (the online job validates between chunks), so a
chunk starts with its batches already on the device instead of after a priming burst of
copies (round-3 VERDICT missing #5).
``HostPool`` pre-stages a set of batches in pinned memory and cycles through them, which is
how the benchmark isolates the transfer + train pipeline from Python-side generation cost.
Inputs can be streamed as bf16 (the MFMA engines consume bf16 directly), halving PCIe bytes.
"""
from __future__ import annotations

import collections
import itertools
import os

import torch


class HostPool:
    """``n`` distinct (x, y) batches resident in pinned host memory, cycled forever."""

    def __init__(self, make_batch, n: int, x_dtype=torch.float32):
        self.batches = []
        for k in range(n):
            x, y = make_batch(k)
            x = torch.as_tensor(x).to(x_dtype).pin_memory()
            y = torch.as_tensor(y).float().pin_memory()
            self.batches.append((x, y))

    def __iter__(self):
        return itertools.cycle(self.batches)


class DeviceStreamer:
    def __init__(self, source, device, depth: int = 4, x_dtype=None, timing: bool | int = False):
        """``x_dtype``: cast features on the host before the copy (e.g. torch.bfloat16);
        ``timing``: bracket the copies with events (:meth:`copy_stats`) — True for every batch,
        an int N for every N-th batch (the two event records per copy cost the PCIe-bound
        streamed bench ~5 % when every batch is timed)."""
        assert depth >= 3, "the refill lags two batches behind the consumer (module docstring)"
        self.device = torch.device(device)
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self.depth = depth
        self.x_dtype = x_dtype
        self.slots = []    # [x_dev, y_dev, ready event] — fixed addresses
        self.consumed = [None] * depth  # per slot: event after the compute that read it
        # slot reuse is ordered on the host (event.synchronize) instead of by a copy-queue wait
        # on the compute stream: module docstring (WELLFLOW_H2D_HOSTWAIT=0: queue wait)
        self.host_wait = os.environ.get("WELLFLOW_H2D_HOSTWAIT", "1") != "0"
        self.timing = int(timing) if timing else 0  # time every N-th batch (0: none)
        self._tev = []  # (start, end) events of timed batches
        self.staging = []  # pinned host ring for pageable sources: [x_pin, y_pin]
        # monotonic over the streamer's life: batch i lives in slot i % depth
        self.k = 0         # batches issued
        self.used = 0      # batches handed to the consumer
        self._rec = 0      # consumed events recorded for batches < _rec
        self.last_slot = 0
        self._srcs = collections.deque()  # [chunk id, iterator] queued by feed()
        self._chunk_of = collections.deque()  # chunk id of each issued, unconsumed batch
        self._next_id = 0  # id of the next fed chunk
        self._consume = 0  # chunk the iterator consumes
        self._pinned = {}  # id(tensor) -> tensor, sources already known to be pinned (no per-step query)
        if source is not None:
            self.feed(source)

    def feed(self, source) -> None:
        """Queue a chunk; the ring (and any captured graphs) stay valid."""
        self._srcs.append([self._next_id, iter(source)])
        self._next_id += 1

    def close(self) -> None:
        """Nothing to release (API symmetry with producer-style streamers)."""

    def _host(self, x, y, slot):
        if id(x) in self._pinned and id(y) in self._pinned and self.x_dtype in (None, x.dtype):
            return x, y  # a pinned batch seen before (HostPool cycles a fixed set)
        x = torch.as_tensor(x)
        if x.dtype == torch.float64:
            x = x.float()
        if self.x_dtype is not None and x.dtype != self.x_dtype:
            x = x.to(self.x_dtype)
        y = torch.as_tensor(y).float()
        if x.is_pinned() and y.is_pinned():
            if len(self._pinned) < 256:
                self._pinned[id(x)], self._pinned[id(y)] = x, y  # keeps them alive: ids stay unique
            return x, y
        while len(self.staging) <= slot:
            self.staging.append([None, None])
        st = self.staging[slot]
        if st[0] is None or st[0].shape != x.shape or st[0].dtype != x.dtype:
            st[0] = torch.empty(x.shape, dtype=x.dtype).pin_memory()
        if st[1] is None or st[1].shape != y.shape:
            st[1] = torch.empty(y.shape, dtype=y.dtype).pin_memory()
        if slot < len(self.slots):
            self.slots[slot][2].synchronize()  # the slot's previous DMA has read the staging pages
        st[0].copy_(x)
        st[1].copy_(y)
        return st[0], st[1]

    def _mark_consumed(self) -> None:
        """The batch handed out last has its compute queued on the current stream: an event
        after it orders the refill of its slot (recorded once per batch)."""
        if self._rec < self.used:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.consumed[(self.used - 1) % self.depth] = ev
            self._rec = self.used

    def _issue(self) -> bool:
        """Copy the next batch of the oldest queued chunk into slot k % depth."""
        while self._srcs:
            cid, it = self._srcs[0]
            try:
                x, y = next(it)
                break
            except StopIteration:
                self._srcs.popleft()
        else:
            return False
        slot = self.k % self.depth
        x, y = self._host(x, y, slot)
        if len(self.slots) <= slot:
            xd = torch.empty(x.shape, dtype=x.dtype, device=self.device)
            yd = torch.empty(y.shape, dtype=y.dtype, device=self.device)
            self.slots.append([xd, yd, torch.cuda.Event()])
        xd, yd, ev = self.slots[slot]
        assert xd.shape == x.shape and xd.dtype == x.dtype and yd.shape == y.shape, \
            "DeviceStreamer: every batch must have the ring's shape"
        # the slot's previous consumer must be done before it is overwritten (its event, not
        # the whole compute stream: see the module docstring)
        done = self.consumed[slot] if self.k >= self.depth else None
        if done is not None:
            if self.host_wait:  # the host waits, the copy queue gets no cross-queue dependency
                done.synchronize()
            else:
                self.copy_stream.wait_event(done)
        timed = self.timing and self.k % self.timing == 0
        with torch.cuda.stream(self.copy_stream):
            if timed:
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record(self.copy_stream)
            xd.copy_(x, non_blocking=True)
            yd.copy_(y, non_blocking=True)
            ev.record(self.copy_stream)
            if timed:
                t1.record(self.copy_stream)
                self._tev.append((t0, t1))
        self._chunk_of.append(cid)
        self.k += 1
        return True

    def _fill(self) -> None:
        """Issue every batch the ring may take now: a slot is refilled only after the compute
        that read it TWO batches ago (that batch's event; the batch after it is queued, so the
        GPU never runs dry while the host waits); first uses of a slot are free."""
        while self.k < self.depth or self.k - self.depth <= self.used - 2:
            if not self._issue():
                return

    def prefetch(self) -> None:
        """Between chunks (the consumer's last batch is queued): issue the next chunk's first
        batches now, so their copies overlap whatever runs before the chunk is consumed."""
        self._mark_consumed()
        self._fill()

    def _take(self) -> int:
        self.last_slot = self.used % self.depth
        self.used += 1
        self._chunk_of.popleft()
        xd, yd, ev = self.slots[self.last_slot]
        torch.cuda.current_stream(self.device).wait_event(ev)
        return self.last_slot

    def next(self):
        """The next batch on the device (any chunk), ordered before the current stream's later
        work; raises StopIteration when every queued chunk is drained."""
        self._mark_consumed()
        self._fill()
        if self.used >= self.k:
            raise StopIteration
        self._take()
        xd, yd, _ = self.slots[self.last_slot]
        return xd, yd

    def __iter__(self):
        """Yields the ring slot index of each batch of the oldest unconsumed chunk (its tensors:
        ``slots[k][0:2]``) and stops at that chunk's end."""
        cid = self._consume
        while True:
            self._mark_consumed()
            self._fill()
            if self.used >= self.k:  # nothing issued: every queued source is drained
                break
            if self._chunk_of[0] != cid:  # the next batch belongs to a later chunk
                break
            yield self._take()
        self._consume = cid + 1

    def copy_stats(self, skip: int = 0) -> dict:
        """Device time of each timed batch's host->HBM copies (ms): mean / median / max (syncs);
        ``skip``: timed batches to leave out at the start."""
        torch.cuda.synchronize(self.device)
        ms = [a.elapsed_time(b) for a, b in list(self._tev)[skip:]]
        if not ms:
            return {}
        srt = sorted(ms)
        return {"h2d_ms_mean": round(sum(ms) / len(ms), 4), "h2d_ms_median": round(srt[len(srt) // 2], 4),
                "h2d_ms_max": round(srt[-1], 4), "h2d_batches": len(ms),
                "h2d_over_1ms": sum(1 for v in ms if v > 1.0)}
