"""NUMA-aware host placement for host -> HBM streaming (the dynamic/online model).

Pinned host buffers are first-touched by the allocating thread, so their pages land on that
thread's NUMA node. A DMA from pages on the socket that is NOT attached to the GPU's PCIe
root crosses the inter-socket link: measured on the MI355X box, the online MLP's per-step
9.4 MB batch copy ran at ~13 GB/s in some runs and ~45 GB/s in others (0.70 vs 0.45 ms per
step), depending only on where the process happened to be scheduled. Binding the process to
the CPUs local to its GPU before the pinned ring is allocated removes that lottery.

Only the sysfs PCI topology is used (no numactl / libnuma dependency); everything degrades to
a no-op when the information or the permission is missing.
"""
from __future__ import annotations

import os


def _parse_cpulist(text: str) -> set:
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def gpu_local_cpus(device_index: int) -> set:
    """CPUs on the NUMA node of GPU ``device_index`` (empty set if unknown)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        bus = getattr(p, "pci_bus_id", None)
        dom = getattr(p, "pci_domain_id", 0) or 0
        dev = getattr(p, "pci_device_id", 0) or 0
        if bus is None:
            return set()
        path = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dev:02x}.0/local_cpulist"
        with open(path) as f:
            return _parse_cpulist(f.read())
    except Exception:  # noqa: BLE001 - topology is an optimisation hint only
        return set()


def bind_to_gpu_numa(device_index: int) -> list:
    """Restrict this process to the CPUs local to its GPU (intersected with the CPUs it may
    already use). Returns the new CPU list, or [] when nothing was changed."""
    if os.environ.get("WELLFLOW_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return []
    local = gpu_local_cpus(device_index)
    if not local:
        return []
    allowed = os.sched_getaffinity(0)
    target = local & allowed
    if not target or target == allowed:
        return []
    try:
        os.sched_setaffinity(0, target)
    except OSError:
        return []
    return sorted(target)
