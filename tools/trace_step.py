#!/usr/bin/env python3
"""Per-kernel duration and the idle gap before each kernel, from a rocprofv3 --kernel-trace
CSV (kernel_trace.csv), over the last --tail dispatches (the steady-state steps of a bench run).

    python tools/trace_step.py gpurun_out/.../run_kernel_trace.csv [--tail 400]

Kernels are grouped by name (first 60 characters); "gap" is the time between the previous
dispatch's end and this one's start on the same queue order (a hipGraph replay's launch
overhead and the drain / ramp between dependent kernels show up there).
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--tail", type=int, default=400)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.tail:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"][:60]
        dur[name].append(e - s)
        if prev_end is not None:
            gap[name].append(s - prev_end)
        prev_end = e
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"{len(rows)} dispatches over {span:.1f} us")
    print(f"{'kernel':60s} {'calls':>6s} {'mean us':>9s} {'gap us':>8s}")
    for name in sorted(dur, key=lambda n: -sum(dur[n])):
        d, g = dur[name], gap.get(name, [0])
        print(f"{name:60s} {len(d):6d} {sum(d) / len(d) / 1e3:9.2f} {sum(g) / max(len(g), 1) / 1e3:8.2f}")


if __name__ == "__main__":
    main()
