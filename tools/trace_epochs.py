#!/usr/bin/env python3
"""Training-step spans per epoch from a rocprofv3 kernel trace of a job: consecutive runs of the
step's kernels (names matching --step, default the MLP step's four) separated by anything
else; per run: steps, span (first start -> last end), the sum of the kernels' own durations,
and the idle time inside the span (host launch latency, gaps between replays).

    python tools/trace_epochs.py run_kernel_trace.csv [--step mlp2_step128,mlp2_dw2g,mlp2_reduce,adam_dev]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", default="mlp2_step128,mlp2_dw2g,mlp2_reduce,adam_dev")
    a = ap.parse_args()
    keys = a.step.split(",")
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], []
    for r in rows:
        if any(k in r["Kernel_Name"] for k in keys):
            cur.append(r)
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    first = keys[0]
    for run in runs:
        steps = sum(1 for r in run if first in r["Kernel_Name"])
        t0, t1 = int(run[0]["Start_Timestamp"]), int(run[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in run)
        span = (t1 - t0) / 1e3
        print(f"steps {steps:4d}  span {span:9.1f} us  kernels {busy / 1e3:9.1f} us  idle {span - busy / 1e3:8.1f} us"
              f"  per step {span / max(steps, 1):7.1f} us")


if __name__ == "__main__":
    main()
