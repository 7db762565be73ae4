#!/usr/bin/env python3
"""Does host idle time between bursts slow the next burst's steps? (the static MLP job's
kernels ran ~7 % slower than the bench's: profiles/r5/job2). Runs the bench's MLP step as
bursts of --burst steps (one graph replay of n steps each), with --idle-ms of host sleep between
bursts, and prints the device-timed rows/s of the bursts for each idle value.

    python tools/idle_gap_probe.py [--burst 36] [--idle 0,2,5,20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--burst", type=int, default=36)
    ap.add_argument("--idle", default="0,2,5,20")
    ap.add_argument("--bursts", type=int, default=12)
    a = ap.parse_args()
    import torch

    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.parallel.dist import DistContext
    from wellflow.train.step import StepRunner

    dev = torch.device("cuda")
    B, F = 262144, 16
    eng = NativeMLP(F, (256, 256), B, device=dev)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=0).to(dev))
    eng.sync_weights()
    opt = FlatAdam(eng.params, eng.grads, lr=1e-3, shadow=eng.shadow, zero_grads=True, shadow_t=eng.shadow_t)
    x, y = synth_tabular_batch(B, F, seed=0)
    x, y = x.to(dev, eng.input_dtype), y.to(dev)
    run = StepRunner(eng, opt, DistContext(device=dev), 1.0 / B, lambda k: (x, y))
    for _ in range(4):
        run.run()
    run.run_many(a.burst)
    torch.cuda.synchronize()
    for idle in [float(v) for v in a.idle.split(",")]:
        rates = []
        for _ in range(a.bursts):
            time.sleep(idle / 1e3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run.run_many(a.burst)
            e1.record()
            torch.cuda.synchronize()
            rates.append(a.burst * B / (e0.elapsed_time(e1) / 1e3))
        rates = rates[1:]
        print(f"idle {idle:5.1f} ms: burst rows/s mean {sum(rates) / len(rates) / 1e9:.4f} G, "
              f"min {min(rates) / 1e9:.4f}, max {max(rates) / 1e9:.4f}", flush=True)


if __name__ == "__main__":
    main()
