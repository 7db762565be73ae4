#!/usr/bin/env python3
"""Rows/s of the MLP training step (the bench's config: B = 262,144, F = 16, Adam with the
shadow writes, 8-step graph replays), event-timed, for A/Bs of WF_DIAG knobs that bench.py
refuses to load (a diagnostic build). One setting per process: the knobs are read once.

    WELLFLOW_MLP_PRIO128=0 python tools/mlp_step_rate.py [--steps 800]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=800)
    a = ap.parse_args()
    import torch

    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.parallel.dist import DistContext
    from wellflow.train.step import StepRunner

    dev = torch.device("cuda")
    B, F, n = 262144, 16, 8
    eng = NativeMLP(F, (256, 256), B, device=dev)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=0).to(dev))
    eng.sync_weights()
    opt = FlatAdam(eng.params, eng.grads, lr=1e-3, shadow=eng.shadow, zero_grads=True, shadow_t=eng.shadow_t)
    x, y = synth_tabular_batch(B, F, seed=0)
    x, y = x.to(dev, eng.input_dtype), y.to(dev)
    run = StepRunner(eng, opt, DistContext(device=dev), 1.0 / B, lambda k: (x, y))
    for _ in range(4):
        run.run()
    for _ in range(10):
        run.run_many(n)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps // n):
        run.run_many(n)
    e1.record()
    torch.cuda.synchronize()
    steps = a.steps // n * n
    print(f"rows_per_s {steps * B / (e0.elapsed_time(e1) / 1e3):.4e}", flush=True)


if __name__ == "__main__":
    main()
