#!/usr/bin/env python3
"""Headline benchmark: rows/sec (whole node) of LSTM seq-64 hidden-512 regression training.

BASELINE.json:2 / :11 — "LSTM seq-len=64 hidden=512 time-series regression, DP=8 bf16".
One row = one training sample (a 64-step window of well-log features and its flow
target). Each timed step is a FULL training step: forward over all 64 timesteps, MSE
loss, backward through time, RCCL gradient all-reduce (world > 1), fused Adam update and
the bf16 weight repack. Weak scaling: the per-GPU batch is fixed, global = per-GPU x N.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B_per_gpu]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8192, help="per-GPU batch (rows)")
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--features", type=int, default=16)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--dw-chunk", type=int, default=None, help="timesteps per overlapped dW chunk (0 = serial)")
    ap.add_argument("--fwd-variant", type=int, default=None)
    ap.add_argument("--bwd-variant", type=int, default=None)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.parallel.dist import DistContext

    ctx = DistContext.from_env()
    world, rank = ctx.world_size, ctx.rank
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = ctx.device
    torch.manual_seed(1234 + rank)

    B, T, F, H = args.batch, args.seq, args.features, args.hidden
    eng = NativeLSTM(F, H, T, B, device=dev)
    if args.dw_chunk is not None:
        eng.dw_chunk = args.dw_chunk
    if args.fwd_variant is not None:
        eng.fwd_variant = args.fwd_variant
    if args.bwd_variant is not None:
        eng.bwd_variant = args.bwd_variant
    eng.params.copy_(init_lstm_flat(F, H, seed=0).to(dev))
    ctx.broadcast_(eng.params)  # C1: identical init on every rank
    eng.sync_weights()
    opt = FlatAdam(eng.params, eng.grads, lr=args.lr)

    # synthetic well-log windows (Gilbert-consistent targets), resident on the GPU
    x, y = synth_lstm_batch(B, T, F, seed=rank)
    x, y = x.to(dev), y.to(dev)
    grad_scale = 1.0 / (B * world)

    def step():
        eng.forward_backward(x, y, grad_scale)
        ctx.all_reduce_sum_(eng.grads)  # C2: one flat bucket over RCCL / xGMI
        opt.step()
        eng.sync_weights()

    for _ in range(args.warmup):
        step()
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ctx.max_scalar(elapsed)
    loss = eng.loss_sum.item() / B

    ms = 1000.0 * elapsed / max(args.steps, 1)
    rows_per_s = B * world * args.steps / elapsed
    if rank == 0:
        rec = {
            "metric": "rows/sec (whole node), LSTM seq64 regression training",
            "value": round(rows_per_s, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (Gilbert-equation well-log windows, random-init weights)",
            "config": {
                "model": f"LSTM seq_len={T} hidden={H} features={F} -> linear head, MSE, Adam",
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": T,
                "parallelism": f"dp{world}",
            },
            "final_train_mse": round(loss, 6),
        }
        print(json.dumps(rec), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
