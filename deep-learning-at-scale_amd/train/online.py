"""Dynamic (online) ANN training (Readme.md:19 "Dynamic model"; BASELINE.json:10 "Dynamic
(online) MLP with streaming mini-batches, DP=8").

The stream is the training data in ARRIVAL order (no epoch shuffle), cut into chunks of
``cfg.online_chunk`` rows that are consumed once each: every rank trains on its disjoint
slice of the chunk (one flat all-reduce per mini-batch), then the model is validated;
early stopping and best-model checkpointing act per chunk. Combined with the warm start
from the previous submission's ``.mdl`` (train/job.py) the model keeps adapting as new
well data arrives, which is what distinguishes it from the static model.
``cfg.epochs`` bounds the passes over the stream (default 1 for pure online learning
when the stream is long).
"""
from __future__ import annotations

import time

import torch

from .trainer import _to_dev


def stream_chunks(X, Y, chunk: int):
    for s in range(0, len(X), chunk):
        yield X[s : s + chunk], Y[s : s + chunk]


def fit_online(trainer, train, val):
    cfg, ctx, eng = trainer.cfg, trainer.ctx, trainer.eng
    Xtr, Ytr = train
    chunk = max(cfg.online_chunk, ctx.world_size)
    passes = max(1, cfg.epochs)
    done_chunks = int(trainer.extra_state.get("chunks_done", 0))
    k = 0
    for p in range(passes):
        for Xc, Yc in stream_chunks(Xtr, Ytr, chunk):
            if k < done_chunks:  # resume: skip chunks already consumed
                k += 1
                continue
            t0 = time.perf_counter()
            Xd, Yd = _to_dev(Xc, eng.device), _to_dev(Yc, eng.device)
            per_rank = len(Xd) // ctx.world_size
            order = torch.arange(ctx.rank * per_rank, (ctx.rank + 1) * per_rank, device=eng.device)
            b = max(1, min(cfg.batch_size, per_rank, getattr(eng, "B", cfg.batch_size)))
            tr_loss, rows, dt = trainer.train_steps(Xd, Yd, order, b)
            v_loss, v_mse = trainer.evaluate(*val)
            k += 1
            trainer.extra_state["chunks_done"] = k
            trainer.epoch += 1
            h = trainer.history
            h.loss.append(tr_loss)
            h.val_loss.append(v_loss)
            h.val_mse.append(v_mse)
            h.epoch_time.append(time.perf_counter() - t0)
            h.rows_per_s.append(rows / dt if dt > 0 else 0.0)
            if cfg.verbose >= 2:
                trainer.log(f"Chunk {k} (pass {p + 1}/{passes}) - {len(Xc)} rows - loss: {tr_loss:.6f}"
                            f" - val_loss: {v_loss:.6f} - rows/s: {h.rows_per_s[-1]:.0f}", flush=True)
            improved = v_loss < trainer.stopper.best
            trainer.stopper.update(v_loss)
            if improved and trainer.on_best is not None:
                ctx.barrier()
                if ctx.is_main:
                    trainer.on_best(trainer)
                ctx.barrier()
            trainer.save_state()
            if trainer.stopper.stopped or (cfg.max_steps and trainer.global_step >= cfg.max_steps):
                return trainer.history
    return trainer.history
