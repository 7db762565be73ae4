"""One submitted learning job, end to end (the body of cnn.py, fixed and generalised).

    python3 <script>.py columnNames columnTypes targetColumn storagePath [dataPath] [--opts]

Flow: argv -> RunConfig -> DistContext (torchrun env; one process per
GPU; RCCL or gloo) -> table (CSV or synthetic) -> features (fit on train) -> engine
(native HIP engine on GPU in bf16, fp32 PyTorch oracle on CPU or with --precision fp32)
-> param broadcast (C1) -> fit (early stopping, best .mdl, resumable .ckpt) -> test
evaluation -> the reference's two stdout lines.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

from ..config import RunConfig, parse_argv
from ..data.pipeline import prepare
from ..data.schema import parse_schema
from ..models import registry
from ..models.gilbert import GilbertModel
from ..optim.flat import make_optimizer
from ..parallel.dist import DistContext
from ..utils import checkpoint as ckpt
from .trainer import Trainer


def _optimizer(cfg: RunConfig, eng):
    """The optimizer with the same launch fusions bench.py times: on a native engine the update
    also clears the gradient bucket (zero_grads), and it refreshes the engine's compute copies in
    the same launch — NativeLSTM / NativeCNN through their fused writebacks, NativeMLP through
    its bf16 shadow and the transposed W2 block — so no zero-fill or sync_weights launches run
    per step (without them the MLP job's step ran ~17 % slower on the device than the bench's)."""
    native = bool(getattr(eng, "native", False))
    if cfg.optimizer == "sgd":
        return make_optimizer("sgd", eng.params, eng.grads, lr=cfg.lr, momentum=cfg.momentum,
                              decay=cfg.decay, nesterov=cfg.nesterov, zero_grads=native,
                              writeback=eng if hasattr(eng, "fused_sgd") else None)
    kw = {}
    if hasattr(eng, "fused_adam"):
        kw["writeback"] = eng
    elif native and getattr(eng, "shadow", None) is not None and hasattr(eng, "shadow_t"):
        kw.update(shadow=eng.shadow, shadow_t=eng.shadow_t)  # NativeMLP
    return make_optimizer("adam", eng.params, eng.grads, lr=cfg.lr, weight_decay=cfg.weight_decay,
                          zero_grads=native, **kw)


def _save_best(cfg, name, ref, prepared):
    def cb(trainer):
        registry.engine_to_reference(trainer.eng, ref)
        extra = {"epoch": trainer.epoch, "val_loss": trainer.history.val_loss[-1],
                 "features": prepared.pipeline.state() if prepared.pipeline else None}
        ckpt.save_mdl(cfg.mdl_path(name), name, registry.keras_layers(name, ref), extra)
    return cb


def run_gilbert(cfg: RunConfig, ctx: DistContext, prepared, log):
    t0 = time.time()
    model = GilbertModel()
    feats, y = prepared.test
    test_mse = model.mse(feats, y)
    elapsed = time.time() - t0
    if ctx.is_main:
        A, B, C, unit = model.constants()
        ckpt.save_mdl(cfg.mdl_path("gilbert"), "gilbert",
                      [("Gilbert", [torch.tensor([A, B, C], dtype=torch.float64)])],
                      {"correlation": model.correlation, "glr_unit": unit})
        log("\nTime elapsed: %f s" % elapsed)
        log("Testing set loss: %f" % test_mse)
    return {"test_loss": test_mse, "test_mse": test_mse, "elapsed": elapsed}


AUTO_MIN_STEPS = 8  # an auto-sized batch still leaves >= 8 steps per epoch


def auto_batch(model: str, cfg: RunConfig, dev, n_rank: int) -> int:
    """``batch_size 0`` (auto, the default of lstm / mlp / mlp_online): the rows per GPU that
    fill the device — lstm: one co-resident persistent grid (NativeLSTM.full_grid_batch: 8192
    at H = 512 on 256 CUs), mlp / mlp_online: NativeMLP.full_batch (262,144) — capped so an
    epoch still has AUTO_MIN_STEPS steps on this rank's share of the training rows, in whole
    64-row tiles. It depends on the DEVICE only, never on --precision: the bf16 engine and the
    fp32 oracle of one job config train with the same batch (round-3 ADVICE). A CPU run takes
    256 (the reference's small-batch regime; cnn.py:128 used 20)."""
    if dev.type != "cuda":
        return 256
    if model == "lstm":
        from ..models.lstm import NativeLSTM

        fill = NativeLSTM.full_grid_batch(cfg.hidden, dev)
    elif model in ("mlp", "mlp_online"):
        from ..models.mlp import NativeMLP

        fill = NativeMLP.full_batch(dev)
    else:
        return 256
    b = min(fill, max(64, n_rank // AUTO_MIN_STEPS))
    return max(64, b - b % 64)


ONLINE_CHUNK_ROWS = 1 << 21  # auto stream chunk: rows per rank (the round-4 default: 8 x 262,144)
ONLINE_MIN_CHUNKS = 4        # ... but at least this many chunks (validation points) per pass
ONLINE_MIN_BATCHES = 32      # ... and at least this many mini-batches per chunk


def auto_online_chunk(batch: int, n_rank: int, world: int) -> int:
    """``online_chunk 0`` (auto): stream-chunk rows over ALL ranks, sized in ROWS, not in
    mini-batches (round-5 ADVICE): a chunk ends with a validation pass, a checkpoint and an
    early-stopping update (train/online.py), so at the job default batch of 256 a chunk of a few
    mini-batches would make validation I/O dominate and let patience=5 stop after ~40K rows.
    Per rank: ONLINE_CHUNK_ROWS, capped so a pass still has ONLINE_MIN_CHUNKS chunks, never
    under ONLINE_MIN_BATCHES mini-batches (a chunk's first replay and final sync are ~0.1 ms of
    host time the GPU waits out: 2 % of a 32-batch chunk of 262,144 rows), in whole batches."""
    batch = max(1, int(batch))
    per_rank = min(ONLINE_CHUNK_ROWS, max(1, n_rank // ONLINE_MIN_CHUNKS))
    per_rank = max(per_rank - per_rank % batch, ONLINE_MIN_BATCHES * batch)
    return per_rank * max(1, int(world))


def run_job(model: str, argv, log=print) -> dict:
    cfg = parse_argv(model, argv)
    return run_config(cfg, log=log)


def run_config(cfg: RunConfig, log=print) -> dict:
    device = None if cfg.device == "auto" else cfg.device
    ctx = DistContext.from_env(device=device, comm_dtype=cfg.comm_dtype)
    say = log if ctx.is_main else (lambda *a, **k: None)
    schema = parse_schema(cfg.column_names, cfg.column_types)
    say(schema)  # cnn.py:62
    say("Categorical variables: " + ", ".join(schema.categorical(exclude=(cfg.target,))))  # cnn.py:73
    prepared = prepare(cfg)
    if cfg.model == "gilbert":
        out = run_gilbert(cfg, ctx, prepared, say)
        ctx.shutdown()
        return out

    dev = ctx.device
    native = dev.type == "cuda" and cfg.precision == "bf16"
    n_train = len(prepared.train[0])
    n_rank = n_train // max(ctx.world_size, 1)
    if cfg.batch_size <= 0:
        cfg.batch_size = auto_batch(cfg.model, cfg, dev, n_rank)
        say(f"Batch size (auto): {cfg.batch_size} rows per GPU")
    if cfg.model == "mlp_online" and cfg.online_chunk <= 0:
        cfg.online_chunk = auto_online_chunk(cfg.batch_size, n_rank, ctx.world_size)
        say(f"Stream chunk (auto): {cfg.online_chunk} rows")
    b = max(1, min(cfg.batch_size, n_rank))
    if native and cfg.model == "lstm" and b >= 64:
        b -= b % 64  # the persistent kernels take batches in whole 64-row tiles
        cfg.batch_size = b  # the Trainer's per-rank batch (Trainer._local_batch) is then exactly b
    eng, ref = registry.build_engine(cfg.model, cfg, prepared.n_features, prepared.n_outputs, b,
                                     dev, native, seed=cfg.seed)
    ctx.broadcast_(eng.params)  # C1
    eng.sync_weights()
    opt = _optimizer(cfg, eng)
    trainer = Trainer(cfg, eng, opt, ctx, cfg.model, on_best=_save_best(cfg, cfg.model, ref, prepared),
                      n_outputs=prepared.n_outputs, log=log)
    resumed = trainer.try_resume()
    if cfg.model == "mlp_online":
        from .online import fit_online

        if not resumed:
            _warm_start(cfg, eng, ref, say)
        t0 = time.time()
        fit_online(trainer, prepared.train, prepared.val)
    else:
        t0 = time.time()
        trainer.fit(prepared.train, prepared.val)
    elapsed = time.time() - t0
    test_loss, test_mse = trainer.evaluate(*prepared.test)
    trainer.check_device()  # running completion totals cover every persistent launch of the job
    say("\nTime elapsed: %f s" % elapsed)  # cnn.py:133 (py3-correct)
    say("Testing set loss: %f" % test_loss)  # cnn.py:134
    result = {
        "model": cfg.model, "native": native, "world_size": ctx.world_size, "n_features": prepared.n_features,
        "epochs": trainer.epoch, "steps": trainer.global_step, "elapsed": elapsed,
        "test_loss": test_loss, "test_mse": test_mse,
        "best_val_loss": trainer.stopper.best, "history": trainer.history.__dict__,
    }
    if hasattr(eng, "persistent_stats"):  # csrc/persistent_guard.h totals (checked just above)
        result["persistent"] = {k: {kk: vv for kk, vv in v.items() if kk != "first_exit"}
                                for k, v in eng.persistent_stats().items()}
    if ctx.is_main and os.environ.get("WELLFLOW_RESULT_JSON"):
        with open(os.environ["WELLFLOW_RESULT_JSON"], "w") as f:
            json.dump(result, f)
    ctx.shutdown()
    return result


def _warm_start(cfg, eng, ref, say):
    """Dynamic model: continue from the last saved .mdl of this storage path if present."""
    path = cfg.mdl_path(cfg.model)
    if not os.path.exists(path):
        return
    try:
        name, layers, _ = ckpt.load_mdl(path)
        registry.load_keras_layers(cfg.model, ref, layers)
        registry.reference_to_engine(ref, eng)
        say(f"Warm start from {path}")
    except Exception as e:  # incompatible shapes (features changed between submissions)
        say(f"Warm start skipped ({e})")


def main(model: str) -> int:
    run_job(model, sys.argv[1:])
    return 0
