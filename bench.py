#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): rows/sec (whole node) of LSTM seq-64 hidden-512
time-series regression training, DP over 1/2/4/8 MI355X, bf16.

One row = one training sample (a 64-step window of well-log features and its flow target).
Every timed step is a FULL training step: forward over all 64 timesteps, MSE loss,
backward through time, weight gradients, RCCL gradient all-reduce (world > 1), fused Adam
update and the bf16 weight repack. Weak scaling: per-GPU batch fixed, global = per-GPU x N.
The step is the production one (wellflow/train/step.py StepRunner, also driven by the
job's Trainer): after two eager steps it replays as ONE hipGraph per step, the RCCL
all-reduce captured inside it.

Secondary configs (BASELINE.json:8-10), same JSON contract:
  --model mlp         static 3-layer MLP (F -> 256 -> 256 -> 1), resident batch
  --model mlp_online  dynamic MLP: every step trains on a NEW mini-batch streamed host -> HBM
  --model cnn         the reference's own 1-D CNN (cnn.py:110-118), SGD-Nesterov, 65,536 windows
The default invocation times all three AFTER the headline's timed region, then the same
models at the submission API's own batches (cnn_b20, mlp_b256, mlp_online_b256: CNN 20
windows, MLP / online MLP 256 rows; one-GPU runs only, by default: the K-steps-per-launch
paths), and reports them
in a nested "secondary" object of the same JSON line (each with its own steps, ms/step,
rows/s, timed seconds); the headline "value" is the LSTM alone.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B_per_gpu] [--model ...]

With --gpus N > 1 and no torchrun environment, this process (which never touches the GPU)
starts `torch.distributed.run --nproc-per-node N` on itself and exits with its status; under
torchrun (WORLD_SIZE set) every rank runs the benchmark and rank 0 prints the JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "rows/sec (whole node), LSTM seq64 regression at 1/2/4/8 MI355X; val MSE parity"
# per-GPU rows per step. MLP: 262144 rows (bf16 activations ~270 MB of 288 GB HBM) — at
# 65536 the 0.24 ms step is launch/stream-overhead bound (216-272 M rows/s vs 382 M here)
DEFAULT_BATCH = {"lstm": 8192, "mlp": 262144, "mlp_online": 262144, "cnn": 65536}


# Timing-only / test-hook variables: a production _C.so ignores the first two (csrc/
# persistent_guard.h kDbgMask, mlp_fused.hip kMlpDbgMask), the test hooks make a run fail; the
# bench refuses all of them so no number is ever taken with one set (round-3 VERDICT item 2).
DIAG_ENV = ("WELLFLOW_PF_DBG", "WELLFLOW_MLP_DBG", "WELLFLOW_FORCE_TIMEOUT", "WELLFLOW_SPIN_LIMIT",
            "WELLFLOW_DIAG_BUILD")
ENV_PREFIXES = ("WELLFLOW_", "HSA_", "HIP_", "NCCL_", "RCCL_", "GPU_MAX_", "ROCR_", "AMD_", "TORCH_NCCL_")


def _diag_env() -> dict:
    return {k: os.environ[k] for k in DIAG_ENV if os.environ.get(k, "") not in ("", "0")}


def _env_record() -> dict:
    """Every tuning / runtime variable this process saw (WELLFLOW_* knobs, HSA / HIP / RCCL
    settings), so the JSON line says exactly what configuration produced the number."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(ENV_PREFIXES)}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn_ranks(n: int, argv) -> int:
    """Launcher mode: N ranks on this node via torch.distributed.run (127.0.0.1 rendezvous).
    The parent imports nothing GPU-related; each child pins its own GPU (LOCAL_RANK)."""
    env = dict(os.environ)
    # dmabuf IPC: the MI355X hosts of this pool support only dmabuf IPC, and without it RCCL's
    # and torch's cross-process GPU memory sharing fails with hipIpcGetMemHandle: invalid
    # argument. The pool exports it already (then setdefault changes nothing); the JSON line
    # reports the value the ranks ran with.
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__), *argv]
    return subprocess.run(cmd, env=env, cwd=ROOT).returncode


_LAST_TIMED = {"untimed": 0}  # steps the last _timed() ran outside its window (warm-up, probe, captures)
_SAMPLER = {}  # "s": this rank's GpuStateSampler (GPU runs), bracketing every timed window


def _timed(ctx, step, steps, warmup, min_s: float = 0.0, many=None, graph_steps: int = 1, warm_ms: float = 25.0):
    """W untimed warmup steps, then EXACTLY `steps` timed steps bracketed by barrier +
    synchronize on both sides; the max over ranks. With min_s > 0 (the secondary configs) a
    short untimed probe first raises `steps` until the timed window is >= min_s on the slowest
    rank, so one hiccup of tens of microseconds is not a percent of the number (round-3 VERDICT
    weak #5). ``many(n)`` (StepRunner.run_many): the timed steps run as replays of one
    ``graph_steps``-step graph (every step complete, the remainder as single steps).
    Returns (seconds, timed steps, total steps run)."""
    import math

    import torch

    def sync():
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(warmup):
        step()
    total = warmup
    per = None  # seconds per step, from the probe (secondaries)
    if min_s > 0:
        probe = 20
        ctx.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(probe):
            step()
        sync()
        ctx.barrier()
        per = ctx.max_scalar(time.perf_counter() - t0) / probe
        total += probe
        # 1.5x margin: the probe's per-step estimate carries its own sync overhead and the
        # streamed config varies step to step (round 4: 1.1x left 0.079-0.098 s windows)
        steps = max(steps, int(math.ceil(min_s * 1.5 / max(per, 1e-9))))
    n = graph_steps if many is not None and graph_steps > 1 else 1
    if min_s > 0 and n > 1:  # a secondary's raised window: whole replays / launches only
        steps = -(-steps // n) * n
    if n > 1:
        many(n)  # capture (untimed) + one n-step replay of warmup
        total += n
        # the capture leaves the GPU idle for a while and its clock ramps down (an 8-step MLP replay
        # after 10 ms idle runs ~14 % slow: tools/idle_gap_probe.py); more untimed replays, ~warm_ms
        # of steps, bring it back before the window opens (the line reports them: untimed_steps)
        if per is None:
            sync()
            t1 = time.perf_counter()
            many(n)
            sync()
            per = ctx.max_scalar(time.perf_counter() - t1) / n
            total += n
        extra = int(math.ceil(warm_ms / 1e3 / (n * per))) if (per and warm_ms > 0) else 0
        for _ in range(min(extra, 64)):
            many(n)
            total += n
    smp = _SAMPLER.get("s")
    if smp is not None:
        smp.start()  # a sysfs read + a sleeping thread: nothing on the GPU's queues
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps // n):
        many(n) if n > 1 else step()
    for _ in range(steps % n):
        step()
    sync()
    ctx.barrier()
    el = time.perf_counter() - t0
    _LAST_TIMED["untimed"] = total
    _LAST_TIMED["gpu_state"] = smp.stop() if smp is not None else None
    return ctx.max_scalar(el), steps, total + steps


def _comm_ms(ctx, buf, iters: int = 20) -> float | None:
    """Timed C2 (the flat gradient all-reduce of ``buf``, in the run's comm dtype) at this world
    size, outside the step (inside the step it is one node of the captured graph): HIP events
    on a GPU, the host clock on the CPU (gloo rehearsal). Max over ranks; None at world size 1."""
    import torch

    if not ctx.distributed or ctx.world_size == 1:
        return None
    scratch = buf.clone()
    for _ in range(3):
        ctx.all_reduce_sum_(scratch)
    ctx.barrier()
    if ctx.device.type != "cuda":
        t0 = time.perf_counter()
        for _ in range(iters):
            ctx.all_reduce_sum_(scratch)
        return ctx.max_scalar((time.perf_counter() - t0) * 1000.0 / iters)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ctx.all_reduce_sum_(scratch)
    e1.record()
    torch.cuda.synchronize()
    return ctx.max_scalar(e0.elapsed_time(e1) / iters)


def _rccl_debug_setup(ctx_rank: int) -> str | None:
    """Ask RCCL for its INIT/GRAPH log in a per-rank file (before the process group exists;
    RCCL reads the variables when the communicator is created), so the JSON line can say
    what RCCL built at this world size: ranks, channels and the transport of each ring hop."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or "NCCL_DEBUG_FILE" in os.environ:
        return None
    path = f"/tmp/wellflow_rccl.{os.getpid()}.r{ctx_rank}.log"
    os.environ.setdefault("NCCL_DEBUG", "INFO")
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH")
    os.environ["NCCL_DEBUG_FILE"] = path
    return path


def _rccl_summary(path: str | None) -> dict | None:
    import re
    from collections import Counter

    if not path or not os.path.exists(path):
        return None
    nranks, chans, via, version = None, set(), Counter(), None
    with open(path, errors="replace") as f:
        for line in f:
            m = re.search(r"nRanks (\d+)", line)
            if m:
                nranks = int(m.group(1))
            m = re.search(r"Channel (\d+)/\d+ :.* via (\S+(?: \S+)?)", line)
            if m:
                chans.add(int(m.group(1)))
                via[m.group(2)] += 1
            m = re.search(r"(RCCL version \S+)", line)
            if m and version is None:
                version = m.group(1)
    return {"nranks": nranks, "channels": len(chans), "transport": dict(via), "version": version, "log": path}


def bench_lstm(args, ctx):
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.train.step import StepRunner

    B, T, F, H = args.batch, args.seq, args.features, args.hidden
    model = f"LSTM seq-len={T} hidden={H} time-series regression (features={F}, linear head, MSE, Adam)"
    if ctx.device.type == "cpu":
        return _cpu_rehearsal(args, ctx, model)
    eng = NativeLSTM(F, H, T, B, device=ctx.device)
    if args.dw_chunk is not None:
        eng.dw_chunk = args.dw_chunk
    if args.fwd_variant is not None:
        eng.fwd_variant = args.fwd_variant
    if args.bwd_variant is not None:
        eng.bwd_variant = args.bwd_variant
    eng.params.copy_(init_lstm_flat(F, H, seed=0).to(ctx.device))
    ctx.broadcast_(eng.params)  # C1: identical init on every rank
    eng.sync_weights()
    # Adam clears the gradient bucket in its own launch (no fill kernel before the backward)
    # Adam refreshes the engine's bf16 weight copies (Wp, WhhT) in the same launch
    opt = FlatAdam(eng.params, eng.grads, lr=args.lr, zero_grads=True, writeback=eng)
    x, y = synth_lstm_batch(B, T, F, seed=ctx.rank)  # Gilbert-consistent windows, GPU-resident
    x, y = x.to(ctx.device), y.to(ctx.device)
    run = StepRunner(eng, opt, ctx, 1.0 / (B * ctx.world_size), lambda k: (x, y),
                     graph=not (args.no_graph or eng.dw_chunk > 0), comm_in_graph=not args.eager_comm)
    el, k, n = _timed(ctx, run.run, args.steps, args.warmup, args.min_timed_s, run.run_many, args.graph_steps,
                      warm_ms=args.warm_ms)
    eng.check_device_errors()  # a timed-out persistent hand-off anywhere in the run fails the bench
    extra = {"persistent_fwd": eng.last_forward_persistent, "persistent_bwd": eng.last_backward_persistent}
    # the engine adds each step's loss straight into the runner's accumulator: mean over the run
    return el, k, B, model, run.take_loss() / (B * n), run, eng, extra


def _cpu_rehearsal(args, ctx, model):
    """--device cpu: the same timed DP step (C1 broadcast, C2 flat all-reduce, flat Adam)
    on the fp32 PyTorch reference model over gloo, through the same StepRunner. It exists so
    the launch / timing / JSON contract at world size > 1 is exercised without GPUs
    (tests/test_bench_cpu.py); its numbers are NOT the benchmark (the line says dtype fp32
    and data 'cpu rehearsal')."""
    import torch

    from wellflow.data.synth import synth_lstm_batch, synth_tabular_batch
    from wellflow.models.base import TorchEngine
    from wellflow.models.lstm import LSTMRegressor
    from wellflow.models.mlp import MLPRegressor
    from wellflow.optim.flat import FlatAdam
    from wellflow.train.step import StepRunner

    torch.manual_seed(0)
    B, F = args.batch, args.features
    if args.model == "lstm":
        eng = TorchEngine(LSTMRegressor(F, args.hidden))
        x, y = synth_lstm_batch(B, args.seq, F, seed=ctx.rank)
    elif args.model == "cnn":
        from wellflow.models.cnn import CNN1DRegressor

        eng = TorchEngine(CNN1DRegressor(), loss="mae_clip", clip=6.0)
        series = torch.randn(B, 60).cumsum(1) * 0.1
        x, y = series[:, :48].contiguous(), series[:, 48:].contiguous()
    else:
        eng = TorchEngine(MLPRegressor(F, (256, 256)))
        x, y = synth_tabular_batch(B, F, seed=ctx.rank)
    ctx.broadcast_(eng.params)
    opt = FlatAdam(eng.params, eng.grads, lr=args.lr)
    run = StepRunner(eng, opt, ctx, 1.0 / (B * ctx.world_size), lambda k: (x, y))
    el, k, n = _timed(ctx, run.run, args.steps, args.warmup, args.min_timed_s)
    return el, k, B, model, run.take_loss() / (B * n), run, eng, {}


def bench_cnn(args, ctx):
    """The reference's own model (cnn.py:110-118): Conv1D(1->100, k=13, ReLU) -> Dropout 0.5 ->
    Dense 3600->12, clipped-MAE loss, Keras SGD-Nesterov (lr .001, momentum .99, decay 1e-6),
    on 48-step windows; the step is NativeCNN (im2col + MFMA GEMMs with fused bias / ReLU /
    dropout epilogues, split-K weight gradients) through the same StepRunner."""
    import torch

    from wellflow.models.cnn import CNN1DRegressor, CnnLayout, NativeCNN
    from wellflow.optim.flat import FlatSGD
    from wellflow.train.step import StepRunner

    lay = CnnLayout()
    B = args.batch
    model = "1-D CNN (reference cnn.py): 48-step window, Conv1D 100x13 + ReLU, dropout 0.5, Dense 3600->12, clipped MAE, SGD-Nesterov"
    ref = CNN1DRegressor(lay.input_len, lay.in_ch, lay.filters, lay.kernel, lay.outputs)
    if ctx.device.type == "cpu":
        return _cpu_rehearsal(args, ctx, model)
    eng = NativeCNN(lay, B, ctx.device)
    eng.params.copy_(ref.to_flat().to(ctx.device))
    ctx.broadcast_(eng.params)
    eng.sync_weights()
    # SGD refreshes the engine's bf16 operand images in the same launch (no pack launch per step)
    opt = FlatSGD(eng.params, eng.grads, zero_grads=True, writeback=eng)
    g = torch.Generator(device="cpu").manual_seed(ctx.rank)
    series = torch.randn(B, lay.input_len + lay.outputs, generator=g).cumsum(1) * 0.1  # random-walk windows
    x = series[:, : lay.input_len].contiguous().to(ctx.device)
    y = series[:, lay.input_len :].contiguous().to(ctx.device)
    gscale = 1.0 / (B * ctx.world_size * lay.outputs)
    run = StepRunner(eng, opt, ctx, gscale, lambda k: (x, y), graph=not args.no_graph,
                     comm_in_graph=not args.eager_comm)
    step, many, gsteps, extra = run.run, run.run_many, args.graph_steps, {}
    if ctx.world_size == 1 and not args.no_small and eng.small_steps_reason(B, opt, x) is None:
        # small batches (the reference's 20 windows, one process): the Trainer's path — n complete
        # steps per persistent launch (NativeCNN.fused_steps, csrc/cnn_small.hip)
        gsteps = _small_launch_steps(args)
        ridx = torch.arange(B, device=ctx.device).repeat(gsteps)  # the one resident batch, every step

        def many(n):  # noqa: F811
            eng.fused_steps(x, y, B, n, opt, gscale, rows=ridx[: n * B], loss_into=run.loss_acc)

        def step():  # noqa: F811
            many(1)

        extra["small_fused_steps_per_launch"] = gsteps
    el, k, n = _timed(ctx, step, args.steps, args.warmup, args.min_timed_s, many, gsteps, warm_ms=args.warm_ms)
    if extra:
        eng.check_device_errors()
    return el, k, B, model, run.take_loss() / (B * lay.outputs * n), run, eng, extra


def bench_mlp(args, ctx, online: bool):
    import torch

    from wellflow.data.stream import DeviceStreamer, HostPool
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.train.step import StepRunner

    B, F, hid = args.batch, args.features, (256, 256)
    kind = "dynamic (online, host->HBM streamed mini-batches)" if online else "static (resident batch)"
    model = f"{kind} 3-layer MLP regression F={F} -> 256 -> 256 -> 1, MSE, Adam"
    if ctx.device.type == "cpu":
        return _cpu_rehearsal(args, ctx, model)
    eng = NativeMLP(F, hid, B, device=ctx.device)
    eng.params.copy_(init_mlp_flat(F, hid, seed=0).to(ctx.device))
    ctx.broadcast_(eng.params)
    eng.sync_weights()
    # Adam writes the bf16 compute copy and clears the gradient bucket in its own launch
    opt = FlatAdam(eng.params, eng.grads, lr=args.lr, shadow=eng.shadow, zero_grads=True,
                   shadow_t=eng.shadow_t)
    gscale = 1.0 / (B * ctx.world_size)
    graph = not args.no_graph
    extra = {}
    if online:
        from wellflow.utils.numa import bind_to_gpu_numa

        # pinned ring pages on the GPU's NUMA node (utils/numa.py), before anything is pinned
        extra["numa_bound_cpus"] = len(bind_to_gpu_numa(ctx.device.index or 0))
        # features cross PCIe as bf16 (the engine's MFMA input format: identical numerics to
        # streaming fp32 and casting on the device, half the bytes); targets stay fp32
        x_dtype = torch.float32 if args.stream_fp32 else torch.bfloat16
        pool = HostPool(lambda k: synth_tabular_batch(B, F, seed=1000 * ctx.rank + k), n=args.host_pool,
                        x_dtype=x_dtype)
        # copies bracketed by events: the JSON reports their device time (a shared host's PCIe
        # load shows up here, not in the kernels)
        # every 16th batch's copies timed (all of them cost this PCIe-bound config ~5 %)
        streamer = DeviceStreamer(pool, ctx.device, depth=args.stream_depth,
                                  timing=0 if args.no_h2d_timing else 16)
        # one captured step per ring slot (the graph reads that slot's buffers)
        run = StepRunner(eng, opt, ctx, gscale, lambda k: tuple(streamer.slots[k][:2]), graph=graph,
                         comm_in_graph=not args.eager_comm)

        def step():
            streamer.next()
            run.run(streamer.last_slot)

        many = None
        if ctx.world_size == 1 and not args.no_small and eng.small_steps_reason(B, opt) is None:
            # small batches on one GPU: the job's path (train/online.py _ChunkStage) — a stream
            # chunk of n batches crosses PCIe as ONE async copy into a device buffer (two,
            # alternating: the next chunk's copy overlaps this launch) and its batches train as
            # n complete steps per persistent launch (NativeMLP.fused_steps)
            nmax = _small_launch_steps(args)
            xh, yh = synth_tabular_batch(nmax * B, F, seed=1000 * ctx.rank)
            xh = eng.to_input_format(xh).pin_memory()
            yh = yh.float().pin_memory()
            bufs = [(torch.empty_like(xh, device=ctx.device), torch.empty_like(yh, device=ctx.device)) for _ in range(2)]
            cstream, events, staged, launches = torch.cuda.Stream(ctx.device), [None, None], [0, 0], [0]

            def stage(j, rows):  # launch j's rows (the next launch's: prefetched behind this one)
                compute = torch.cuda.current_stream(ctx.device)  # (the copy stream inside the `with`)
                with torch.cuda.stream(cstream):
                    # buffer j % 2 was last read by launch j - 2, enqueued before this copy
                    cstream.wait_stream(compute)
                    bufs[j % 2][0][:rows].copy_(xh[:rows], non_blocking=True)
                    bufs[j % 2][1][:rows].copy_(yh[:rows], non_blocking=True)
                    events[j % 2] = torch.cuda.Event()
                    events[j % 2].record(cstream)
                staged[j % 2] = rows

            def many(n):
                j = launches[0]
                launches[0] += 1
                if j == 0 or staged[j % 2] < n * B:
                    stage(j, n * B)
                torch.cuda.current_stream(ctx.device).wait_event(events[j % 2])
                xb, yb = bufs[j % 2]
                eng.fused_steps(xb, yb, B, n, opt, gscale, loss_into=run.loss_acc)
                stage(j + 1, n * B)

            def step():  # noqa: F811
                many(1)

            extra["small_fused_steps_per_launch"] = nmax
            extra["online_chunk_rows"] = nmax * B
    else:
        nb = max(1, args.mlp_batches)
        x, y = synth_tabular_batch(B * nb, F, seed=ctx.rank)
        # resident in the engine's input format, as the job path keeps its datasets (Trainer);
        # --mlp-batches N: N distinct resident batches, step i of a graph replay reads batch
        # i % N (fresh rows every step, as a training pass over a table does)
        x, y = eng.to_input_format(x.to(ctx.device)), y.to(ctx.device)

        def inputs(k):
            j = (k[1] if isinstance(k, tuple) else 0) % nb
            return x[j * B : (j + 1) * B], y[j * B : (j + 1) * B]

        run = StepRunner(eng, opt, ctx, gscale, inputs, graph=graph, comm_in_graph=not args.eager_comm)
        step = run.run
        many = run.run_many
        if ctx.world_size == 1 and not args.no_small and eng.small_steps_reason(B, opt) is None:
            # small batches (<= 256 rows, one process): the Trainer's path — n complete steps
            # (forward, backward, Adam) per persistent launch (NativeMLP.fused_steps); step i of
            # a launch reads batch i % N of the resident set through row ids
            # as the Trainer: up to 256 steps per launch (the timed window is one launch at <= 256 steps)
            nmax = _small_launch_steps(args)
            ridx = torch.arange(nmax * B, device=ctx.device) % (B * nb)

            def many(n):  # noqa: F811 - replaces the graph replay for this path
                eng.fused_steps(x, y, B, n, opt, gscale, rows=ridx[: n * B], loss_into=run.loss_acc)

            def step():  # noqa: F811
                many(1)

            extra["small_fused_steps_per_launch"] = nmax
    # the streamed config changes its input slot every step: single-step replays
    el, k, n = _timed(ctx, step, args.steps, args.warmup, args.min_timed_s, many,
                      extra.get("small_fused_steps_per_launch", args.graph_steps), warm_ms=args.warm_ms)
    if "small_fused_steps_per_launch" in extra:
        eng.check_device_errors()
    if online and "small_fused_steps_per_launch" not in extra:
        extra.update(streamer.copy_stats(skip=1))
        extra["h2d_mb_per_step"] = round((streamer.slots[0][0].numel() * streamer.slots[0][0].element_size()
                                          + streamer.slots[0][1].numel() * 4) / 1e6, 3)
    # the engine adds each step's loss straight into the runner's accumulator: mean over the run
    return el, k, B, model, run.take_loss() / (B * n), run, eng, extra


SECONDARY = ("mlp", "mlp_online", "cnn", "cnn_b20", "mlp_b256", "mlp_online_b256")
# the submission API's own defaults as secondaries (config.py MODEL_DEFAULTS: CNN 20 windows,
# cnn.py:128; MLP / online MLP 256 rows): on one GPU the K-steps-per-launch paths
SMALL_SECONDARY = {"cnn_b20": ("cnn", 20), "mlp_b256": ("mlp", 256), "mlp_online_b256": ("mlp_online", 256)}


def _auto_secondary(default_headline: bool, world: int) -> list:
    """The configs a default invocation times after the headline: all of SECONDARY on one GPU;
    under DP without the job-default ones (they show the one-GPU K-steps-per-launch paths; at
    DP they would time per-step launches behind a latency-bound all-reduce — pass them
    explicitly for that)."""
    if not default_headline:
        return []
    return [m for m in SECONDARY if world <= 1 or m not in SMALL_SECONDARY]


def _small_launch_steps(args) -> int:
    """Steps per persistent launch of the small-batch paths: the Trainer's 256; the headline
    times exactly --steps (<= 256 of them as one launch, as its graph replays), a secondary
    (min_timed_s > 0, steps raised to fill its window) runs the Trainer's launches."""
    if getattr(args, "min_timed_s", 0.0) > 0:
        return 256
    return max(1, min(args.steps, 256))
CPU_BATCH = {"lstm": 256, "mlp": 8192, "mlp_online": 8192, "cnn": 1024}


def _run_model(args, ctx):
    if args.model == "lstm":
        return bench_lstm(args, ctx)
    if args.model == "cnn":
        return bench_cnn(args, ctx)
    return bench_mlp(args, ctx, online=args.model == "mlp_online")


def _secondary(args, ctx, models) -> dict:
    """BASELINE.json:8-10 in the same invocation, AFTER the headline's timed region: each
    config's own full training step (same StepRunner, same timing bracket: barrier +
    synchronize on both sides, max over ranks), default per-GPU batch, the headline's
    steps / warmup. The headline's engine is freed first."""
    import gc

    import torch

    out = {}
    for m in models:
        a = argparse.Namespace(**vars(args))
        if m in SMALL_SECONDARY:
            a.model, a.batch = SMALL_SECONDARY[m]
        else:
            a.model = m
            a.batch = (CPU_BATCH if ctx.device.type == "cpu" else DEFAULT_BATCH)[m]
        a.min_timed_s = args.secondary_min_s  # the headline keeps the driver's --steps exactly
        gc.collect()
        if ctx.device.type == "cuda":
            torch.cuda.empty_cache()
        el, k, B, desc, loss, run, eng, extra = _run_model(a, ctx)
        untimed = _LAST_TIMED["untimed"]
        W = ctx.world_size
        # this config's OWN gradient bucket all-reduced at this world size (round-5 VERDICT item 5:
        # the DP=8 MLP configs need their comm figure next to their step time, not the headline's)
        comm = _comm_ms(ctx, eng.grads)
        ms = 1000.0 * el / max(k, 1)
        comm_rec = {"comm_ms": None if comm is None else round(comm, 4),
                    "grad_bucket_mb": round(eng.grads.numel() * 4 / 2**20, 3), "comm_dtype": args.comm_dtype,
                    # the all-reduce runs serially inside the step (after the backward, before the
                    # optimizer): its share of the timed step is the DP efficiency it costs
                    "comm_share": None if comm is None else round(comm / ms, 4)}
        out[m] = {"metric": f"rows/sec (whole node), {a.model} regression training", "value": round(B * W * k / el, 1),
                  "unit": "rows/s", "ms_per_step": round(1000.0 * el / max(k, 1), 4), "steps": k,
                  "warmup": a.warmup, "untimed_steps": untimed, "timed_s": round(el, 4), "per_gpu_batch": B,
                  "global_batch": B * W,
                  "model": desc, "train_loss": round(loss, 6), "step_graph": bool(run.graphs),
                  "graph_steps": max((key[2] for key in run.graphs if isinstance(key, tuple) and key[0] == "many"),
                                     default=1),
                  **comm_rec,
                  **{k: v for k, v in extra.items()
                     if k.startswith("h2d") or k in ("persistent_fwd", "small_fused_steps_per_launch")}}
        if _LAST_TIMED.get("gpu_state") is not None:
            out[m]["gpu_state"] = _LAST_TIMED["gpu_state"]
        if W > 1 and ctx.device.type == "cuda":
            out[m]["rccl"] = _rccl_summary(os.environ.get("NCCL_DEBUG_FILE"))
        del run, eng
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", choices=["lstm", "mlp", "mlp_online", "cnn"], default="lstm")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (rows)")
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--features", type=int, default=16)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--dw-chunk", type=int, default=None, help="timesteps per overlapped dW chunk (0 = serial)")
    ap.add_argument("--fwd-variant", type=int, default=None)
    ap.add_argument("--bwd-variant", type=int, default=None)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--mlp-batches", type=int, default=1,
                    help="mlp: distinct resident batches cycled through a graph replay's steps")
    ap.add_argument("--warm-ms", type=float, default=25.0,
                    help="untimed n-step replays of about this much work after the graph capture")
    ap.add_argument("--graph-steps", type=int, default=8,
                    help="timed steps per captured graph replay (StepRunner.run_many; 1 = one replay per step)")
    ap.add_argument("--eager-comm", action="store_true", help="all-reduce between two graphs, not captured")
    ap.add_argument("--no-small", action="store_true",
                    help="mlp <= 256 rows / cnn <= 64 windows: the regular step graphs instead of the "
                         "persistent K-step launch")
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="C2 gradient all-reduce precision (parallel/dist.py; default fp32)")
    ap.add_argument("--stream-fp32", action="store_true", help="mlp_online: stream fp32 features")
    ap.add_argument("--stream-depth", type=int, default=4, help="mlp_online: device ring slots")
    ap.add_argument("--no-h2d-timing", action="store_true", help="mlp_online: no events around the copies (default: every 16th batch timed)")
    ap.add_argument("--host-pool", type=int, default=8, help="mlp_online: distinct pinned host batches cycled")
    ap.add_argument("--device", choices=["auto", "cpu"], default="auto",
                    help="cpu: rehearse the launch/timing/JSON contract on the fp32 reference over gloo")
    ap.add_argument("--secondary", default="auto",
                    help="comma list of configs timed after the headline (mlp,mlp_online,cnn), 'none'; "
                         "auto = all three after the default LSTM headline, none otherwise")
    ap.add_argument("--secondary-min-s", type=float, default=None,
                    help="minimum timed window per secondary config (its steps are raised to reach it); "
                         "default 0.1 s on the GPU, 0 on the CPU rehearsal")
    ap.add_argument("--parity", choices=["auto", "on", "none"], default="auto",
                    help="after every timed region: 20-step Adam trajectory of the headline shape vs fp32 "
                         "torch on the same GPU (auto = with the default headline)")
    args = ap.parse_args()
    args.min_timed_s = 0.0  # the headline: exactly --steps
    if args.secondary_min_s is None:
        args.secondary_min_s = 0.0 if args.device == "cpu" else 0.1
    if args.batch is None:
        args.batch = DEFAULT_BATCH[args.model]
        if args.device == "cpu":  # the fp32 CPU rehearsal: N ranks share one host's memory
            args.batch = CPU_BATCH[args.model]
    default_headline = args.model == "lstm" and (args.batch, args.seq, args.hidden, args.features) == (
        DEFAULT_BATCH["lstm"] if args.device != "cpu" else CPU_BATCH["lstm"], 64, 512, 16)
    if args.secondary == "auto":
        secondary = _auto_secondary(default_headline, max(args.gpus, int(os.environ.get("WORLD_SIZE", "1"))))
    else:
        secondary = [m for m in args.secondary.split(",") if m and m != "none"]
        bad = [m for m in secondary if m not in SECONDARY]
        if bad:
            ap.error(f"--secondary: unknown {bad}")

    bad = _diag_env()
    if bad:
        # timing-only switches produce a faster, WRONG step: never a benchmark number
        print(f"bench.py: refusing to run with diagnostic variables set: {bad}", file=sys.stderr)
        return 3
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return _spawn_ranks(args.gpus, sys.argv[1:])

    import torch

    from wellflow.parallel.dist import DistContext

    if args.device == "auto" and not torch.cuda.is_available():
        # never fall back silently: a CPU number is not the benchmark
        print("bench.py: no GPU visible (use --device cpu for the contract rehearsal)", file=sys.stderr)
        return 2
    rccl_log = _rccl_debug_setup(int(os.environ.get("RANK", "0"))) if args.device != "cpu" else None
    ctx = DistContext.from_env(device="cpu" if args.device == "cpu" else None, comm_dtype=args.comm_dtype)
    cpu = ctx.device.type == "cpu"
    if ctx.world_size != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ctx.world_size}", file=sys.stderr)
        ctx.shutdown()
        return 2
    if not cpu:
        from wellflow.ops.native import lib

        if lib().diag_build():
            print("bench.py: the loaded _C.so is a WF_DIAG build (timing-only variants live); "
                  "rebuild without WELLFLOW_DIAG_BUILD", file=sys.stderr)
            ctx.shutdown()
            return 3
    torch.manual_seed(1234 + ctx.rank)
    if not cpu:
        from wellflow.utils.gpustate import GpuStateSampler

        smp = GpuStateSampler(ctx.device.index or 0)
        if smp.available:
            _SAMPLER["s"] = smp
    elapsed, steps, B, model, loss, run, eng, extra = _run_model(args, ctx)
    untimed = _LAST_TIMED["untimed"]
    gpu_state = _LAST_TIMED.get("gpu_state")
    assert steps == args.steps
    comm = _comm_ms(ctx, eng.grads)
    grad_mb = round(eng.grads.numel() * 4 / 2**20, 3)
    step_graph, comm_in_graph = bool(run.graphs), bool(run.captured_comm)
    graph_steps = max((key[2] for key in run.graphs if isinstance(key, tuple) and key[0] == "many"), default=1)
    del run, eng
    sec = _secondary(args, ctx, secondary) if secondary else None
    par = None
    if not cpu and (args.parity == "on" or (args.parity == "auto" and default_headline)):
        # numerics of the headline step, after every timed region (rank 0's GPU; the others wait)
        if ctx.is_main:
            import gc

            from wellflow.train.parity import cnn_sgd_trajectory, lstm_adam_trajectory, mlp_adam_trajectory

            par = {}
            for name, fn in (("lstm", lstm_adam_trajectory), ("mlp", mlp_adam_trajectory), ("cnn", cnn_sgd_trajectory)):
                gc.collect()
                torch.cuda.empty_cache()
                r = fn(ctx.device)
                r.pop("native", None)
                r.pop("fp32", None)
                par[name] = r
            par["pass"] = all(par[k]["pass"] for k in ("lstm", "mlp", "cnn"))
        ctx.barrier()

    W = ctx.world_size
    if ctx.is_main:
        import torch.distributed as dist

        rccl = None
        if not cpu:
            try:
                v = torch.cuda.nccl.version()
                rccl = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
            except Exception:  # noqa: BLE001 - version probe only
                rccl = None
        rec = {
            "metric": METRIC if args.model == "lstm" else f"rows/sec (whole node), {args.model} regression training",
            "value": round(B * W * args.steps / elapsed, 1),
            "unit": "rows/s",
            "n_gpus": W,
            "steps": args.steps,
            "warmup": args.warmup,
            # every step run outside the timed window: the W warm-up steps, the graph captures'
            # replays and the post-capture warm replays (--warm-ms)
            "untimed_steps": untimed,
            "ms_per_step": round(1000.0 * elapsed / max(args.steps, 1), 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,  # the reference publishes no numbers (BASELINE.json "published": {})
            "dtype": "fp32" if cpu else "bf16",
            "data": ("synthetic random-walk windows" if args.model == "cnn"
                     else "synthetic (Gilbert-equation well-log data)") + ", random-init weights"
                    + ("; CPU contract rehearsal, not a benchmark" if cpu else ""),
            "config": {
                "model": model,
                "global_batch": B * W,
                "per_gpu_batch": B,
                "seq_len": args.seq if args.model == "lstm" else 1,
                "parallelism": f"dp{W}",
            },
            "world_size": dist.get_world_size() if dist.is_initialized() else 1,
            "backend": ctx.backend or ("none" if W == 1 else None),
            "rccl_version": rccl,
            "comm_ms": None if comm is None else round(comm, 4),
            "grad_bucket_mb": grad_mb,
            "comm_dtype": args.comm_dtype,
            "step_graph": step_graph,
            "graph_steps": graph_steps,
            "comm_in_graph": comm_in_graph,
            "train_loss": round(loss, 6),  # mean over the run
            "timed_s": round(elapsed, 4),
            **extra,
        }
        if W > 1 and not cpu:
            rec["rccl"] = _rccl_summary(rccl_log)
            rec["hsa_enable_ipc_mode_legacy"] = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
        # rank 0's GPU over the headline's timed window: sampled gfx clock, socket power, hotspot
        # temperature and the firmware's limiter residencies (utils/gpustate.py); None off-GPU
        rec["gpu_state"] = gpu_state
        if sec is not None:
            rec["secondary"] = sec
        if par is not None:
            rec["parity"] = par
        rec["env"] = _env_record()
        print(json.dumps(rec), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
