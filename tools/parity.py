#!/usr/bin/env python3
"""Val-MSE parity with error bars (BASELINE.json:2 "val MSE parity"): the native bf16 MI355X
engine vs the fp32 PyTorch oracle over several seeds, both through the production job path
(train/job.py: argv contract -> features -> engine -> Trainer/StepRunner); only
``--precision`` differs (bf16 = hand-written HIP kernels, fp32 = torch reference module).

    python tools/parity.py --model lstm --seeds 0,1,2 --out profiles/r2/parity_lstm.json

Each seed fixes the synthetic table, the split, the init and the batch order of BOTH runs.
Reported: per-precision mean +- std of the final and best val MSE, the mean gap, and the
verdict ``pass`` = |mean gap| <= max(fp32 seed-to-seed std, 2 % of the fp32 mean).
Defaults are the LSTM headline shapes (seq 64, hidden 512, batch 2048 per GPU) on a table
large enough for ~40 steps per epoch. ``--dropout 0`` (the CNN default here) removes the
only RNG that differs between the engines (native counter hash vs torch's Philox), so the
CNN comparison isolates kernel error. The Gilbert physical model's val MSE (standardised
target units) is the non-learned baseline.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from wellflow.config import parse_argv  # noqa: E402
from wellflow.train.job import run_config  # noqa: E402

NAMES = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
TYPES = "string,string,int,float,float,float,float,float,float,float"
DEFAULTS = {  # model: (wells, steps, batch, epochs, extra argv)
    "lstm": (96, 1500, 2048, 8, ["--seq-len", "64", "--hidden", "512"]),
    "mlp": (64, 2000, 4096, 8, []),
    "cnn": (32, 1500, 256, 8, ["--lr", "0.01", "--dropout", "0"]),
}


def gilbert_val_mse(cfg):
    """Gilbert prediction on the validation rows, standardised like the learned targets."""
    from wellflow.data.features import FeaturePipeline, random_split, take
    from wellflow.data.io import load_table
    from wellflow.data.schema import parse_schema
    from wellflow.models.gilbert import GilbertModel

    schema = parse_schema(cfg.column_names, cfg.column_types)
    table = load_table(cfg.data, schema, synth_wells=cfg.synth_wells, synth_steps=cfg.synth_steps,
                       seed=cfg.seed)
    idx = random_split(len(table["flow"]), cfg.split, cfg.seed)
    pipe = FeaturePipeline(schema, "flow", standardize_target=True).fit(take(table, idx[0]))
    val = take(table, idx[1])
    q = GilbertModel().flow_rate(val["whp"], val["choke"], val["glr"])
    y = (val["flow"] - pipe.y_mean) / pipe.y_std
    p = (q - pipe.y_mean) / pipe.y_std
    return float(np.mean((p - y) ** 2))


def _ms(xs):
    return {"mean": statistics.fmean(xs), "std": statistics.stdev(xs) if len(xs) > 1 else 0.0, "values": xs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lstm", choices=sorted(DEFAULTS))
    ap.add_argument("--seeds", default="0,1,2")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--wells", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    wells, steps, batch, epochs, extra = DEFAULTS[a.model]
    wells, steps = a.wells or wells, a.steps or steps
    batch, epochs = a.batch or batch, a.epochs or epochs
    seeds = [int(s) for s in a.seeds.split(",")]
    runs = {"bf16": [], "fp32": []}
    for seed in seeds:
        base = [NAMES, TYPES, "flow", f"/tmp/wellflow_parity_{a.model}_{seed}/", "--epochs", str(epochs),
                "--patience", str(epochs + 1), "--synth-wells", str(wells), "--synth-steps", str(steps),
                "--batch-size", str(batch), "--device", "cuda", "--verbose", "0", "--seed", str(seed)] + extra
        for prec in ("bf16", "fp32"):
            cfg = parse_argv(a.model, base + ["--precision", prec])
            out = run_config(cfg, log=lambda *x, **k: None)
            h = out["history"]
            runs[prec].append({"seed": seed, "native": out["native"], "val_mse": h["val_mse"],
                               "final_val_mse": h["val_mse"][-1], "best_val_mse": min(h["val_mse"]),
                               "test_mse": out["test_mse"], "steps": out["steps"], "elapsed_s": out["elapsed"]})
            print(f"seed {seed} {prec}: native={out['native']} steps={out['steps']} "
                  f"val_mse={['%.5f' % v for v in h['val_mse']]}", flush=True)
    fin = {p: _ms([r["final_val_mse"] for r in runs[p]]) for p in runs}
    best = {p: _ms([r["best_val_mse"] for r in runs[p]]) for p in runs}
    gap = fin["bf16"]["mean"] - fin["fp32"]["mean"]
    tol = max(fin["fp32"]["std"], 0.02 * fin["fp32"]["mean"])
    summary = {
        "model": a.model, "epochs": epochs, "per_gpu_batch": batch, "seeds": seeds,
        "data": f"synthetic Gilbert well logs, {wells} wells x {steps} steps, time-block split",
        "config_extra": extra,
        "final_val_mse": fin, "best_val_mse": best,
        "mean_gap_bf16_minus_fp32": gap, "relative_mean_gap": gap / fin["fp32"]["mean"],
        "tolerance": tol, "pass": abs(gap) <= tol,
        "runs": runs,
    }
    if a.model in ("lstm", "mlp"):
        cfg = parse_argv("gilbert", [NAMES, TYPES, "flow", "/tmp/wellflow_parity/", "--synth-wells", str(wells),
                                     "--synth-steps", str(steps), "--seed", str(seeds[0])])
        summary["gilbert_val_mse_standardized"] = gilbert_val_mse(cfg)
    print(json.dumps({k: v for k, v in summary.items() if k != "runs"}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(summary, fh, indent=1)
    return 0 if summary["pass"] else 1


if __name__ == "__main__":
    sys.exit(main())
