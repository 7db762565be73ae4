#!/usr/bin/env python3
"""Val-MSE parity (BASELINE.json:2 "val MSE parity"): native bf16 MI355X engine vs the fp32
PyTorch oracle, same data, same split, same init, same optimizer and batch order.

    python tools/parity.py --model lstm --epochs 10 [--out profiles/parity_lstm.json]

Both runs go through the production job path (train/job.py: argv contract -> features ->
engine -> trainer); only ``--precision`` differs (bf16 = hand-written HIP kernels, fp32 =
torch reference module). The Gilbert physical model's MSE on the same validation rows is
reported as the non-learned baseline (in the standardised target units the learned models
train on).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from wellflow.config import parse_argv  # noqa: E402
from wellflow.train.job import run_config  # noqa: E402

NAMES = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
TYPES = "string,string,int,float,float,float,float,float,float,float"


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lstm", choices=["lstm", "mlp", "cnn"])
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--wells", type=int, default=32)
    ap.add_argument("--steps", type=int, default=800)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    base = [NAMES, TYPES, "flow", "/tmp/wellflow_parity/", "--epochs", str(a.epochs), "--patience",
            str(a.epochs + 1), "--synth-wells", str(a.wells), "--synth-steps", str(a.steps),
            "--batch-size", str(a.batch), "--device", "cuda", "--verbose", "0"]
    if a.model == "cnn":
        base += ["--lr", "0.01"]
    res = {}
    for prec in ("bf16", "fp32"):
        cfg = parse_argv(a.model, base + ["--precision", prec])
        out = run_config(cfg, log=lambda *x, **k: None)
        res[prec] = {"val_mse": out["history"]["val_mse"], "val_loss": out["history"]["val_loss"],
                     "test_mse": out["test_mse"], "test_loss": out["test_loss"],
                     "native": out["native"], "elapsed_s": out["elapsed"]}
        print(f"{prec}: native={out['native']} val_mse={['%.5f' % v for v in out['history']['val_mse']]}",
              flush=True)
    b, f = res["bf16"]["val_mse"][-1], res["fp32"]["val_mse"][-1]
    summary = {
        "model": a.model, "epochs": a.epochs, "batch": a.batch,
        "data": f"synthetic Gilbert well logs, {a.wells} wells x {a.steps} steps",
        "final_val_mse_bf16_native": b, "final_val_mse_fp32_oracle": f,
        "relative_gap": (b - f) / f, "best_val_mse_bf16": min(res["bf16"]["val_mse"]),
        "best_val_mse_fp32": min(res["fp32"]["val_mse"]),
        "test_mse_bf16": res["bf16"]["test_mse"], "test_mse_fp32": res["fp32"]["test_mse"],
        "runs": res,
    }
    if a.model in ("lstm", "mlp"):
        cfg = parse_argv("gilbert", base)
        summary["gilbert_val_mse_standardized"] = gilbert_val_mse(cfg)
    print(json.dumps({k: v for k, v in summary.items() if k != "runs"}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(summary, fh, indent=1)


if __name__ == "__main__":
    main()
