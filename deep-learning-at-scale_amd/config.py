"""Submission argv contract + typed run configuration.

Reference contract (cnn.py:2, 41-44): ``<script>.py columnNames columnTypes targetColumn
storagePath`` — four positional strings; names and types are comma-separated lists of
equal length. Hyper-parameters were hard-coded constants (cnn.py:31, 39, 68, 117, 121,
128); here they are explicit :class:`RunConfig` fields whose defaults equal the
reference values for the reference model (the CNN) and documented choices for the
declared-only models.

Compatibility decisions:
* the 4 positionals are unchanged; an optional 5th positional (or ``--data``) is the data
  path — the reference read ``sys.argv[2]`` (the TYPES string) as the CSV path (#1).
  Without it, synthetic Gilbert well-log data is generated (``--data synth``).
* ``storagePath + "models/<name>.mdl"`` string concatenation is preserved, so both
  ``/x/`` and ``/x`` forms work the way the web component used them (#11: ``/x`` gets a
  separator inserted instead of writing ``/xmodels``).
"""
from __future__ import annotations

import argparse
import dataclasses
import os

# per-model defaults for the declared-only families (the CNN keeps reference constants)
MODEL_DEFAULTS = {
    "cnn": dict(loss="mae_clip", optimizer="sgd", lr=0.001, momentum=0.99, decay=1e-6,
                nesterov=True, batch_size=20, epochs=1000, patience=10),
    # batch_size 0 = auto (train/job.py auto_batch): on a GPU the rows that fill the device
    # (mlp: NativeMLP.full_batch, 262,144 on 256 CUs; lstm: one co-resident persistent grid,
    # NativeLSTM.full_grid_batch, 8192 at H = 512), capped at 1/8 of the rank's training rows,
    # the same for --precision bf16 and fp32; 256 on the CPU. online_chunk 0 = auto: sized in
    # rows (train/job.py auto_online_chunk: up to 2M rows per rank, >= 4 chunks per pass).
    # The LSTM defaults to auto (its val-MSE parity at the auto batch: profiles/r3/
    # parity_lstm_paired_10seeds.json). The MLPs keep the small-batch regime (256) as their job
    # default: the fill-the-GPU batch leaves ~8 Adam steps per epoch on a 2M-row table and its
    # val MSE was never shown equal to batch 256 (round-4 ADVICE); pass --batch-size 0 (or a
    # size) for throughput runs, as bench.py and tools/job_throughput.py do.
    "mlp": dict(loss="mse", optimizer="adam", lr=1e-3, batch_size=256, epochs=200, patience=10),
    "mlp_online": dict(loss="mse", optimizer="adam", lr=1e-3, batch_size=256, epochs=50, patience=5,
                       online_chunk=0),
    "lstm": dict(loss="mse", optimizer="adam", lr=1e-3, batch_size=0, epochs=100, patience=10),
    "gilbert": dict(loss="mse", epochs=0, batch_size=0),
}


@dataclasses.dataclass
class RunConfig:
    model: str = "cnn"
    column_names: str = ""
    column_types: str = ""
    target: str = ""
    storage_path: str = "./"
    data: str = "synth"          # CSV path or "synth"
    header: bool = False         # cnn.py:65 read with header=False
    seed: int = 42               # reference had np.random.seed commented out (cnn.py:35)
    split: tuple = (0.64, 0.16, 0.2)
    epochs: int = 1000
    batch_size: int = 20
    patience: int = 10
    loss: str = "mae_clip"
    clip: float = 6.0
    optimizer: str = "sgd"
    lr: float = 0.001
    momentum: float = 0.99
    decay: float = 1e-6
    nesterov: bool = True
    weight_decay: float = 0.0
    # model shapes
    hidden: int = 512            # LSTM hidden (BASELINE.json:11)
    seq_len: int = 64            # LSTM window (BASELINE.json:11)
    mlp_hidden: tuple = (256, 256)
    cnn_input_len: int = 48      # implied by Dense(3600, 12) = 100 x 36 (cnn.py:111-114)
    cnn_filters: int = 100
    cnn_kernel: int = 13
    cnn_outputs: int = 12
    dropout: float = 0.5
    # runtime
    device: str = "auto"         # auto | cpu | cuda
    precision: str = "bf16"      # bf16 (native MFMA path) | fp32 (torch oracle)
    comm_dtype: str = "fp32"     # C2 gradient all-reduce precision: fp32 | bf16 (parallel/dist.py)
    group_col: str = ""          # series id column for windowing (default: first string col)
    # windowed models (lstm, cnn): "time" = contiguous per-series blocks in time order with a
    # one-window gap between splits (no row of a val/test window inside any training window);
    # "random" = windows drawn at random (overlapping windows then leak across splits)
    window_split: str = "time"
    synth_wells: int = 16
    synth_steps: int = 600
    online_chunk: int = 4096     # dynamic model: rows per streamed chunk (mlp_online default 0 = auto)
    max_steps: int = 0           # 0 = no cap (tests / smoke)
    resume: bool = False
    verbose: int = 2             # Keras verbose=2: one line per epoch (cnn.py:128)
    metrics_path: str = ""       # JSONL: one record per epoch / chunk (rank 0)
    fail_at_step: int = -1       # fault injection for resume tests (env WELLFLOW_FAIL_AT_STEP)

    @property
    def model_dir(self) -> str:
        sp = self.storage_path
        if sp and not sp.endswith(("/", os.sep)):
            sp = sp + os.sep
        return sp + "models"

    def mdl_path(self, name: str | None = None) -> str:
        return os.path.join(self.model_dir, f"{name or self.model}.mdl")

    def ckpt_path(self, name: str | None = None) -> str:
        return os.path.join(self.model_dir, f"{name or self.model}.ckpt")


def _tuple_floats(s: str):
    return tuple(float(v) for v in s.split(","))


def _tuple_ints(s: str):
    return tuple(int(v) for v in s.split(","))


def build_parser(model: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(
        prog=f"{model}.py",
        description="Usage: python3 <script> columnNames columnTypes targetColumn storagePath [dataPath]",
    )
    ap.add_argument("columnNames")
    ap.add_argument("columnTypes")
    ap.add_argument("targetColumn")
    ap.add_argument("storagePath")
    ap.add_argument("dataPath", nargs="?", default=None)
    ap.add_argument("--data", default=None, help="CSV path or 'synth' (overrides dataPath)")
    ap.add_argument("--header", action="store_true")
    ap.add_argument("--seed", type=int)
    ap.add_argument("--split", type=_tuple_floats)
    ap.add_argument("--epochs", type=int)
    ap.add_argument("--batch-size", type=int, dest="batch_size",
                    help="per-GPU rows per step (lstm, mlp, mlp_online: 0 = auto, sized to fill the GPU)")
    ap.add_argument("--patience", type=int)
    ap.add_argument("--loss", choices=["mse", "mae_clip"])
    ap.add_argument("--clip", type=float)
    ap.add_argument("--optimizer", choices=["adam", "sgd"])
    ap.add_argument("--lr", type=float)
    ap.add_argument("--momentum", type=float)
    ap.add_argument("--decay", type=float)
    ap.add_argument("--no-nesterov", dest="nesterov", action="store_false", default=None)
    ap.add_argument("--weight-decay", type=float, dest="weight_decay")
    ap.add_argument("--hidden", type=int)
    ap.add_argument("--seq-len", type=int, dest="seq_len")
    ap.add_argument("--mlp-hidden", type=_tuple_ints, dest="mlp_hidden")
    ap.add_argument("--dropout", type=float)
    ap.add_argument("--device", choices=["auto", "cpu", "cuda"])
    ap.add_argument("--precision", choices=["bf16", "fp32"])
    ap.add_argument("--comm-dtype", dest="comm_dtype", choices=["fp32", "bf16"],
                    help="data-parallel gradient all-reduce precision (default fp32)")
    ap.add_argument("--group-col", dest="group_col")
    ap.add_argument("--window-split", dest="window_split", choices=["time", "random"])
    ap.add_argument("--synth-wells", type=int, dest="synth_wells")
    ap.add_argument("--synth-steps", type=int, dest="synth_steps")
    ap.add_argument("--online-chunk", type=int, dest="online_chunk")
    ap.add_argument("--max-steps", type=int, dest="max_steps")
    ap.add_argument("--resume", action="store_true", default=None)
    ap.add_argument("--verbose", type=int)
    ap.add_argument("--metrics", dest="metrics_path", help="append per-epoch JSON lines here")
    return ap


def parse_argv(model: str, argv) -> RunConfig:
    """argv excludes the program name (sys.argv[1:])."""
    if model not in MODEL_DEFAULTS:
        raise ValueError(f"unknown model {model!r}")
    ns = build_parser(model).parse_args(list(argv))
    cfg = RunConfig(model=model, **MODEL_DEFAULTS[model])
    cfg.column_names, cfg.column_types = ns.columnNames, ns.columnTypes
    cfg.target, cfg.storage_path = ns.targetColumn, ns.storagePath
    cfg.data = ns.data or ns.dataPath or "synth"
    for k, v in vars(ns).items():
        if k in ("columnNames", "columnTypes", "targetColumn", "storagePath", "dataPath", "data"):
            continue
        if v is not None and hasattr(cfg, k):
            setattr(cfg, k, v)
    env_fail = os.environ.get("WELLFLOW_FAIL_AT_STEP")
    if env_fail is not None:
        cfg.fail_at_step = int(env_fail)
    # elastic restarts (torchrun --max-restarts): a restarted worker resumes from .ckpt
    if int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0:
        cfg.resume = True
    return cfg
