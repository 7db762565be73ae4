#!/usr/bin/env python3
"""Per-phase timeline of the one-launch MLP training step (csrc/mlp_step.hip): lane 0 of every
wave stamps s_memtime (shader cycles) at 13 phase boundaries of one pass when
WELLFLOW_MLP_STAMP=1 in a WF_DIAG build (WELLFLOW_DIAG_BUILD=1; the stamps change no result,
they only go to an unused scratch region) — the 128-row kernel (mlp2_step128_kernel, the
default; its 3rd pass) or, with WELLFLOW_MLP_STEP128=0, the 64-row one (its 5th chunk).

    WELLFLOW_MLP_STAMP=1 python tools/mlp_timeline.py [--batch 262144]

Prints, per phase, the mean / max over all waves of the cycles spent in it.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES128 = ["layer 1 + H1 store", "B2 wait", "layer 2 MFMA", "H2 epilogue + head partials",
             "B3 wait", "prediction + dy", "dZ2 + stage next X", "B4 wait + X prefetch", "dZ2 copy-out + db2",
             "dH1 MFMA", "dZ1", "dW1 + db1"]  # 12 intervals of 13 stamps
PHASES = ["chunk top", "layer 1 + H1 store", "B2 wait", "layer 2 MFMA", "H2 epilogue + head partials",
          "B3 wait", "dy + dZ2 + stage next X", "B4 wait", "X prefetch", "dH1 MFMA",
          "W2 issue + stores + dZ1 + sums", "dW1"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--features", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    os.environ.setdefault("WELLFLOW_MLP_STAMP", "1")
    import torch

    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat
    dev = torch.device("cuda")
    eng = NativeMLP(a.features, (256, 256), a.batch, device=dev)
    eng.params.copy_(init_mlp_flat(a.features, (256, 256), seed=0).to(dev))
    eng.sync_weights()
    x, y = synth_tabular_batch(a.batch, a.features, seed=1)
    x, y = x.to(dev).to(torch.bfloat16), y.to(dev)
    off = 64 * 9216 + 4 * 65536 + 256 * 8192 + 200 * 65536  # csrc/kernels.h kMlpRedSlab2Off + row 200
    for _ in range(a.steps):
        st = eng.red[off: off + 2 * 256 * 8 * 16].view(torch.int64)
        st.zero_()
        eng.forward_backward(x, y, 1.0 / a.batch)
        torch.cuda.synchronize()
    t = st.view(256, 8, 16)[:, :, :13].cpu().double()
    valid = (t > 0).all(dim=2)
    t = t[valid]
    d = t[:, 1:] - t[:, :-1]
    print(f"waves stamped: {int(valid.sum())}; chunk span mean {float((t[:, -1] - t[:, 0]).mean()):.0f} cycles")
    phases = PHASES128 if eng.w2t is not None else PHASES
    for i, name in enumerate(phases):
        print(f"{i:2d} {name:30s} mean {float(d[:, i].mean()):8.0f}  max {float(d[:, i].max()):8.0f}")


if __name__ == "__main__":
    main()
