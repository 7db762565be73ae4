"""LSTM native step on a batch of the JOB's data (the well-log pipeline, as
tools/job_throughput.py builds it) next to a batch of the bench's data (synth_lstm_batch):
flat gradient vs an fp32 autograd reference (tests/test_numerics_gpu.py _Fp32LSTM, same
weights and batch), and the time of one native forward+backward on each.

Why: kernel-traced job runs showed the persistent backward at 0.53 ms per step against
1.76 ms in bench.py at the same shape. This checks that the job's backward is correct, and
whether the time difference follows the data."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_numerics_gpu import _Fp32LSTM, _cos, _rel  # noqa: E402

from wellflow.config import parse_argv  # noqa: E402
from wellflow.data.pipeline import prepare  # noqa: E402
from wellflow.data.synth import synth_lstm_batch  # noqa: E402
from wellflow.models.lstm import NativeLSTM, init_lstm_flat  # noqa: E402

NAMES = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
TYPES = "string,string,int,float,float,float,float,float,float,float"
B, T, H = 8192, 64, 512
cfg = parse_argv("lstm", [NAMES, TYPES, "flow", "/tmp/wellflow_jgc/", "--synth-wells", "6", "--synth-steps", "40000",
                          "--seq-len", str(T), "--hidden", str(H), "--batch-size", str(B)])
prep = prepare(cfg)
Xw, Yw = prep.train
F = prep.n_features
sel = torch.randperm(len(Xw), generator=torch.Generator().manual_seed(0))[:B].numpy()
dev = torch.device("cuda")
xj = torch.as_tensor(Xw[sel], dtype=torch.float32).to(dev)
yj = torch.as_tensor(Yw[sel], dtype=torch.float32).to(dev)
xs, ys = synth_lstm_batch(B, T, F, seed=0)
xs, ys = xs.to(dev), ys.to(dev)
flat = init_lstm_flat(F, H, seed=1).to(dev)

for name, x, y in (("job", xj, yj), ("bench", xs, ys)):
    eng = NativeLSTM(F, H, T, B, device=dev)
    eng.params.copy_(flat)
    eng.sync_weights()
    eng.forward_backward(x, y, 1.0 / B)
    torch.cuda.synchronize()
    g = eng.grads.clone()
    ts = []
    for _ in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.forward_backward(x, y, 1.0 / B)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ref = _Fp32LSTM(eng.lay, flat)
    L, _ = ref.loss_pred(x, y)
    (L / B).backward()
    gr = ref.flat.grad
    print(f"{name}: F={F} fwd+bwd {statistics.median(ts[1:]):.3f} ms, persistent fwd/bwd "
          f"{eng.last_forward_persistent}/{eng.last_backward_persistent}, error word {eng.persistent_error()}, "
          f"grad rel-L2 vs fp32 {_rel(g, gr):.3e}, cosine {_cos(g, gr):.6f}, |x| mean {x.abs().mean().item():.3f}, "
          f"|y| mean {y.abs().mean().item():.3f}", flush=True)
