"""The production LSTM job pattern on the GPU: graph-replayed training epochs with the
evaluation's native prefetcher filling PINNED slots between them. In round 2 this drained
every persistent backward workgroup from epoch 2 on: the per-launch reset, a memset node
starting 4 B into its allocation, left 0x04040404 in the error word under graph replay
(profiles/r3_early_exit.md). The running completion totals must cover every launch."""
import pytest
import torch

pytestmark = pytest.mark.gpu

NAMES = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
TYPES = "string,string,int,float,float,float,float,float,float,float"


@pytest.mark.parametrize("pin", ["1", "0"])
def test_lstm_job_graph_replay_with_pinned_eval_completes(tmp_path, monkeypatch, pin):
    from wellflow.train.job import run_job

    monkeypatch.setenv("WELLFLOW_EVAL_PIN", pin)
    out = run_job("lstm", [NAMES, TYPES, "flow", str(tmp_path) + "/", "--epochs", "3", "--patience", "100",
                           "--synth-wells", "6", "--synth-steps", "6000", "--batch-size", "2048",
                           "--seq-len", "64", "--hidden", "512", "--device", "cuda", "--verbose", "0"],
                  log=lambda *a, **k: None)
    assert out["native"] and out["epochs"] == 3
    st = out["persistent"]
    steps = out["steps"]
    assert steps >= 6, out["steps"]
    for k in ("forward", "backward"):
        v = st[k]
        assert v["done"] == v["expect"] and v["started"] == v["expect_wg"] and v["exits"] == 0 and not v["sticky"], (k, v)
    # every training step ran one persistent backward launch; forwards also ran for evaluation
    assert st["backward"]["launches"] >= steps, st
    assert st["forward"]["launches"] > st["backward"]["launches"], st
    assert torch.isfinite(torch.tensor(out["test_loss"]))


def test_device_resident_evaluation_matches_host_path():
    """Trainer.evaluate on host arrays now moves the split to the device once (Trainer.resident)
    and reduces on the device: the same (loss, MSE) as the chunked host-array path it replaced,
    for the MLP (a plain table) and the LSTM (windows over rows), chunk boundaries included."""
    import numpy as np

    from wellflow.config import RunConfig
    from wellflow.data.features import SeriesWindows
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat
    from wellflow.models.mlp import NativeMLP, init_mlp_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.parallel.dist import DistContext
    from wellflow.train.trainer import Trainer

    dev = torch.device("cuda")
    ctx = DistContext(device=dev)
    rng = np.random.default_rng(3)
    cases = []
    eng = NativeMLP(16, (256, 256), 4096, device=dev)
    eng.params.copy_(init_mlp_flat(16, (256, 256), seed=1).to(dev))
    eng.sync_weights()
    X = rng.standard_normal((10000, 16)).astype(np.float32)
    Y = rng.standard_normal(10000).astype(np.float32)
    cases.append((eng, X, Y, "mlp"))
    eng2 = NativeLSTM(16, 512, 32, 1024, device=dev)
    eng2.params.copy_(init_lstm_flat(16, 512, seed=2).to(dev))
    eng2.sync_weights()
    rows = rng.standard_normal((6000, 16)).astype(np.float32)
    starts = np.arange(0, 6000 - 32, 2)
    W = SeriesWindows(rows, starts, 32)
    Yw = rng.standard_normal(len(starts)).astype(np.float32)
    cases.append((eng2, W, Yw, "lstm"))
    for eng, X, Y, name in cases:
        cfg = RunConfig(model=name, loss="mse")
        tr = Trainer(cfg, eng, FlatAdam(eng.params, eng.grads), ctx, name)
        dev_loss, dev_mse = tr.evaluate(X, Y)
        assert tr._idx, "the split was not made resident"
        tr.resident = lambda a, b: (a, b)  # the chunked host path
        host_loss, host_mse = tr.evaluate(X, Y)
        assert abs(dev_loss - host_loss) <= 1e-5 * abs(host_loss), (name, dev_loss, host_loss)
        assert abs(dev_mse - host_mse) <= 1e-5 * abs(host_mse), (name, dev_mse, host_mse)
