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
