"""Data-parallel correctness on CPU: gloo, world_size 2 and 4, launched through torchrun on
127.0.0.1 (SURVEY.md §4 distributed tier). The same code path runs RCCL on GPUs."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(tmp_path, body: str, nproc: int, timeout=300, extra_env=None, max_restarts=0):
    script = tmp_path / "worker.py"
    script.write_text(textwrap.dedent(f"""
        import json, os, sys
        sys.path.insert(0, {ROOT!r})
        import torch
        from wellflow.parallel.dist import DistContext
        OUT = {str(tmp_path)!r}
    """) + textwrap.dedent(body))
    env = dict(os.environ)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "1"
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           f"--max-restarts={max_restarts}", "--master-addr", "127.0.0.1", "--master-port",
           str(_free_port()), str(script)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [json.load(open(tmp_path / f"rank{i}.json")) for i in range(nproc)]


@pytest.mark.parametrize("world,kind", [(2, "mlp"), (4, "mlp"), (8, "mlp"), (2, "lstm"), (4, "cnn")])
def test_dp_step_equals_single_process_step(tmp_path, world, kind):
    res = _torchrun(tmp_path, """
        from wellflow.models.base import TorchEngine
        from wellflow.models.mlp import MLPRegressor
        from wellflow.models.lstm import LSTMRegressor
        from wellflow.models.cnn import CNN1DRegressor
        from wellflow.optim.flat import FlatAdam
        KIND = __KIND__
        def make():
            if KIND == "mlp":
                return MLPRegressor(6, (16, 8))
            if KIND == "lstm":
                return LSTMRegressor(6, 8)
            return CNN1DRegressor(input_len=10, in_ch=6, filters=4, kernel=3, outputs=1, dropout=0.0)
        def data(g):
            shape = (32, 6) if KIND == "mlp" else (32, 10, 6) if KIND == "cnn" else (32, 5, 6)
            return torch.randn(*shape, generator=g), torch.randn(32, generator=g)
        ctx = DistContext.from_env(device="cpu")
        W, r = ctx.world_size, ctx.rank
        torch.manual_seed(100 + r)               # different init on purpose ...
        eng = TorchEngine(make(), loss="mse")
        ctx.broadcast_(eng.params)               # ... C1 makes them identical
        opt = FlatAdam(eng.params, eng.grads, lr=1e-2)
        g = torch.Generator().manual_seed(0)
        X, Y = data(g)
        B = 32 // W
        for step in range(3):
            xb, yb = X[r * B:(r + 1) * B], Y[r * B:(r + 1) * B]
            eng.forward_backward(xb, yb, grad_scale=1.0 / 32)
            ctx.all_reduce_sum_(eng.grads)       # C2
            opt.step()
        # single-process reference on the full batch, from the broadcast init
        torch.manual_seed(100)
        ref = TorchEngine(make(), loss="mse")
        ropt = FlatAdam(ref.params, ref.grads, lr=1e-2)
        for step in range(3):
            ref.forward_backward(X, Y, grad_scale=1.0 / 32)
            ropt.step()
        err = (eng.params - ref.params).abs().max().item()
        json.dump({"err": err, "p0": eng.params[:5].tolist()}, open(f"{OUT}/rank{r}.json", "w"))
        ctx.shutdown()
    """.replace("__KIND__", repr(kind)), world)
    for rr in res:
        assert rr["err"] < 1e-5
    assert all(rr["p0"] == res[0]["p0"] for rr in res)


def test_dp_training_job_agrees_on_early_stop_and_rank0_writes(tmp_path):
    res = _torchrun(tmp_path, """
        from wellflow.train.job import run_job
        names = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
        types = "string,string,int,float,float,float,float,float,float,float"
        out = run_job("mlp", [names, types, "flow", OUT + "/store", "--epochs", "30", "--patience", "1",
                              "--synth-wells", "3", "--synth-steps", "120", "--batch-size", "16",
                              "--device", "cpu", "--lr", "0.05"], log=lambda *a, **k: None)
        r = int(os.environ["RANK"])
        json.dump({"epochs": out["epochs"], "test": out["test_loss"], "val": out["history"]["val_loss"]},
                  open(f"{OUT}/rank{r}.json", "w"))
    """, 2)
    assert res[0]["epochs"] == res[1]["epochs"]
    assert res[0]["val"] == res[1]["val"]
    assert abs(res[0]["test"] - res[1]["test"]) < 1e-9
    assert (tmp_path / "store" / "models" / "mlp.mdl").exists()


def test_elastic_restart_resumes_from_checkpoint(tmp_path):
    """torchrun --max-restarts=1: both ranks hit an injected fault once, the group is
    restarted, the workers see TORCHELASTIC_RESTART_COUNT=1, resume from the .ckpt and
    finish all epochs; the metrics JSONL holds one record per epoch."""
    res = _torchrun(tmp_path, """
        from wellflow.train.job import run_job
        names = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
        types = "string,string,int,float,float,float,float,float,float,float"
        out = run_job("mlp", [names, types, "flow", OUT + "/store", "--epochs", "4",
                              "--synth-wells", "3", "--synth-steps", "120", "--batch-size", "16",
                              "--device", "cpu", "--metrics", OUT + "/metrics.jsonl"],
                      log=lambda *a, **k: None)
        r = int(os.environ["RANK"])
        json.dump({"epochs": out["epochs"], "restart": os.environ.get("TORCHELASTIC_RESTART_COUNT")},
                  open(f"{OUT}/rank{r}.json", "w"))
    """, 2, extra_env={"WELLFLOW_FAIL_AT_STEP": "10"}, max_restarts=1)
    assert all(r["epochs"] == 4 for r in res)
    assert all(r["restart"] == "1" for r in res)
    assert (tmp_path / "store" / "models" / ".fault_injected_mlp_r0").exists()
    # 7 steps/epoch: the fault hits epoch 2, the restart resumes after epoch 1 (no replay)
    recs = [json.loads(l) for l in open(tmp_path / "metrics.jsonl")]
    assert [r["epoch"] for r in recs] == [1, 2, 3, 4]


@pytest.mark.parametrize("world,kind", [(2, "lstm"), (4, "mlp"), (4, "lstm")])
def test_dp_step_runner_equals_single_process_step(tmp_path, world, kind):
    """The PRODUCTION step object (train/step.py StepRunner: forward_backward -> C2 flat
    all-reduce -> fused optimizer, the one bench.py times and the Trainer drives) at world 2 / 4
    over gloo, graph off, against a single process running the same StepRunner on the
    concatenated batch. Every rank's parameters must equal the single-process ones after 3
    steps (round-2 verdict: the DP check ran a hand-written loop, not the StepRunner)."""
    res = _torchrun(tmp_path, """
        from wellflow.models.base import TorchEngine
        from wellflow.models.mlp import MLPRegressor
        from wellflow.models.lstm import LSTMRegressor
        from wellflow.optim.flat import FlatAdam
        from wellflow.train.step import StepRunner
        KIND = __KIND__
        N = 32
        def make():
            return MLPRegressor(6, (16, 8)) if KIND == "mlp" else LSTMRegressor(6, 8)
        g = torch.Generator().manual_seed(0)
        X = torch.randn(*((N, 6) if KIND == "mlp" else (N, 5, 6)), generator=g)
        Y = torch.randn(N, generator=g)
        ctx = DistContext.from_env(device="cpu")
        W, r = ctx.world_size, ctx.rank
        torch.manual_seed(100 + r)
        eng = TorchEngine(make(), loss="mse")
        ctx.broadcast_(eng.params)
        opt = FlatAdam(eng.params, eng.grads, lr=1e-2, zero_grads=True)
        B = N // W
        shards = [(X[(r * 3 + s) % W * B:((r * 3 + s) % W + 1) * B], Y[(r * 3 + s) % W * B:((r * 3 + s) % W + 1) * B])
                  for s in range(3)]
        run = StepRunner(eng, opt, ctx, 1.0 / N, lambda k: shards[k], graph=False)
        for s in range(3):
            run.run(s)
        loss = run.take_loss()
        ref_ctx = DistContext(device=torch.device("cpu"))
        torch.manual_seed(100)
        ref = TorchEngine(make(), loss="mse")
        ropt = FlatAdam(ref.params, ref.grads, lr=1e-2, zero_grads=True)
        rrun = StepRunner(ref, ropt, ref_ctx, 1.0 / N, lambda k: (X, Y), graph=False)
        for s in range(3):
            rrun.run(s)
        rloss = rrun.take_loss()
        err = (eng.params - ref.params).abs().max().item()
        (tot,) = ctx.sum_scalars(loss)
        json.dump({"err": err, "p0": eng.params[:5].tolist(), "loss": tot, "rloss": rloss},
                  open(f"{OUT}/rank{r}.json", "w"))
        ctx.shutdown()
    """.replace("__KIND__", repr(kind)), world)
    for rr in res:
        assert rr["err"] < 1e-5, rr
        assert abs(rr["loss"] - rr["rloss"]) < 1e-4 * abs(rr["rloss"]), rr
    assert all(rr["p0"] == res[0]["p0"] for rr in res)


@pytest.mark.parametrize("world,kind", [(2, "lstm"), (4, "mlp")])
def test_dp_bf16_comm_matches_fp32(tmp_path, world, kind):
    """C2 in bf16 (DistContext comm_dtype="bf16": the fp32 bucket rounded into a bf16 twin,
    reduced, widened back; SURVEY.md §2.5 "bf16 halves them"): the reduced gradient of one
    StepRunner step agrees with the fp32 reduction to bf16 rounding (relative L2 < 2^-7) and
    with the single-process gradient of the concatenated batch; every rank holds the same
    result; the twin is one buffer, reused by every step."""
    res = _torchrun(tmp_path, """
        from wellflow.models.base import TorchEngine
        from wellflow.models.mlp import MLPRegressor
        from wellflow.models.lstm import LSTMRegressor
        from wellflow.optim.flat import FlatSGD
        from wellflow.train.step import StepRunner
        KIND = __KIND__
        N = 32
        def make():
            return MLPRegressor(6, (16, 8)) if KIND == "mlp" else LSTMRegressor(6, 8)
        g = torch.Generator().manual_seed(0)
        X = torch.randn(*((N, 6) if KIND == "mlp" else (N, 5, 6)), generator=g)
        Y = torch.randn(N, generator=g)
        ctx = DistContext.from_env(device="cpu", comm_dtype="bf16")
        W, r = ctx.world_size, ctx.rank
        B = N // W
        xs, ys = X[r * B:(r + 1) * B], Y[r * B:(r + 1) * B]
        torch.manual_seed(100)
        eng = TorchEngine(make(), loss="mse")
        p0 = eng.params.clone()
        # lr 0: the step leaves the parameters alone and the reduced gradient in the bucket
        run = StepRunner(eng, FlatSGD(eng.params, eng.grads, lr=0.0, momentum=0.0), ctx, 1.0 / N,
                         lambda k: (xs, ys), graph=False)
        grads = []
        for s in range(2):
            run.run(s)
            grads.append(eng.grads.clone())
        g16 = grads[-1]
        ctx.comm_dtype = "fp32"
        eng.params.copy_(p0)
        run.run(2)
        g32 = eng.grads.clone()
        ref = TorchEngine(make(), loss="mse")
        ref.params.copy_(p0)
        ref.sync_weights() if hasattr(ref, "sync_weights") else None
        ref.forward_backward(X, Y, 1.0 / N)
        rel = lambda a, b: ((a - b).norm() / b.norm()).item()
        json.dump({"r16": rel(g16, g32), "rref": rel(g16, ref.grads), "r32": rel(g32, ref.grads),
                   "same": torch.equal(grads[0], grads[1]), "twins": len(ctx._lowp),
                   "g": g16[:6].tolist()}, open(f"{OUT}/rank{r}.json", "w"))
        ctx.shutdown()
    """.replace("__KIND__", repr(kind)), world)
    for rr in res:
        assert 0 < rr["r16"] < 2 ** -7, rr   # bf16 rounding, and the bf16 path really ran
        assert rr["rref"] < 2 ** -7 and rr["r32"] < 1e-5, rr
        assert rr["same"] and rr["twins"] == 1, rr
    assert all(rr["g"] == res[0]["g"] for rr in res)
