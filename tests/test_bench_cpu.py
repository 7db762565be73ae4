"""bench.py contract at world size 1, 2 and 4 without GPUs (--device cpu: gloo + the fp32
reference model). The driver runs bench.py either under torch.distributed.run or as
`python bench.py --gpus N` (bench.py then spawns the N ranks itself); this rehearses
everything around the kernels for both: rendezvous on 127.0.0.1, C1 broadcast, C2
all-reduce, the barrier-bracketed timing, max over ranks, and exactly ONE JSON line from
rank 0 with the whole-job aggregate value."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, model, extra, torchrun=True):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    args = ["bench.py", "--gpus", str(world), "--steps", "3", "--warmup", "1", "--device", "cpu",
            "--model", model] + extra
    if world > 1 and torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [1, 2, 4])
def test_bench_json_contract_lstm(world):
    B = 4
    rec = _run(world, "lstm", ["--batch", str(B), "--seq", "6", "--hidden", "16"])
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == world and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == B * world and rec["config"]["parallelism"] == f"dp{world}"
    assert rec["config"]["seq_len"] == 6
    assert rec["metric"].startswith("rows/sec (whole node), LSTM seq64")
    # value is the whole-job aggregate: global rows per step / seconds per step
    assert rec["value"] == pytest.approx(B * world / (rec["ms_per_step"] / 1000.0), rel=1e-3)
    assert rec["dtype"] == "fp32" and "rehearsal" in rec["data"]  # never mistaken for the benchmark
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"


def test_bench_self_spawns_ranks():
    """`python bench.py --gpus 4` with no launcher: the parent starts 4 ranks itself
    (torch.distributed.run on 127.0.0.1) and exactly one JSON line comes back, n_gpus 4."""
    B = 4
    rec = _run(4, "lstm", ["--batch", str(B), "--seq", "6", "--hidden", "16"], torchrun=False)
    assert rec["n_gpus"] == 4 and rec["world_size"] == 4 and rec["config"]["parallelism"] == "dp4"
    assert rec["config"]["global_batch"] == 4 * B and rec["backend"] == "gloo"


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--steps", "1"],
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 2 and not r.stdout.strip()


def test_bench_json_contract_mlp_dp2():
    rec = _run(2, "mlp", ["--batch", "64"])
    assert rec["config"]["global_batch"] == 128 and rec["n_gpus"] == 2


def test_bench_refuses_without_gpu():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0"], capture_output=True,
                       text=True, env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 2 and not r.stdout.strip()


def test_bench_secondary_configs_dp2():
    """BASELINE.json:8-10 ride in the headline's JSON line: a nested "secondary" object, one
    entry per config with its own steps, ms/step, rows/s (whole-job aggregate) and timed
    seconds; the headline value stays the LSTM's."""
    B = 4
    rec = _run(2, "lstm", ["--batch", str(B), "--seq", "6", "--hidden", "16", "--secondary", "mlp,mlp_online,cnn"])
    assert rec["value"] == pytest.approx(B * 2 / (rec["ms_per_step"] / 1000.0), rel=1e-3)
    sec = rec["secondary"]
    assert set(sec) == {"mlp", "mlp_online", "cnn"}
    for m, v in sec.items():
        assert v["steps"] == 3 and v["warmup"] == 1 and v["global_batch"] == 2 * v["per_gpu_batch"]
        assert v["value"] == pytest.approx(v["global_batch"] / (v["ms_per_step"] / 1000.0), rel=1e-3), (m, v)
        assert v["timed_s"] == pytest.approx(v["ms_per_step"] * 3 / 1000.0, rel=1e-2)
        # round-5 VERDICT item 5: every secondary carries its OWN bucket's all-reduce time at
        # this world size (gloo here, RCCL on the GPU node) and its share of the step
        assert v["comm_ms"] is not None and v["comm_ms"] > 0, (m, v)
        assert v["grad_bucket_mb"] > 0 and v["comm_dtype"] == "fp32"
        assert v["comm_share"] == pytest.approx(v["comm_ms"] / v["ms_per_step"], rel=1e-2, abs=1e-3)
    assert rec["comm_ms"] is not None and rec["comm_ms"] > 0


def test_gpu_state_sampler_window_math():
    """utils/gpustate.py on a fake metrics table: sampled clock / power / temperature, the
    limiter residencies as fractions of the accumulation counter's delta, per-XCD clocks
    averaged, N/A placeholders skipped."""
    import time

    sys.path.insert(0, ROOT)
    from wellflow.utils.gpustate import GpuStateSampler

    n = {"k": 0}

    def fake(_h):
        n["k"] += 1
        k = n["k"]
        return {"current_gfxclks": [2000 + k, 2000 + k, "N/A"], "current_socket_power": 1000 + k,
                "temperature_hotspot": 70 + k % 3, "accumulation_counter": 100 * k,
                "ppt_residency_acc": 25 * k, "socket_thm_residency_acc": 0, "throttle_status": 1}

    s = GpuStateSampler.__new__(GpuStateSampler)
    s.period_s, s._h, s._get, s._samples, s._t0, s._thread = 0.005, object(), fake, [], None, None
    import threading

    s._stop = threading.Event()
    s.start()
    time.sleep(0.05)
    st = s.stop()
    assert st["samples"] >= 2
    assert 2000 < st["sclk_mhz"]["min"] <= st["sclk_mhz"]["max"] < 2000 + n["k"] + 1
    assert st["power_w"]["max"] > 1000 and 70 <= st["temp_hotspot_c"] <= 72
    assert st["throttle"]["ppt"] == 0.25 and st["throttle"]["socket_thm"] == 0.0
    assert st["throttle"]["throttle_status"] == 1
    off = GpuStateSampler.__new__(GpuStateSampler)
    off._h, off._thread = None, None
    assert not off.available and off.stop() is None


def test_bench_job_default_secondaries():
    """The submission API's own batches ride in the bench line too (CNN 20 windows, MLP and
    online MLP 256 rows): the secondary names map to (model, per-GPU batch)."""
    rec = _run(1, "lstm", ["--batch", "4", "--seq", "6", "--hidden", "16", "--secondary",
                           "cnn_b20,mlp_b256,mlp_online_b256"])
    sec = rec["secondary"]
    assert set(sec) == {"cnn_b20", "mlp_b256", "mlp_online_b256"}
    assert sec["cnn_b20"]["per_gpu_batch"] == 20 and "cnn" in sec["cnn_b20"]["metric"]
    assert sec["mlp_b256"]["per_gpu_batch"] == 256 and sec["mlp_online_b256"]["per_gpu_batch"] == 256
    assert all(v["value"] > 0 for v in sec.values())


def test_small_launch_steps_and_dp_secondaries():
    """The headline times exactly --steps (<= 256 per launch); a secondary's raised window runs
    the Trainer's 256-step launches. Under a DP world the job-default secondaries are left out
    of the automatic set (they show one-GPU paths)."""
    import argparse
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench._small_launch_steps(argparse.Namespace(min_timed_s=0.0, steps=20)) == 20
    assert bench._small_launch_steps(argparse.Namespace(min_timed_s=0.0, steps=1000)) == 256
    assert bench._small_launch_steps(argparse.Namespace(min_timed_s=0.1, steps=20)) == 256
    assert set(bench.SMALL_SECONDARY) <= set(bench.SECONDARY)
    assert bench._auto_secondary(True, 1) == list(bench.SECONDARY)
    assert bench._auto_secondary(True, 8) == ["mlp", "mlp_online", "cnn"]
    assert bench._auto_secondary(False, 1) == []
