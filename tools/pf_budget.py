"""Per-term budget of the persistent LSTM forward (round-6 VERDICT item 1): WELLFLOW_PF_DBG
variants of lstm_fwd_persistent_kernel (a diagnostic build: WELLFLOW_DIAG_BUILD=<set>) timed
INTERLEAVED in one process — windows of 50 back-to-back launches, variants in turn, after
~0.5 s of warm-up launches — so every variant sees the same clock and thermal state (separate
processes drifted by +-5 %, profiles/r6/forward_budget.md).

    python tools/pf_budget.py 0,264192,2048 [rounds]   -> one line per variant: median / min ms

The production kernel is dbg 0. Timing-only variants (results garbage): 4 no C/S stores,
32 no A-fragment LDS reads, 8192 no cell math in the MFMA loop, 8224 = 8192 + 32, 131072 no
LDS-DMA after step 0, 139296 = 131072 + 8224 (bare MFMAs + hand-off + stores), 139300 = that
without C/S stores, 524288 no hand-off (no publish / poll / wait), 663584 / 663588 = 139296 /
139300 without the hand-off. A/B variants (results correct): 2048 accumulators in AGPRs +
copy (round 5), 262144 the round-5 publish delay, 264192 both (the round-5 kernel), 256
per-wave h pieces (no staging barrier), 8 the poll read one chunk after issue (PL = 1).
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
from wellflow.models.lstm import NativeLSTM, decode_pstat, init_lstm_flat, persistent_sync_buffer  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "0").split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
B, H, F, T = 8192, 512, 16, 64
eng = NativeLSTM(F, H, T, B, device="cuda")
eng.params.copy_(init_lstm_flat(F, H, seed=1).cuda())
eng.sync_weights()
x = torch.randn(B, T, F, device="cuda")
C, dims = eng._C, eng._dims(B)
C.lstm_pack_x(x, eng.XH, *dims, True)


# one sync buffer per variant: variants may publish a different number of times per launch
# (the publish delay), so they must not share the monotonic hand-off counters
syncs = {v: persistent_sync_buffer(B, 32, "cuda") for v in variants}


def launch(v: str, n: int) -> None:
    os.environ["WELLFLOW_PF_DBG"] = v  # read by the binding at every launch (lstm_dims)
    for _ in range(n):
        C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, syncs[v], *dims)


def stats(v: str) -> dict:
    return decode_pstat(syncs[v][-64:].cpu().tolist())


for v in variants:  # each variant once, checked, before any timing
    print(f"pf dbg{v}: launching", flush=True)
    launch(v, 1)
    torch.cuda.synchronize()
    st = stats(v)
    assert st["done"] == st["expect"], (v, st)
for _ in range(6):
    for v in variants:
        launch(v, 60 // len(variants) + 1)
torch.cuda.synchronize()
ts = {v: [] for v in variants}
waits = {v: 0 for v in variants}  # WF_DIAG: blocking hand-off waits (STAT word 20), per launch below
for _ in range(rounds):
    for v in variants:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        w0 = int(syncs[v][-64 + 20].item())
        os.environ["WELLFLOW_PF_DBG"] = v
        a.record()
        launch(v, 50)
        b.record()
        b.synchronize()
        ts[v].append(a.elapsed_time(b) / 50)
        waits[v] += int(syncs[v][-64 + 20].item()) - w0
os.environ["WELLFLOW_PF_DBG"] = "0"
for v in variants:
    st = stats(v)
    print(f"pf dbg{v} {statistics.median(ts[v]):.4f} {min(ts[v]):.4f} ms  waits/launch "
          f"{waits[v] / (50 * rounds):.1f}  "
          f"(rounds {' '.join('%.3f' % t for t in ts[v])})  launches {st['launches']} "
          f"incomplete {st['expect'] - st['done']}", flush=True)
