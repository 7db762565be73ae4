"""MODELED (not measured) data-parallel weak scaling of the bench configs on one 8-GPU MI355X node.

This sandbox exposes one GPU and 8-GPU runs belong to the round-end driver (SCALE_rNN.json),
so the multi-GPU columns here are a model, labelled as such everywhere they are quoted
(round-4 VERDICT item 5):

    t_step(N) = t_step(1) (measured, DP=1 bench line) + t_allreduce(N, S)
    t_allreduce(N, S) = L(N) + 2 (N - 1) / N * S / BW          (ring all-reduce, one flat bucket)

S is the per-step gradient bucket (fp32 master gradients, or bf16 with --comm-dtype bf16;
parallel/dist.py). The all-reduce runs after the optimizer-feeding gradient is complete
(nothing of the step is left to overlap it with: the LSTM dW GEMM is the last kernel of the
backward, the MLP/CNN gradients come out of one fused kernel), so it adds to the step.
Assumptions (none measured here): L(N) = 10 / 20 / 30 us at N = 2 / 4 / 8 (RCCL launch +
protocol floor for small messages); BW between one link (153 GB/s, a single ring) and seven
links (7 x 153 GB/s, RCCL's multi-channel rings over the fully connected xGMI mesh).
Rows flagged "comm > 5 %" are configs whose modeled communication exceeds 5 % of the step at
the pessimistic bandwidth.

The ONLINE (streamed) MLP is modeled differently (round-5 VERDICT weak #4): its mini-batch
crosses PCIe on a copy stream while the previous batch computes, so

    t_step(N) = max(t_copy(N), t_compute + t_allreduce(N, S))
    t_copy(N) = bytes_per_step / min(PCIe rate per GPU, host DRAM rate per socket / GPUs per socket)

with the DP=1 copy rate measured (~48 GB/s, profiles/r5/online_sampled_timing.log: 9.44 MB per
step in the 0.195-ms streamed step; compute alone 0.155 ms) and a host term for N concurrent
streams of pinned reads: N / 2 GPUs per socket (two sockets, NUMA-bound pools,
utils/numa.py) sharing 300 (pessimistic) .. 450 GB/s (optimistic) of DRAM read bandwidth per
socket (assumed, not measured here).

usage: python tools/dp_model.py [bench.json] > profiles/r5/dp_model.md
"""
import json
import sys

sys.path.insert(0, ".")
from wellflow.models.cnn import CnnLayout  # noqa: E402
from wellflow.models.lstm import init_lstm_flat  # noqa: E402
from wellflow.models.mlp import MlpLayout  # noqa: E402

LAT_US = {2: 10.0, 4: 20.0, 8: 30.0}
LINK_GBS = 153.0
ONLINE_BYTES = 9.44e6        # bf16 features + fp32 targets of one 262,144-row mini-batch
PCIE_GBS = 48.4              # measured DP=1 streamed copy rate (9.44 MB / 0.195 ms)
ONLINE_COMPUTE_MS = 0.155    # the same step with its batch resident (static MLP bench line)
HOST_GBS_PER_SOCKET = (300.0, 450.0)  # assumed DRAM read bandwidth per socket (pessimistic, optimistic)


def online_step_us(n: int, comm_us: float, host_gbs: float, ms_dp1: float) -> float:
    per_gpu = min(PCIE_GBS, host_gbs / max(1.0, n / 2.0))
    copy_us = ONLINE_BYTES / (per_gpu * 1e3)
    # at DP=1 the measured step is the copy-bound one: keep its measured value as the floor
    return max(ms_dp1 * 1e3, copy_us, ONLINE_COMPUTE_MS * 1e3 + comm_us)


def allreduce_us(n: int, nbytes: float, links: int) -> float:
    return LAT_US[n] + 2.0 * (n - 1) / n * nbytes / (links * LINK_GBS * 1e3)  # bytes / (B/us)


def main() -> None:
    src = sys.argv[1] if len(sys.argv) > 1 else "profiles/r4/bench_final3.json"
    d = json.load(open(src))
    sec = d.get("secondary", {})
    rows = [
        ("LSTM seq64 h512 (headline)", d["ms_per_step"], init_lstm_flat(16, 512, seed=0).numel()),
        ("Static MLP 16-256-256-1", sec["mlp"]["ms_per_step"], MlpLayout(16, (256, 256)).numel),
        ("Online MLP (streamed)", sec["mlp_online"]["ms_per_step"], MlpLayout(16, (256, 256)).numel),
        ("Reference CNN", sec["cnn"]["ms_per_step"], CnnLayout().numel),
    ]
    print("# Data-parallel scaling: **modeled, not measured**\n")
    print(f"DP=1 step times from `{src}` (measured, one MI355X). Everything else is the model in "
          "`tools/dp_model.py` (ring all-reduce of one flat bucket after the step; latency floor "
          "10/20/30 us at N=2/4/8; bandwidth 1 link = 153 GB/s (pessimistic) .. 7 links). "
          "Modeled weak-scaling efficiency = t(1) / t(N). The driver's SCALE_rNN.json is the "
          "measurement; this table is what to compare it against.\n")
    for dtype, bpe in (("fp32", 4), ("bf16", 2)):
        print(f"\n## comm_dtype {dtype}\n")
        print("| config | DP=1 ms/step | bucket MB | N | all-reduce us (1 link .. 7 links) | "
              "comm share of step | modeled efficiency | flag |")
        print("|---|---|---|---|---|---|---|---|")
        for name, ms, numel in rows:
            nbytes = numel * bpe
            if name.startswith("Online"):
                for n in (2, 4, 8):
                    lo, hi = allreduce_us(n, nbytes, 7), allreduce_us(n, nbytes, 1)
                    t_best = online_step_us(n, lo, HOST_GBS_PER_SOCKET[1], ms)
                    t_worst = online_step_us(n, hi, HOST_GBS_PER_SOCKET[0], ms)
                    share_hi = max(0.0, t_worst - ms * 1e3) / t_worst
                    flag = "comm > 5 %" if share_hi > 0.05 else ""
                    print(f"| {name} | {ms:.3f} | {nbytes / 1e6:.3f} | {n} | {lo:.1f} .. {hi:.1f} | "
                          f"hidden under the copy: +{max(0.0, t_best - ms * 1e3) / t_best * 100:.1f} .. "
                          f"+{share_hi * 100:.1f} % | {ms * 1e3 / t_worst * 100:.1f} .. "
                          f"{ms * 1e3 / t_best * 100:.1f} % | {flag} |")
                continue
            for n in (2, 4, 8):
                lo, hi = allreduce_us(n, nbytes, 7), allreduce_us(n, nbytes, 1)
                share_hi = hi / (ms * 1e3 + hi)
                eff_lo, eff_hi = ms * 1e3 / (ms * 1e3 + hi), ms * 1e3 / (ms * 1e3 + lo)
                flag = "comm > 5 %" if share_hi > 0.05 else ""
                print(f"| {name} | {ms:.3f} | {nbytes / 1e6:.3f} | {n} | {lo:.1f} .. {hi:.1f} | "
                      f"{lo / (ms * 1e3 + lo) * 100:.1f} .. {share_hi * 100:.1f} % | "
                      f"{eff_lo * 100:.1f} .. {eff_hi * 100:.1f} % | {flag} |")
    print("\nOnline rows: max(copy, compute + all-reduce) with the host-DRAM term; at 8 GPUs each socket "
          "feeds 4 streams of ~48 GB/s (~194 GB/s), inside the assumed 300-450 GB/s, so the copy stays "
          "PCIe-bound and the ~30-us all-reduce hides under it (0.155 + 0.03 < 0.195 ms).")
    print("\nReading: the LSTM headline's 4.7 MB fp32 bucket costs at most ~2 % of its ~4 ms step, so "
          "its DP scaling is compute-bound by construction. The MLP/CNN steps are ~0.2 ms, so even "
          "a 0.28 MB all-reduce is dominated by the RCCL latency floor: those configs are flagged "
          "(> 5 %) and bf16 communication does not help them (latency, not bytes). At the default "
          "per-GPU batch their DP=8 efficiency is therefore EXPECTED at ~80 % (static MLP ~83 %, CNN "
          "~78 %); a per-GPU batch that makes the floor <= 5 % of the step (static MLP ~1.6 M rows, "
          "CNN ~0.4 M windows: bench.py --batch) trades Adam steps per epoch for throughput and is "
          "not the default, because its val-MSE parity at that global batch is not established.")


if __name__ == "__main__":
    main()
