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
            for n in (2, 4, 8):
                lo, hi = allreduce_us(n, nbytes, 7), allreduce_us(n, nbytes, 1)
                share_hi = hi / (ms * 1e3 + hi)
                eff_lo, eff_hi = ms * 1e3 / (ms * 1e3 + hi), ms * 1e3 / (ms * 1e3 + lo)
                flag = "comm > 5 %" if share_hi > 0.05 else ""
                print(f"| {name} | {ms:.3f} | {nbytes / 1e6:.3f} | {n} | {lo:.1f} .. {hi:.1f} | "
                      f"{lo / (ms * 1e3 + lo) * 100:.1f} .. {share_hi * 100:.1f} % | "
                      f"{eff_lo * 100:.1f} .. {eff_hi * 100:.1f} % | {flag} |")
    print("\nReading: the LSTM headline's 4.7 MB fp32 bucket costs at most ~2 % of its ~4 ms step, so "
          "its DP scaling is compute-bound by construction. The MLP/CNN steps are ~0.2 ms, so even "
          "a 0.28 MB all-reduce is dominated by the RCCL latency floor: those configs are flagged "
          "(> 5 %) and bf16 communication does not help them (latency, not bytes); the remedy "
          "there is a larger per-GPU batch (288 GB of HBM3E leaves room) so the fixed floor is "
          "amortised over more rows.")


if __name__ == "__main__":
    main()
