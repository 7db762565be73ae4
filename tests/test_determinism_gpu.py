"""Race detection by determinism (SURVEY.md §5 "Race detection / sanitizers"): GPU
AddressSanitizer is not available on this pool, so the device-side check is to run the
pipelined kernels twice on identical inputs and compare BITS. Every kernel whose output
is written by exactly one lane (GEMM mainloops with glds rings, the fused LSTM step
kernels, head, Adam) must reproduce bit-for-bit; a missing barrier / vmcnt wait in an
LDS ring shows up here as a run-to-run difference long before it shows in a tolerance
test. Outputs reduced with fp32 atomics (split-K dW, loss sums) only have a fixed set of
addends, so they are checked to a tight tolerance instead.

Also: a hipGraph replay of a full LSTM training step equals the eager step.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lstm(B=512, T=16, F=16, H=256, seed=0):
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(init_lstm_flat(F, H, seed=seed).to(DEV))
    eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F, seed=seed)
    return eng, x.to(DEV), y.to(DEV)


@pytest.mark.parametrize("fwd_variant,bwd_variant", [(0, 0), (6, 8)])
def test_lstm_step_bitwise_reproducible(fwd_variant, bwd_variant):
    eng, x, y = _lstm()
    eng.fwd_variant, eng.bwd_variant = fwd_variant, bwd_variant
    runs = []
    for _ in range(3):
        loss = eng.forward_backward(x, y, 1.0 / len(y)).clone()
        torch.cuda.synchronize()
        runs.append((eng.XH.clone(), eng.Cst.clone(), eng.S.clone(), eng.DG.clone(), eng.pred.clone(),
                     eng.grads.clone(), loss))
    for r in runs[1:]:
        for name, a, b in zip(("XH", "C", "S", "DG", "pred"), runs[0][:5], r[:5]):
            assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                               b.view(torch.int16) if b.dtype == torch.bfloat16 else b), name
        g0, g1 = runs[0][5], r[5]
        assert (g0 - g1).abs().max().item() <= 1e-5 * g0.abs().max().item() + 1e-9
        assert abs(runs[0][6].item() - r[6].item()) <= 1e-5 * abs(runs[0][6].item())


def test_gemm_glds_ring_bitwise_reproducible():
    from wellflow.ops.native import gemm

    torch.manual_seed(1)
    M, N, K = 1024, 768, 4096  # many K iterations through the 3-stage LDS ring
    A = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    Bm = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    outs = []
    for _ in range(3):
        o = torch.empty(M, N, device=DEV)
        gemm(A, Bm, M, N, K, outF=o)
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_lstm_graph_replay_equals_eager():
    from wellflow.optim.flat import FlatAdam

    eng_e, x, y = _lstm(seed=3)
    eng_g, _, _ = _lstm(seed=3)
    opt_e = FlatAdam(eng_e.params, eng_e.grads, lr=1e-3)
    opt_g = FlatAdam(eng_g.params, eng_g.grads, lr=1e-3)
    gs = 1.0 / len(y)

    def step_e():
        eng_e.forward_backward(x, y, gs)
        opt_e.step()
        eng_e.sync_weights()

    def body_g():
        eng_g.forward_backward(x, y, gs)
        opt_g.step()
        eng_g.sync_weights()

    # warm up both identically, then capture the graph one
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step_e()
            body_g()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body_g()
    # capture did not execute: replay == one more step
    for _ in range(3):
        step_e()
        g.replay()
    torch.cuda.synchronize()
    # split-K fp32 atomics make the summation order (not the math) vary between runs, and
    # Adam divides by sqrt(v): near-zero gradients turn 1e-7 grad noise into ~1e-6 param
    # noise. A broken capture (stale buffer, missing launch) moves params by >= lr = 1e-3.
    d = (eng_e.params - eng_g.params).abs().max().item()
    assert d <= 5e-5, d
