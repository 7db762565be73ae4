"""Kernel numerics on a real MI355X: every HIP op against a plain PyTorch fp32 reference.

GEMM checks use ASYMMETRIC operands and odd shapes (cdna_hip_programming.md §3: an
A = I / symmetric-B check hides a transposed C write).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _bf(x):
    return x.to(torch.bfloat16)


def _ref_gemm(A, B):  # A [M,K], B [N,K] logical, bf16 values in fp32 math
    return A.float() @ B.float().t()


@pytest.mark.parametrize("a_mn", [False, True])
@pytest.mark.parametrize("b_mn", [False, True])
@pytest.mark.parametrize("shape", [(128, 128, 64), (200, 72, 136), (256, 384, 512), (64, 8, 1000)])
def test_gemm_layouts(a_mn, b_mn, shape):
    from wellflow.ops.native import gemm

    M, N, K = shape
    if a_mn and M % 8:
        pytest.skip("MN-contiguous needs M % 8 == 0")
    torch.manual_seed(0)
    A = _bf(torch.randn(M, K, device=DEV) + 0.1 * torch.arange(K, device=DEV) / K)
    B = _bf(torch.randn(N, K, device=DEV) * torch.linspace(0.5, 2.0, N, device=DEV)[:, None])
    Ast = A.t().contiguous() if a_mn else A
    Bst = B.t().contiguous() if b_mn else B
    out = torch.empty(M, N, device=DEV)
    gemm(Ast, Bst, M, N, K, a_mn=a_mn, b_mn=b_mn, outF=out)
    torch.cuda.synchronize()
    ref = _ref_gemm(A, B)
    err = (out - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item() + 1e-3, err


def test_gemm_identity_asymmetric():
    from wellflow.ops.native import gemm

    M = N = K = 128
    A = _bf(torch.eye(M, device=DEV))
    Bm = _bf(torch.arange(N * K, device=DEV, dtype=torch.float32).view(N, K) % 97 - 48)
    out = torch.empty(M, N, device=DEV)
    gemm(A, Bm, M, N, K, outF=out)
    torch.cuda.synchronize()
    assert torch.equal(out, Bm.float().t())


def test_gemm_epilogue_bias_relu_colsum_bf16():
    from wellflow.ops.native import gemm

    M, N, K = 300, 256, 40
    torch.manual_seed(1)
    A, B = _bf(torch.randn(M, K, device=DEV)), _bf(torch.randn(N, K, device=DEV))
    bias = torch.randn(N, device=DEV)
    outH = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    cs = torch.zeros(N, device=DEV)
    gemm(A, B, M, N, K, outH=outH, bias=bias, act=1, colsum=cs)
    torch.cuda.synchronize()
    ref = torch.relu(_ref_gemm(A, B) + bias)
    assert (outH.float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()
    assert torch.allclose(cs, ref.sum(0), rtol=2e-2, atol=1e-1)


def test_gemm_mask_and_splitk_atomic():
    from wellflow.ops.native import gemm

    M, N, K = 256, 256, 4096
    torch.manual_seed(2)
    A, B = _bf(torch.randn(M, K, device=DEV)), _bf(torch.randn(N, K, device=DEV))
    out = torch.zeros(M, N, device=DEV)
    gemm(A.t().contiguous(), B.t().contiguous(), M, N, K, a_mn=True, b_mn=True, outF=out,
         atomic=True, ksplit=8, alpha=0.5)
    mask = _bf(torch.randn(M, N, device=DEV))
    outm = torch.empty(M, N, device=DEV)
    gemm(A, B, M, N, K, outF=outm, mask=mask, mask_scale=2.0)
    torch.cuda.synchronize()
    ref = _ref_gemm(A, B)
    assert torch.allclose(out, 0.5 * ref, rtol=1e-3, atol=5e-2)
    refm = torch.where(mask.float() > 0, 2.0 * ref, torch.zeros_like(ref))
    assert torch.allclose(outm, refm, rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("F,H,T,B,ksplit", [(9, 128, 12, 96, 0), (16, 512, 4, 64, 0), (16, 512, 3, 256, 3)])
def test_lstm_forward_backward_matches_torch(F, H, T, B, ksplit):
    """(16, 512, ...) exercises the persistent forward and the 128x288 split-K dW tile."""
    from wellflow.models.lstm import LSTMRegressor, LstmLayout, NativeLSTM

    torch.manual_seed(3)
    ref = LSTMRegressor(F, H).to(DEV)
    x = torch.randn(B, T, F, device=DEV)
    y = torch.randn(B, device=DEV)
    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.dw_ksplit = ksplit
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()

    pred = eng.forward(x).clone()
    rp = ref(x)
    assert (pred - rp).abs().max().item() < 3e-2, (pred - rp).abs().max().item()

    loss_sum = eng.forward_backward(x, y, grad_scale=1.0 / B)
    torch.cuda.synchronize()
    loss = ((rp - y) ** 2).mean()
    assert abs(loss_sum.item() / B - loss.item()) < 2e-2 * loss.item() + 1e-3
    ref.zero_grad()
    loss.backward()
    # reference grads in flat layout
    lay = LstmLayout(F, H)
    gref = torch.zeros(lay.numel, device=DEV)
    W, w_out, b_out = lay.views(gref)
    nat = torch.zeros(lay.G, lay.KA, device=DEV)
    nat[:, :F] = ref.lstm.weight_ih_l0.grad
    nat[:, F] = ref.lstm.bias_ih_l0.grad
    nat[:, lay.KX:] = ref.lstm.weight_hh_l0.grad
    W.copy_(nat[lay.perm().to(DEV)])
    w_out.copy_(ref.head.weight.grad.view(-1))
    b_out.copy_(ref.head.bias.grad)
    g = eng.grads
    rel = (g - gref).norm() / gref.norm()
    assert rel.item() < 3e-2, rel.item()
    cos = torch.nn.functional.cosine_similarity(g, gref, dim=0)
    assert cos.item() > 0.999


def test_adam_and_sgd_match_reference():
    from wellflow.ops.native import lib

    C = lib()
    n = 1001
    torch.manual_seed(4)
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=1e-3)
    for step in range(1, 4):
        C.adam(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1 - 0.9 ** step, 1 - 0.999 ** step, 1.0)
        pr.grad = g.clone()
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, pr.detach(), atol=1e-6)
    # Keras-0.x Nesterov SGD
    p2, vel = torch.randn(n, device=DEV), torch.zeros(n, device=DEV)
    pc, vc = p2.clone(), vel.clone()
    for it in range(3):
        lr_t = 0.01 / (1 + 1e-6 * it)
        C.sgd(p2, g, vel, lr_t, 0.99, True, 1.0)
        vc = 0.99 * vc - lr_t * g
        pc = pc + 0.99 * vc - lr_t * g
    torch.cuda.synchronize()
    assert torch.allclose(p2, pc, atol=1e-6)


@pytest.mark.parametrize("n", [1001, 70401, 3_000_001])
def test_fused_device_adam(n):
    """Graph-capturable Adam (device step counter advanced by the last workgroup, bf16 shadow
    written and the gradient bucket cleared in the same launch) vs torch.optim.Adam fp32."""
    from wellflow.optim.flat import FlatAdam

    torch.manual_seed(5)
    p = torch.randn(n, device=DEV)
    g = torch.zeros(n, device=DEV)
    shadow = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    # + a transposed bf16 copy of one [rows][cols] block at an unaligned offset (MLP W2^T)
    t_off, t_r, t_c = 7, 24, 40
    shadow_t = torch.empty(t_r * t_c, dtype=torch.bfloat16, device=DEV)
    opt = FlatAdam(p, g, lr=1e-3, shadow=shadow, zero_grads=True, shadow_t=(shadow_t, t_off, t_r, t_c))
    pr = p.clone().requires_grad_(True)
    ref = torch.optim.Adam([pr], lr=1e-3)
    for step in range(1, 6):
        gs = torch.randn(n, device=DEV)
        g.add_(gs)  # the bucket was cleared by the previous update
        opt.step()
        pr.grad = gs.clone()
        ref.step()
        torch.cuda.synchronize()
        assert opt.step_dev[0].item() == float(step) and opt.step_dev[1].item() == 0.0
        assert g.abs().max().item() == 0.0
    assert torch.allclose(p, pr.detach(), atol=1e-6, rtol=1e-5)
    assert torch.equal(shadow, p.to(torch.bfloat16))
    want_t = p[t_off : t_off + t_r * t_c].view(t_r, t_c).t().contiguous().to(torch.bfloat16).view(-1)
    assert torch.equal(shadow_t, want_t)


def test_losses():
    from wellflow.ops.native import lib

    C = lib()
    B, O = 37, 12
    torch.manual_seed(5)
    pred = torch.randn(B, O, device=DEV) * 5
    y = torch.randn(B, O, device=DEV) * 5
    for kind in (0, 1):
        ls = torch.zeros(1, device=DEV)
        d = torch.empty(B, O, dtype=torch.bfloat16, device=DEV)
        cs = torch.zeros(O, device=DEV)
        scale = 1.0 / (B * O)
        C.loss(kind, pred, y, B, O, 6.0, scale, ls, d, None, cs)
        pr = pred.clone().requires_grad_(True)
        if kind == 0:
            L = ((pr - y) ** 2).sum()
        else:
            L = torch.clamp((y - pr).abs(), 0, 6).sum()
        L.backward()
        torch.cuda.synchronize()
        assert abs(ls.item() - L.item()) < 1e-3 * abs(L.item()) + 1e-3
        assert torch.allclose(d.float(), pr.grad * scale, rtol=1e-2, atol=1e-4)
        assert torch.allclose(cs, (pr.grad * scale).sum(0), rtol=1e-2, atol=1e-4)


@pytest.mark.parametrize("B,H,T,F", [(8192, 512, 8, 16), (512, 256, 6, 16), (256, 128, 5, 16), (2048, 512, 64, 16),
                                     (16384, 512, 4, 16), (12288, 512, 3, 16),
                                     # KX = 128 (64 <= F <= 127): one-hot-heavy feature vectors
                                     (8192, 512, 6, 100), (1024, 512, 4, 100), (2048, 256, 5, 64), (512, 128, 4, 127)])
def test_lstm_persistent_forward_matches_per_step(B, H, T, F):
    """The one-launch persistent forward (csrc/lstm_persistent.hip) must reproduce the
    per-step kernels: same MFMA k-order per output, so h/C/S agree to the last bf16 ulp
    apart from transcendental rounding (tolerance), and its spin bound must not trip.
    B > 8192 at H = 512 runs as consecutive sub-batch launches (no batch cap)."""
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(init_lstm_flat(F, H, seed=1).to(DEV))
    eng.sync_weights()
    x, _ = synth_lstm_batch(B, T, F, seed=2)
    x = x.to(DEV)
    C = eng._C
    dims = eng._dims(B)
    C.lstm_pack_x(x, eng.XH, *dims, True)
    C.lstm_forward(eng.XH, eng.Wp, eng.Cst, eng.S, eng.dcarry, *dims, 6)
    ref = (eng.XH.clone(), eng.Cst.clone(), eng.S.clone())
    eng.XH[B * eng.lay.KA:].zero_()
    C.lstm_pack_x(x, eng.XH, *dims, True)
    eng.Cst[B * H:].zero_()
    eng.S.zero_()
    ok = C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *dims)
    torch.cuda.synchronize()
    assert ok, "persistent launch refused"
    assert eng.lay.KX == (64 if F < 64 else 128)
    assert eng.persistent_error() == 0, "spin bound tripped"
    for name, a, b in zip(("XH", "C", "S"), (eng.XH, eng.Cst, eng.S), ref):
        d = (a.float() - b.float()).abs().max().item()
        assert d <= 2e-2, (name, d)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("ksplit", [1, 4])
@pytest.mark.parametrize("N", [576, 192])
def test_weight_gradient_tiles_match_reference(tile, ksplit, N):
    """Every split-K MN x MN weight-gradient tile (128x128, 256x128, 128x288, the
    rotation-swizzled 256x192 with its 64-deep 2-stage ring, 5- and 4-slot 32-deep rings and
    staggered wave groups, and the default 256x288 32-deep ring) against fp32 torch, on the
    LSTM dW shape family (N = KA: 576 at H = 512, 192 at H = 128, where tile 7 takes 256x192)."""
    from wellflow.ops.native import gemm

    torch.manual_seed(7)
    M, K = 512, 2048
    Amn = _bf(torch.randn(K, M, device=DEV))                     # A(m, k) = Amn[k, m]
    # one spare k-row: the whole-tile paths may read the last row up to a 128-column boundary
    # (binding.cpp glds_ok), so N = 192 takes the direct-to-LDS tiles too
    Bmn = _bf(torch.randn(K + 1, N, device=DEV) * torch.linspace(0.5, 2, N, device=DEV))
    out = torch.zeros(M, N, device=DEV)
    gemm(Amn, Bmn, M, N, K, a_mn=True, b_mn=True, outF=out, atomic=True, ksplit=ksplit, tile=tile)
    torch.cuda.synchronize()
    ref = Amn.float().t() @ Bmn[:K].float()
    err = (out - ref).abs().max().item()
    assert err < 2e-3 * ref.abs().max().item(), (tile, err)


@pytest.mark.parametrize("B,H,T,F", [(8192, 512, 8, 16), (512, 256, 6, 16), (256, 128, 5, 16), (2048, 512, 64, 16),
                                     (16384, 512, 4, 16), (8192, 512, 6, 100)])
def test_lstm_persistent_backward_matches_per_step(B, H, T, F):
    """The one-launch persistent BPTT (csrc/lstm_persistent_bwd.hip) against the per-step
    backward kernels on the same forward state: the K-split dh partials are summed in a
    different fp32 order, so DG agrees to bf16 rounding and the weight gradient closely."""
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(init_lstm_flat(F, H, seed=4).to(DEV))
    eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F, seed=5)
    x, y = x.to(DEV), y.to(DEV)
    res = {}
    for pb in (False, True):
        eng.persistent_bwd = pb
        eng.forward_backward(x, y, grad_scale=1.0 / B)
        torch.cuda.synchronize()
        if pb:
            assert eng.last_backward_persistent, "persistent backward refused"
            assert eng.persistent_error() == 0, "spin bound tripped"
            assert int(eng.sync_bwd[16].item()) > 0, "persistent backward did not run"
        res[pb] = (eng.DG.clone(), eng.grads.clone())
    (dg0, g0), (dg1, g1) = res[False], res[True]
    scale = dg0.float().abs().max().item()
    d = (dg0.float() - dg1.float()).abs().max().item()
    assert d <= 2e-2 * scale + 1e-6, (d, scale)
    rel = ((g0 - g1).norm() / g0.norm()).item()
    assert rel < 5e-3, rel


def test_persistent_timeout_is_sticky_and_raises(monkeypatch):
    """A hand-off wait that times out must not be silent (round-1 advice): with a diagnostic
    spin bound of 1 poll the persistent kernels drain early, the STICKY word survives the
    next launch's reset, check_device_errors() raises, and the StepRunner raises on its
    first steps. After reset_device_errors() and the normal bound, steps are clean again."""
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.parallel.dist import DistContext
    from wellflow.train.step import StepRunner

    B, T, F, H = 8192, 8, 16, 512
    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(init_lstm_flat(F, H, seed=0).to(DEV))
    eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F, seed=0)
    x, y = x.to(DEV), y.to(DEV)
    monkeypatch.setenv("WELLFLOW_SPIN_LIMIT", "1")
    monkeypatch.setenv("WELLFLOW_FORCE_TIMEOUT", "1")
    eng.forward_backward(x, y, 1.0 / B)
    torch.cuda.synchronize()
    assert eng.persistent_error() != 0, "an unreachable target with a 1-poll spin bound must trip"
    monkeypatch.delenv("WELLFLOW_SPIN_LIMIT")
    monkeypatch.delenv("WELLFLOW_FORCE_TIMEOUT")
    eng.forward_backward(x, y, 1.0 / B)  # a clean launch: resets its per-launch block, keeps the STAT block
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="spin bound"):
        eng.check_device_errors()
    eng.reset_device_errors()
    eng.forward_backward(x, y, 1.0 / B)
    torch.cuda.synchronize()
    eng.check_device_errors()
    # the production step raises on its first steps
    monkeypatch.setenv("WELLFLOW_SPIN_LIMIT", "1")
    monkeypatch.setenv("WELLFLOW_FORCE_TIMEOUT", "1")
    opt = FlatAdam(eng.params, eng.grads, lr=1e-3, zero_grads=True)
    run = StepRunner(eng, opt, DistContext(device=torch.device(DEV)), 1.0 / B, lambda k: (x, y), graph=False)
    with pytest.raises(RuntimeError, match="spin bound"):
        run.run()
    monkeypatch.delenv("WELLFLOW_SPIN_LIMIT")
    monkeypatch.delenv("WELLFLOW_FORCE_TIMEOUT")
    eng.reset_device_errors()


def test_persistent_completion_counters():
    """The persistent kernels keep RUNNING completion totals (csrc/persistent_guard.h): steps
    done vs grid x steps expected and workgroups started vs launched, over every launch and
    sub-batch since the last reset. Equal after clean steps; a short count in an EARLIER
    launch is still caught after later clean launches (round-2 advice: the old per-launch
    count was erased by the next launch); reset clears it."""
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    B, T, F, H = 16384, 8, 16, 512  # two sub-batch launches per pass at H = 512
    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(init_lstm_flat(F, H, seed=0).to(DEV))
    eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F, seed=0)
    x, y = x.to(DEV), y.to(DEV)
    eng.forward_backward(x, y, 1.0 / B)
    torch.cuda.synchronize()
    assert eng.last_forward_persistent and eng.last_backward_persistent
    st = eng.persistent_stats()
    fw, bw = st["forward"], st["backward"]
    assert fw["launches"] == 2 and bw["launches"] == 2, st
    assert fw["expect"] > 0 and fw["done"] == fw["expect"] and fw["expect"] % T == 0, fw
    assert bw["expect"] > 0 and bw["done"] == bw["expect"] and bw["expect"] % (T - 1) == 0, bw
    assert fw["started"] == fw["expect_wg"] and bw["started"] == bw["expect_wg"], st
    eng.check_device_errors()
    eng.sync_bwd[-64 + 1] -= T - 1  # one workgroup of this pass "left early"
    for _ in range(2):  # later clean passes do not erase it
        eng.forward_backward(x, y, 1.0 / B)
    torch.cuda.synchronize()
    assert eng.persistent_stats()["backward"]["launches"] == 6
    with pytest.raises(RuntimeError, match="backward .*completed"):
        eng.check_device_errors()
    eng.reset_device_errors()
    eng.forward_backward(x, y, 1.0 / B)
    torch.cuda.synchronize()
    eng.check_device_errors()


def test_persistent_exit_record(monkeypatch):
    """An early exit leaves a record (block, step, reason, words seen) in the STAT block: with
    a 1-poll spin bound the first exiting wave says why (its own bound, or the error word
    another workgroup's bound set)."""
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    B, T, F, H = 8192, 8, 16, 512
    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(init_lstm_flat(F, H, seed=0).to(DEV))
    eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F, seed=0)
    # an unreachable hand-off target + a 1-poll bound: the exit no longer depends on the grid's
    # timing (a faster step top left every workgroup inside a 1-poll bound)
    monkeypatch.setenv("WELLFLOW_SPIN_LIMIT", "1")
    monkeypatch.setenv("WELLFLOW_FORCE_TIMEOUT", "1")
    eng.forward_backward(x.to(DEV), y.to(DEV), 1.0 / B)
    torch.cuda.synchronize()
    monkeypatch.delenv("WELLFLOW_SPIN_LIMIT")
    monkeypatch.delenv("WELLFLOW_FORCE_TIMEOUT")
    fw = eng.persistent_stats()["forward"]
    assert fw["sticky"] == 1 and fw["exits"] > 0 and fw["done"] < fw["expect"], fw
    rec = fw["first_exit"]
    assert rec is not None and rec["reason"] in (1, 2, 4) and 1 <= rec["step"] < T, rec
    eng.reset_device_errors()


def test_persistent_sync_signature_mismatch_fails_loudly():
    """Round-5 ADVICE: the hand-off epoch targets assume every launch on one sync buffer had the
    same (row tiles per workgroup, steps, column blocks). A launch of another shape on a buffer
    that is not re-zeroed must fail LOUDLY (exit reason 5, check_device_errors raises) instead
    of reading unpublished h; after reset_device_errors the new shape runs clean."""
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    B, T, F, H = 8192, 8, 16, 512
    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(init_lstm_flat(F, H, seed=0).to(DEV))
    eng.sync_weights()
    x, _ = synth_lstm_batch(B, T, F, seed=0)
    C = eng._C
    C.lstm_pack_x(x.to(DEV), eng.XH, *eng._dims(B), True)
    assert C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *eng._dims(B))
    torch.cuda.synchronize()
    assert eng.persistent_error() == 0
    short = (B, T - 3, F, eng.lay.KX, H)  # same buffers, fewer steps: another signature
    assert C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *short)
    torch.cuda.synchronize()
    fw = eng.persistent_stats()["forward"]
    assert fw["sticky"] == 1 and fw["done"] < fw["expect"], fw
    assert fw["first_exit"] is not None and fw["first_exit"]["reason"] == 5, fw
    with pytest.raises(RuntimeError):
        eng.check_device_errors()
    eng.reset_device_errors()
    assert C.lstm_forward_persistent(eng.XH, eng.Wp, eng.Cst, eng.S, eng.sync, *short)
    torch.cuda.synchronize()
    assert eng.persistent_error() == 0
    eng.reset_device_errors()


def test_diag_env_ignored_by_production_build(monkeypatch):
    """A production _C.so ignores the timing-only switches (round-3 VERDICT item 2):
    WELLFLOW_PF_DBG=1 (skip the persistent hand-off wait) and WELLFLOW_MLP_DBG=1 (skip the
    MLP epilogue atomics) set, the LSTM and MLP steps still match their fp32 references and
    the LSTM steps give bit-for-bit the same forward as without the variables."""
    from wellflow.data.synth import synth_lstm_batch, synth_tabular_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat
    from wellflow.models.mlp import MLPRegressor, NativeMLP
    from wellflow.ops.native import lib
    from wellflow.train.parity import Fp32LSTM

    assert not lib().diag_build(), "the tested _C.so must be the production build"
    B, T, F, H = 8192, 16, 16, 512
    eng = NativeLSTM(F, H, T, B, device=DEV)
    flat = init_lstm_flat(F, H, seed=2).to(DEV)
    eng.params.copy_(flat)
    eng.sync_weights()
    x, y = synth_lstm_batch(B, T, F, seed=3)
    x, y = x.to(DEV), y.to(DEV)
    eng.forward_backward(x, y, 1.0 / B)
    torch.cuda.synchronize()
    clean = eng.pred[:B].clone()
    for k, v in {"WELLFLOW_PF_DBG": "1", "WELLFLOW_MLP_DBG": "3"}.items():
        monkeypatch.setenv(k, v)
    ls = eng.forward_backward(x, y, 1.0 / B).item()
    torch.cuda.synchronize()
    eng.check_device_errors()
    assert eng.last_forward_persistent and eng.last_backward_persistent
    assert torch.equal(eng.pred[:B], clean), "WELLFLOW_PF_DBG changed the production forward"
    ref = Fp32LSTM(eng.lay, flat)
    L, pred_r = ref.loss_pred(x, y)
    (L / B).backward()
    assert ((eng.pred[:B] - pred_r.detach()).norm() / pred_r.norm()).item() < 2e-2
    assert abs(ls - L.item()) <= 2e-2 * L.item()
    g_r = ref.flat.grad
    assert ((eng.grads - g_r).norm() / g_r.norm()).item() < 3e-2
    # MLP (fused 8-wave kernels, spread reduction) under WELLFLOW_MLP_DBG
    Bm, Fm = 65536, 16
    torch.manual_seed(0)
    mref = MLPRegressor(Fm, (256, 256)).to(DEV)
    meng = NativeMLP(Fm, (256, 256), Bm, device=DEV)
    meng.params.copy_(mref.to_flat().to(DEV))
    meng.sync_weights()
    xm, ym = synth_tabular_batch(Bm, Fm, seed=4)
    xm, ym = xm.to(DEV), ym.to(DEV)
    lm = meng.forward_backward(xm, ym, 1.0 / Bm).item()
    torch.cuda.synchronize()
    pred = mref(xm)
    Lm = ((pred - ym) ** 2).sum()
    (Lm / Bm).backward()
    assert abs(lm - Lm.item()) <= 2e-2 * Lm.item()
    gref = MLPRegressor(Fm, (256, 256))
    for pr, pg in zip(gref.parameters(), mref.parameters()):
        pr.data.copy_(pg.grad.cpu())
    g_m = gref.to_flat().to(DEV)
    assert ((meng.grads - g_m).norm() / g_m.norm()).item() < 3e-2


def test_persistent_sync_buffer_at_offset_under_graph_replay():
    """The rule behind the round-2 early exit (profiles/r3_early_exit.md): the per-launch reset
    is ONE memset node that must start 16-B aligned and cover a multiple of 16 B — not "start
    its own allocation". Both sync buffers are placed at non-zero, 16-B aligned offsets inside
    larger allocations (256 B and 16 B in), the step is captured and replayed, and every
    persistent launch completes every step (STAT block) with the same parameters as buffers at
    the start of their own allocations."""
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat
    from wellflow.optim.flat import FlatAdam
    from wellflow.parallel.dist import DistContext
    from wellflow.train.step import StepRunner

    B, T, F, H = 8192, 16, 16, 512
    x, y = synth_lstm_batch(B, T, F, seed=7)
    x, y = x.to(DEV), y.to(DEV)
    out = {}
    for offset in (False, True):
        eng = NativeLSTM(F, H, T, B, device=DEV)
        eng.params.copy_(init_lstm_flat(F, H, seed=6).to(DEV))
        eng.sync_weights()
        if offset:
            n_f, n_b = eng.sync.numel(), eng.sync_bwd.numel()
            big_f = torch.zeros(n_f + 64, dtype=torch.int32, device=DEV)
            big_b = torch.zeros(n_b + 64, dtype=torch.int32, device=DEV)
            eng.sync, eng.sync_bwd = big_f[64:64 + n_f], big_b[4:4 + n_b]
            assert eng.sync.data_ptr() % 512 != 0 or eng.sync_bwd.data_ptr() % 512 != 0
            assert eng.sync.data_ptr() % 16 == 0 and eng.sync_bwd.data_ptr() % 16 == 0
        opt = FlatAdam(eng.params, eng.grads, lr=1e-3, zero_grads=True)
        run = StepRunner(eng, opt, DistContext(device=torch.device(DEV)), 1.0 / B, lambda k: (x, y), graph=True)
        for _ in range(8):  # 2 eager steps, then the capture and 6 replays (the capture itself runs nothing)
            run.run()
        torch.cuda.synchronize()
        assert run.graphs
        eng.check_device_errors()
        st = eng.persistent_stats()
        assert st["forward"]["launches"] == 8 and st["backward"]["launches"] == 8, st
        out[offset] = eng.params.clone()
    d = (out[False] - out[True]).abs().max().item()
    assert d <= 5e-5, d


@pytest.mark.parametrize("shape,dtype", [((100003, 16), torch.bfloat16), ((50001,), torch.float32),
                                         ((7777, 3), torch.float32), ((4096, 32), torch.bfloat16)])
def test_gather_rows_matches_index_select(shape, dtype):
    """csrc/elementwise.hip gather_rows (the trainer's per-epoch shuffle copy) against
    torch.index_select: bit-identical rows for 32-B / 64-B rows (16-B pieces) and 4-B / 12-B rows
    (4-B pieces); ids are clamped to the table."""
    from wellflow import _C

    src = torch.randn(shape, device="cuda").to(dtype)
    n = shape[0]
    idx = torch.randint(0, n, (n // 2 + 3,), device="cuda")
    out = torch.empty((len(idx),) + tuple(shape[1:]), dtype=dtype, device="cuda")
    _C.gather_rows(src, idx, out)
    assert torch.equal(out, src.index_select(0, idx))
    idx2 = torch.tensor([-5, 0, n - 1, n + 7], device="cuda")
    out2 = torch.empty((4,) + tuple(shape[1:]), dtype=dtype, device="cuda")
    _C.gather_rows(src, idx2, out2)
    assert torch.equal(out2, src.index_select(0, idx2.clamp(0, n - 1)))
