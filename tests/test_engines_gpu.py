"""Native MLP / CNN engines vs the fp32 PyTorch reference modules, and end-to-end native
training jobs on the MI355X (forward values, flat gradients, learning curves)."""
import os
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _flat_grads_ref(ref):
    return torch.cat([p.grad.reshape(-1) for p in ref.parameters()])


@pytest.mark.parametrize("loss", ["mse", "mae_clip"])
def test_native_mlp_matches_reference(loss):
    from wellflow.models.base import per_element_loss
    from wellflow.models.mlp import MLPRegressor, NativeMLP

    torch.manual_seed(0)
    F, Hs, B = 13, (256, 128), 300
    ref = MLPRegressor(F, Hs).to(DEV)
    eng = NativeMLP(F, Hs, batch=512, device=DEV, loss=loss)
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()
    x, y = torch.randn(B, F, device=DEV), torch.randn(B, device=DEV)
    p = eng.forward(x).clone()
    r = ref(x)
    assert _rel(p, r) < 2e-2
    eng.forward_backward(x, y, grad_scale=1.0 / B)
    per_element_loss(loss, ref(x), y).sum().mul(1.0 / B).backward()
    gref = MLPRegressor(F, Hs)
    for pr, pg in zip(gref.parameters(), ref.parameters()):
        pr.data.copy_(pg.grad.cpu())
    gflat = gref.to_flat().to(DEV)
    assert _rel(eng.grads, gflat) < 3e-2, _rel(eng.grads, gflat)


@pytest.mark.parametrize("loss", ["mae_clip", "mse"])
def test_native_cnn_matches_reference(loss):
    from wellflow.models.base import per_element_loss
    from wellflow.models.cnn import CNN1DRegressor, NativeCNN

    torch.manual_seed(1)
    ref = CNN1DRegressor(dropout=0.0).init_keras(3).to(DEV)
    eng = NativeCNN(ref.layout, batch=64, device=DEV, dropout=0.0, loss=loss)
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()
    B = 40
    x, y = torch.randn(B, 48, 1, device=DEV), torch.randn(B, 12, device=DEV)
    assert _rel(eng.forward(x), ref(x)) < 2e-2
    ls = eng.forward_backward(x, y, grad_scale=1.0 / (B * 12))
    L = per_element_loss(loss, ref(x), y).sum()
    (L / (B * 12)).backward()
    assert abs(ls.item() - L.item()) < 2e-2 * L.item()
    gref = CNN1DRegressor(dropout=0.0)
    for pr, pg in zip(gref.parameters(), ref.parameters()):
        pr.data.copy_(pg.grad.cpu())
    assert _rel(eng.grads, gref.to_flat().to(DEV)) < 3e-2


def _cnn_ref_with_mask(ref, x, y, loss, mask, keep_scale=2.0):
    """fp32 reference forward of the CNN with an explicit dropout keep mask [B, T, Fp]."""
    from wellflow.models.base import per_element_loss

    B = x.shape[0]
    h = torch.relu(ref.conv(x.transpose(1, 2))).transpose(1, 2)  # [B, T, F]
    h = h * mask[:, :, : ref.filters].float() * keep_scale
    out = ref.dense(h.reshape(B, -1))
    return per_element_loss(loss, out, y).sum(), out


def _flat_grad(ref):
    from wellflow.models.cnn import CNN1DRegressor

    g = CNN1DRegressor(dropout=0.0)
    for pr, pg in zip(g.parameters(), ref.parameters()):
        pr.data.copy_(pg.grad.cpu())
    return g.to_flat().to(DEV)


def test_lstm_adam_writeback_equals_adam_then_pack():
    """FlatAdam(writeback=NativeLSTM): Adam and the bf16 weight copies Wp / WhhT in one launch
    (csrc/elementwise.hip lstm_adam_pack_kernel) == adam_dev followed by lstm_pack_weights, on
    identical gradients (the engine's own backward sums some terms with atomics, so two runs of it
    differ in the last bits: the gradients here are given)."""
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat
    from wellflow.optim.flat import FlatAdam

    B, T, F, H = 512, 8, 16, 512
    engs, opts = [], []
    for wb in (False, True):
        eng = NativeLSTM(F, H, T, B, device=DEV)
        eng.params.copy_(init_lstm_flat(F, H, seed=2).to(DEV))
        eng.sync_weights()
        engs.append(eng)
        opts.append(FlatAdam(eng.params, eng.grads, lr=1e-3, zero_grads=True, writeback=eng if wb else None))
    gen = torch.Generator(device=DEV).manual_seed(5)
    for _ in range(3):
        gr = torch.randn(engs[0].grads.shape, device=DEV, generator=gen) * 1e-2
        for eng, opt in zip(engs, opts):
            eng.grads.copy_(gr)
            opt.step()
            if opt.writeback is None:
                eng.sync_weights()
    torch.cuda.synchronize()
    a, b = engs
    # the same Adam arithmetic in two kernels (fp contraction may differ by an ulp)
    for x, y in ((a.params, b.params), (opts[0].m, opts[1].m), (opts[0].v, opts[1].v)):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-8)
    assert torch.equal(opts[0].step_dev, opts[1].step_dev)
    # the images written by the fused launch ARE lstm_pack_weights of the updated parameters
    wp, wt = b.Wp.clone(), b.WhhT.clone()
    b.sync_weights()
    torch.cuda.synchronize()
    assert torch.equal(wp, b.Wp) and torch.equal(wt, b.WhhT)
    assert b.grads.abs().max().item() == 0.0  # the bucket was cleared


def test_cnn_sgd_writeback_equals_sgd_then_pack():
    """FlatSGD(writeback=NativeCNN): the update and the bf16 operand images in one launch
    (csrc/cnn_fused.hip cnn_sgd_pack_kernel) == the plain SGD launch followed by cnn_pack on
    given gradients: same parameters and velocities (to an ulp), device step counter, and images
    bit-identical to a pack of the updated parameters."""
    from wellflow.models.cnn import CNN1DRegressor, NativeCNN
    from wellflow.optim.flat import FlatSGD

    torch.manual_seed(3)
    ref = CNN1DRegressor(dropout=0.5).init_keras(5).to(DEV)
    engs, opts = [], []
    for wb in (False, True):
        eng = NativeCNN(ref.layout, batch=512, device=DEV, dropout=0.5, loss="mae_clip", seed=3)
        eng.params.copy_(ref.to_flat().to(DEV))
        eng.sync_weights()
        engs.append(eng)
        opts.append(FlatSGD(eng.params, eng.grads, lr=0.01, zero_grads=True, writeback=eng if wb else None))
    gen = torch.Generator(device=DEV).manual_seed(6)
    for _ in range(3):
        gr = torch.randn(engs[0].grads.shape, device=DEV, generator=gen) * 1e-2
        for eng, opt in zip(engs, opts):
            eng.grads.copy_(gr)
            opt.step()
            if opt.writeback is None:
                eng.sync_weights()
    torch.cuda.synchronize()
    a, b = engs
    # the same SGD arithmetic in two kernels (fp contraction may differ by an ulp)
    torch.testing.assert_close(a.params, b.params, rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(opts[0].vel, opts[1].vel, rtol=1e-5, atol=1e-8)
    assert torch.equal(opts[0].step_dev, opts[1].step_dev)
    # the images written by the fused launch ARE cnn_pack of the updated parameters
    imgs = {nm: getattr(b, nm).clone() for nm in ("WcA", "WdF", "WdB")}
    b.sync_weights()
    torch.cuda.synchronize()
    for nm, t in imgs.items():
        assert torch.equal(t, getattr(b, nm)), nm
    assert b.grads.abs().max().item() == 0.0


@pytest.mark.parametrize("loss,B,p", [("mse", 1000, 0.5), ("mae_clip", 4096, 0.5), ("mse", 64, 0.5), ("mse", 1000, 0.0),
                                      ("mae_clip", 65536, 0.5)])
def test_native_cnn_bit_exact_vs_bf16_emulation(loss, B, p):
    """The fused CNN step against a torch emulation of ITS OWN roundings (bf16 x, weights,
    pre-activation, dOut x keep-scale and dAct; fp32 sums) with the same dropout mask: dOut and
    both weight gradients agree to fp32 summation order. The fp32-reference tests above have
    2-5 % tolerances (bf16 vs fp32), which a corrupted MFMA operand passed in round 5 (2 % of
    dOut wrong from a VALU write of the conv MFMA's SrcB at 0 wait states); this one does not."""
    from wellflow.models.base import per_element_loss
    from wellflow.models.cnn import CNN1DRegressor, NativeCNN, cnn_dropout_mask

    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    torch.manual_seed(2)
    ref = CNN1DRegressor(dropout=p).init_keras(4).to(DEV)
    with torch.no_grad():
        ref.conv.bias.uniform_(-0.05, 0.05)
        ref.dense.bias.uniform_(-0.1, 0.1)
    eng = NativeCNN(ref.layout, batch=max(4096, B), device=DEV, dropout=p, loss=loss, seed=7)
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()
    x, y = torch.randn(B, 48, 1, device=DEV), torch.randn(B, 12, device=DEV)
    eng.rng.fill_(5)
    eng.forward_backward(x, y, grad_scale=1.0 / (B * 12))
    torch.cuda.synchronize()
    ks = 2.0 if p > 0 else 1.0
    mask = cnn_dropout_mask(eng.seed32, 5, B, 36, eng.lay.Fp, device=DEV)[:, :, :100].float()
    if p == 0:
        mask = torch.ones_like(mask)
    Wc, bc = ref.conv.weight.detach().view(100, 13), ref.conv.bias.detach()
    Wd, bd = ref.dense.weight.detach().view(12, 36, 100), ref.dense.bias.detach()
    xw = bf(x.view(B, 48))
    win = torch.stack([xw[:, t : t + 13] for t in range(36)], 1)  # [B, T, taps]
    act = torch.relu(bf(win @ bf(Wc).t() + bf(bc))) * mask
    o = (torch.einsum("btf,jtf->bj", act, bf(Wd)) * ks + bd).requires_grad_(True)
    per_element_loss(loss, o, y).sum().mul(1.0 / (B * 12)).backward()
    doA = bf(o.grad * ks)
    gWd = torch.einsum("btf,bj->jtf", act, doA)
    dp = bf(torch.einsum("bj,jtf->btf", doA, bf(Wd))) * (act != 0).float()
    gWc = torch.cat([torch.einsum("btf,btk->fk", dp, win), dp.sum((0, 1))[:, None]], 1)
    Wc_n, Wd_n, _ = eng.lay.views(eng.grads)
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(eng.dout[: B * 16].view(B, 16)[:, :12], o.grad) < 1e-4
    assert rel(Wd_n[:12].view(12, 36, 112)[:, :, :100], gWd) < 1e-4
    assert rel(Wc_n[:100, :14], gWc) < 1e-4


@pytest.mark.parametrize("loss,B", [("mse", 1000), ("mae_clip", 4096), ("mae_clip", 65536)])
def test_native_cnn_dropout_matches_fp32_same_mask(loss, B):
    """The fused CNN step with dropout 0.5 (csrc/cnn_fused.hip) against the fp32 reference
    that applies the SAME keep mask (models/cnn.py cnn_dropout_mask mirrors the kernels' hash
    bit for bit): loss, every gradient block, and the device step counter. B = 1000 leaves a
    partial 16-window group; B = 65,536 is the bench shape (round-4 VERDICT item 2)."""
    from wellflow.models.cnn import CNN1DRegressor, NativeCNN, cnn_dropout_mask

    torch.manual_seed(2)
    ref = CNN1DRegressor(dropout=0.5).init_keras(4).to(DEV)
    with torch.no_grad():  # non-zero biases exercise the folded bias slot and its gradient
        ref.conv.bias.uniform_(-0.05, 0.05)
        ref.dense.bias.uniform_(-0.1, 0.1)
    eng = NativeCNN(ref.layout, batch=max(4096, B), device=DEV, dropout=0.5, loss=loss, seed=7)
    assert eng.fused
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()
    x, y = torch.randn(B, 48, 1, device=DEV), torch.randn(B, 12, device=DEV)
    eng.rng.fill_(5)
    ls = eng.forward_backward(x, y, grad_scale=1.0 / (B * 12)).item()
    torch.cuda.synchronize()
    assert int(eng.rng.item()) == 6
    mask = cnn_dropout_mask(eng.seed32, 5, B, 36, eng.lay.Fp, device=DEV)
    kept = mask[:, :, :100].float().mean().item()
    assert 0.45 < kept < 0.55, kept
    L, _ = _cnn_ref_with_mask(ref, x, y, loss, mask)
    (L / (B * 12)).backward()
    assert abs(ls - L.item()) <= 2e-2 * L.item(), (ls, L.item())
    g_r, g_n = _flat_grad(ref), eng.grads
    Wc_n, Wd_n, bd_n = eng.lay.views(g_n)
    Wc_r, Wd_r, bd_r = eng.lay.views(g_r)
    # the conv gradient is a 36k-term sum of mixed sign per entry through bf16 dA = dout Wd^T:
    # cancellation puts its relative error a little above the dense blocks' (3.05 % measured
    # at B = 1000, MSE)
    for name, a, b, tol in (("conv", Wc_n, Wc_r, 5e-2), ("dense", Wd_n, Wd_r, 3e-2), ("dense bias", bd_n, bd_r, 3e-2)):
        assert _rel(a, b) < tol, (name, _rel(a, b))
    # the filter / output padding carries exactly zero gradient
    assert Wc_n[100:].abs().max().item() == 0.0 and Wc_n[:, 14:].abs().max().item() == 0.0
    assert Wd_n[12:].abs().max().item() == 0.0
    assert Wd_n.view(16, 36, 112)[:, :, 100:].abs().max().item() == 0.0


def test_native_cnn_fused_matches_gemm_path():
    """Fused kernels vs the im2col + GEMM path (dropout 0; both bf16 MFMA): loss, gradients and
    predictions agree to bf16 rounding."""
    from wellflow.models.cnn import CNN1DRegressor, NativeCNN

    ref = CNN1DRegressor(dropout=0.0).init_keras(6)
    B = 2048
    x, y = torch.randn(B, 48, 1, device=DEV), torch.randn(B, 12, device=DEV)
    res = {}
    for fused in (True, False):
        eng = NativeCNN(ref.layout, batch=B, device=DEV, dropout=0.0, loss="mae_clip", fused=fused)
        eng.params.copy_(ref.to_flat().to(DEV))
        eng.sync_weights()
        ls = eng.forward_backward(x, y, 1.0 / (B * 12)).item()
        res[fused] = (ls, eng.grads.clone(), eng.forward(x).clone())
    (la, ga, pa), (lb, gb, pb) = res[True], res[False]
    assert abs(la - lb) <= 1e-2 * abs(lb)
    assert _rel(ga, gb) < 2e-2 and _rel(pa, pb) < 1e-2


@pytest.mark.parametrize("model", ["mlp", "lstm", "cnn", "mlp_online"])
def test_native_training_job_learns(model, tmp_path):
    from wellflow.train.job import run_job

    names = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
    types = "string,string,int,float,float,float,float,float,float,float"
    args = [names, types, "flow", str(tmp_path), "--epochs", "8", "--synth-wells", "8",
            "--synth-steps", "300", "--device", "cuda"]
    if model == "lstm":
        args += ["--seq-len", "32", "--batch-size", "256"]
    if model == "cnn":
        args += ["--batch-size", "64", "--lr", "0.01"]
    if model == "mlp_online":
        args += ["--online-chunk", "256", "--epochs", "3"]
    out = run_job(model, args, log=lambda *a, **k: None)
    assert out["native"] is True
    h = out["history"]
    assert min(h["val_loss"]) < h["val_loss"][0] or h["val_loss"][-1] < 1.0
    assert out["test_loss"] == out["test_loss"]
    assert (tmp_path / "models" / f"{model}.mdl").exists()


def test_lstm_submission_script_from_csv_on_gpu(tmp_path):
    """The reference's submission contract end to end on the MI355X: the LSTM model script
    with names / types / target / storagePath and a CSV data path -> native C++ CSV ingest
    (wellflow/_runtime.so) -> features -> HIP LSTM engine (wellflow/_C.so) -> .mdl + the two
    stdout lines (cnn.py:2, 41-44, 122, 133-134)."""
    import subprocess
    import sys

    from wellflow.data.io import write_csv
    from wellflow.data.synth import TABLE_COLUMNS, well_log_table

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    data = str(tmp_path / "logs.csv")
    write_csv(well_log_table(6, 240, seed=9), data, columns=TABLE_COLUMNS)
    names = ",".join(TABLE_COLUMNS)
    types = "string,string,int,float,float,float,float,float,float,float"
    env = dict(os.environ, WELLFLOW_NATIVE_IO="1")
    r = subprocess.run([sys.executable, os.path.join(root, "Artificial intelligence models", "LSTM models", "lstm.py"),
                        names, types, "flow", str(tmp_path) + "/", data, "--epochs", "3", "--seq-len", "16",
                        "--batch-size", "128", "--device", "cuda"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert lines[-2].startswith("Time elapsed: ") and lines[-1].startswith("Testing set loss: ")
    assert float(lines[-1].split(":")[1]) == float(lines[-1].split(":")[1])  # finite, parseable
    assert (tmp_path / "models" / "lstm.mdl").exists()


@pytest.mark.parametrize("B,F", [(65536, 16), (1000, 9), (64, 32), (3000, 40), (512, 64)])
def test_fused_mlp_forward_matches_per_layer(B, F):
    """The one-launch weight-stationary MLP forward (csrc/mlp_fused.hip) against the
    per-layer GEMM + head path on the same weights: saved activations, predictions, loss and
    the gradients the unchanged backward computes from them."""
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat

    eng = NativeMLP(F, (256, 256), B, device=DEV)
    eng.step_fused = False  # the fused forward + backward PAIR (mask mode writes M2)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=3).to(DEV))
    eng.sync_weights()
    x, y = synth_tabular_batch(B, F, seed=4)
    x, y = x.to(DEV), y.to(DEV)
    res = {}
    masks = None
    # (fused forward, fused backward, H2 as a ReLU bitmask + head gradients in the forward)
    for fused, fused_bwd, mask in ((False, False, False), (True, False, False), (True, True, False),
                                   (True, True, True)):
        eng.fused, eng.fused_bwd, eng.mask_h2 = fused, fused_bwd, mask
        if mask:
            eng.Hs[1].zero_()  # not written in mask mode
        ls = eng.forward_backward(x, y, grad_scale=1.0 / B).item()
        torch.cuda.synchronize()
        res[fused, fused_bwd, mask] = (eng.Hs[0][: B * 256].float().clone(), eng.Hs[1][: B * 256].float().clone(),
                                       eng.pred[:B].clone(), eng.dy[:B].clone(), ls, eng.grads.clone(),
                                       eng.dZ[0][: B * 256].float().clone(), eng.dZ[1][: B * 256].float().clone())
        if mask:
            masks = eng.M2[: B * 8].clone()
    # the bitmask is exactly H2 > 0 of the same fused forward
    h2f = res[True, True, False][1].view(B, 8, 32)
    bits = torch.tensor([1 << i for i in range(31)] + [-(1 << 31)], dtype=torch.int64, device=DEV)
    want = ((h2f > 0).long() * bits).sum(-1)
    want = torch.where(want >= (1 << 31), want - (1 << 32), want).to(torch.int32).view(-1)
    assert torch.equal(masks, want)
    assert res[True, True, True][1].abs().max().item() == 0.0  # H2 never left the CU
    h1a, h2a, pa, da, la, ga, z1a, z2a = res[False, False, False]
    for key in ((True, False, False), (True, True, False), (True, True, True)):
        h1b, h2b, pb, db, lb, gb, z1b, z2b = res[key]
        if key[2]:
            h2b = res[True, True, False][1]
        assert (h1a - h1b).abs().max().item() <= 1e-2 * max(1.0, h1a.abs().max().item()), key
        assert (h2a - h2b).abs().max().item() <= 2e-2 * max(1.0, h2a.abs().max().item()), key
        assert (pa - pb).abs().max().item() <= 1e-2 * max(1.0, pa.abs().max().item()), key
        assert abs(la - lb) <= 1e-3 * abs(la) + 1e-6, key
        assert ((ga - gb).norm() / ga.norm()).item() < 1e-2, key
        assert torch.allclose(da, db, rtol=1e-2, atol=1e-6 * max(1.0, da.abs().max().item())), key
        # saved gradients of the backward (fused kernel vs head kernels + dX GEMM); the fused
        # backward keeps dZ1 on chip (dW1 is accumulated in the kernel), so only dZ2 is compared
        assert ((z2a - z2b).norm() / z2a.norm()).item() < 2e-2, key
        if not key[1]:
            assert ((z1a - z1b).norm() / z1a.norm()).item() < 2e-2, key
    # per-block gradient agreement of the fully fused step (bias / head blocks included)
    from wellflow.models.mlp import MlpLayout
    ga_l, ga_hw, ga_hb = MlpLayout(F, (256, 256)).views(ga)
    for key in ((True, True, False), (True, True, True)):
        gb_l, gb_hw, gb_hb = MlpLayout(F, (256, 256)).views(res[key][5])
        for (Wa, ba), (Wb, bb) in zip(ga_l, gb_l):
            assert ((Wa - Wb).norm() / Wa.norm()).item() < 2e-2, key
            assert ((ba - bb).norm() / ba.norm()).item() < 2e-2, key
        assert ((ga_hw - gb_hw).norm() / ga_hw.norm()).item() < 1e-2, key
        assert torch.allclose(ga_hb, gb_hb, rtol=1e-3, atol=1e-6), key
    # mask mode against the H2-reading fused backward: same forward, same gradients up to
    # fp32 summation order
    gm, gh = res[True, True, True][5], res[True, True, False][5]
    assert ((gm - gh).norm() / gh.norm()).item() < 1e-4


def test_mlp_bf16_input_matches_fp32_input():
    """bf16-streamed features (online bench, data/stream.py) give the same step as fp32
    features: the engine casts fp32 to bf16 itself, so predictions are bitwise equal."""
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat

    B, F = 262144, 16
    eng = NativeMLP(F, (256, 256), B, device=DEV)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=5).to(DEV))
    eng.sync_weights()
    x, y = synth_tabular_batch(B, F, seed=6)
    x, y = x.to(DEV), y.to(DEV)
    out = []
    for xin in (x, x.to(torch.bfloat16)):
        ls = eng.forward_backward(xin, y, grad_scale=1.0 / B).item()
        torch.cuda.synchronize()
        out.append((ls, eng.pred[:B].clone(), eng.grads.clone()))
    (la, pa, ga), (lb, pb, gb) = out
    assert torch.equal(pa, pb)
    # fp32 atomics in the split-K dW reduce in a run-dependent order: compare with a tolerance
    assert abs(la - lb) <= 1e-5 * abs(la) + 1e-6
    assert ((ga - gb).norm() / ga.norm()).item() < 1e-5


def _mlp_step_close(la, pa, ga, lb, pb, gb, tag, flips: bool) -> None:
    """Two MLP training-step paths agree: predictions, loss and gradients up to the fp32 sum
    order (flips=False), or — against mlp2_step128_kernel, which folds b1 / b2 into the MFMA
    accumulator and takes db1 / db2 as MFMA sums of the bf16 dZ1 / dZ2 — up to that order
    moving a few H1 / H2 values across a bf16 rounding boundary (one ulp, 2^-8 relative, in a
    fraction of a percent of the elements; flips=True)."""
    assert torch.isfinite(gb).all(), tag
    if not flips:
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
        assert abs(la - lb) <= 1e-5 * abs(la) + 1e-7, tag
        assert ((ga - gb).norm() / ga.norm()).item() < 1e-4, tag
        return
    d = (pa - pb).abs()
    off = (d > 1e-5 * pa.abs() + 1e-6).float().mean().item()
    scale = pa.abs().max().item() + 1.0
    print(f"{tag}: pred off-tolerance {off:.4%}, max |d| {d.max().item():.2e}, loss rel "
          f"{abs(la - lb) / abs(la):.2e}, grad rel-norm {((ga - gb).norm() / ga.norm()).item():.2e}")
    assert off < 0.01, tag
    assert d.max().item() <= 2e-3 * scale, tag
    assert abs(la - lb) <= 1e-4 * abs(la) + 1e-7, tag
    assert ((ga - gb).norm() / ga.norm()).item() < 2e-3, tag


@pytest.mark.parametrize("B,F", [(262144, 16), (4096, 32), (128, 8)])
def test_mlp_recompute_step_matches_stored_h1(B, F):
    """The H1-free training step (fused forward writes only the H2 bitmask; the fused backward
    and the dW2 kernel recompute H1 from X, csrc/mlp_fused.hip) against the step that stores
    and re-reads H1 with the generic split-K dW2 GEMM: same loss, same gradients up to the
    fp32 summation order (both the fused kernels and the GEMM path are checked against fp32
    torch in test_numerics_gpu.py)."""
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat

    eng = NativeMLP(F, (256, 256), B, device=DEV)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=8).to(DEV))
    eng.sync_weights()
    x, y = synth_tabular_batch(B, F, seed=9)
    x, y = x.to(DEV), y.to(DEV)
    out = {}
    for rec in (False, True):
        eng.recompute_h1 = rec
        eng.Hs[0].fill_(float("nan")) if rec else None  # recompute must not read a stored H1
        ls = eng.forward_backward(x, y, grad_scale=1.0 / B).item()
        torch.cuda.synchronize()
        out[rec] = (ls, eng.pred[:B].clone(), eng.grads.clone())
    assert eng._recompute_ok(B)
    (la, pa, ga), (lb, pb, gb) = out[False], out[True]
    # the training forward (8 waves, 32 units each) sums the head in a different fp32 order;
    # the default recompute step is the 128-row kernel when the engine holds W2^T
    _mlp_step_close(la, pa, ga, lb, pb, gb, "recompute", flips=eng.w2t is not None)


def test_mlp_spread_reduction_matches_direct_atomics():
    """The training step's batch sums through the 64-copy scratch, the backward's per-workgroup
    dW1 rows and mlp2_reduce (csrc/mlp_fused.hip) against direct same-address atomics
    (WELLFLOW_MLP_SPREAD=0); three steps in a row must give the same gradients each time, i.e.
    the reduce re-zeroes the copies and leaves nothing behind for the next step."""
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import MLP_RED_COPY_FLOATS, NativeMLP, init_mlp_flat

    B, F = 65536, 16
    x, y = synth_tabular_batch(B, F, seed=13)
    x, y = x.to(DEV), y.to(DEV)
    flat = init_mlp_flat(F, (256, 256), seed=12).to(DEV)
    engs = {}
    for spread in ("1", "0"):
        os.environ["WELLFLOW_MLP_SPREAD"] = spread
        try:
            eng = NativeMLP(F, (256, 256), B, device=DEV)
        finally:
            os.environ.pop("WELLFLOW_MLP_SPREAD", None)
        eng.params.copy_(flat)
        eng.sync_weights()
        engs[spread] = eng
    assert engs["1"].red is not None and engs["0"].red is None
    ref_ls = engs["0"].forward_backward(x, y, grad_scale=1.0 / B).item()
    torch.cuda.synchronize()
    ref_g = engs["0"].grads.clone()
    for _ in range(3):
        ls = engs["1"].forward_backward(x, y, grad_scale=1.0 / B).item()
        torch.cuda.synchronize()
        g = engs["1"].grads
        assert abs(ls - ref_ls) <= 1e-5 * abs(ref_ls)
        assert ((g - ref_g).norm() / ref_g.norm()).item() < 1e-5
    # the atomic copies are re-zeroed by the reduce (the dW1 rows after them are overwritten)
    assert engs["1"].red[:MLP_RED_COPY_FLOATS].abs().max().item() == 0.0


def test_mlp_row_indexed_step_matches_gathered_batch():
    """forward_backward(dataset, targets, rows=idx) reads the resident dataset through the
    index inside the fused kernels; it must equal the step on the explicitly gathered batch
    (the Trainer's job path uses it, train/trainer.py)."""
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat

    N, B, F = 100000, 16384, 16
    eng = NativeMLP(F, (256, 256), B, device=DEV)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=10).to(DEV))
    eng.sync_weights()
    X, Y = synth_tabular_batch(N, F, seed=11)
    X, Y = X.to(DEV).to(torch.bfloat16), Y.to(DEV)
    idx = torch.randperm(N, device=DEV)[:B]
    ls_a = eng.forward_backward(X.index_select(0, idx), Y.index_select(0, idx), 1.0 / B).item()
    torch.cuda.synchronize()
    pa, ga = eng.pred[:B].clone(), eng.grads.clone()
    ls_b = eng.forward_backward(X, Y, 1.0 / B, rows=idx).item()
    torch.cuda.synchronize()
    assert torch.equal(pa, eng.pred[:B])
    assert abs(ls_a - ls_b) <= 1e-5 * abs(ls_a)
    assert ((ga - eng.grads).norm() / ga.norm()).item() < 1e-4


def _dz2_from_frag(zf: torch.Tensor, B: int) -> torch.Tensor:
    """[B][256] view of a dZ2 written in the fragment layout (csrc/kernels.h launch_mlp2_step):
    element ((S * 16 + b) * 64 + 16 g + l) * 8 + j = row 32 S + 8 g + j, unit 16 b + l."""
    return zf[: B * 256].view(B // 32, 16, 4, 16, 8).permute(0, 2, 4, 1, 3).reshape(B, 256)


@pytest.mark.parametrize("B,F,indexed", [(262144, 16, False), (327680, 16, False), (4096, 32, False), (16384, 16, True),
                                       (128, 8, False), (4160, 16, False), (64, 16, False)])
def test_mlp_one_launch_step_matches_two_kernel_step(B, F, indexed):
    """The training step's forward + backward in ONE launch (csrc/mlp_step.hip: X staged once,
    layer 1 computed once, H2 and dy never leave the workgroup), with dZ2 row-major + the
    LDS-staged dW2 kernel and with dZ2 in the fragment layout + the LDS-free dW2 kernel, against
    the fused forward + fused backward pair (csrc/mlp_fused.hip) it replaces: same predictions,
    loss and gradients up to the fp32 summation order, bit-identical dZ2; the spread scratch
    must be left zeroed. "step_frag" is the 128-row-pass kernel streaming W2 and W2^T
    (mlp2_step128_kernel; B = 4160 and 64 end in a half pass), "step_frag64" the 64-row one."""
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import MLP_RED_COPY_FLOATS, NativeMLP, init_mlp_flat

    eng = NativeMLP(F, (256, 256), B, device=DEV)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=21).to(DEV))
    eng.sync_weights()
    N = 3 * B if indexed else B
    X, Y = synth_tabular_batch(N, F, seed=22)
    X, Y = X.to(DEV), Y.to(DEV)
    idx = torch.randperm(N, device=DEV)[:B] if indexed else None
    if indexed:
        X = X.to(torch.bfloat16)
    out = {}
    w2t = eng.w2t
    assert w2t is not None  # the default engine streams both weight images
    for name, fused, frag in (("pair", False, False), ("step", True, False), ("step_frag", True, True),
                              ("step_frag64", True, True)):
        eng.step_fused, eng.dw2_frag = fused, frag
        eng.w2t = None if name == "step_frag64" else w2t
        eng.dZ[1].fill_(float("nan"))
        ls = eng.forward_backward(X, Y, grad_scale=1.0 / B, rows=idx).item()
        torch.cuda.synchronize()
        z = None if name == "step_mask" else (_dz2_from_frag(eng.dZ[1], B) if frag else eng.dZ[1][: B * 256].view(B, 256))
        out[name] = (ls, eng.pred[:B].clone(), eng.grads.clone(), None if z is None else z.clone())
        assert eng.red[:MLP_RED_COPY_FLOATS].abs().max().item() == 0.0, name
    assert eng._recompute_ok(B)
    la, pa, ga, za = out["pair"]
    for name in ("step", "step_frag", "step_frag64"):
        lb, pb, gb, zb = out[name]
        _mlp_step_close(la, pa, ga, lb, pb, gb, name, flips=name == "step_frag")
        if name != "step_frag":
            # dZ2 (dW2's operand) is bit-identical: same H2 rounding, same dy, same bf16 product
            assert torch.equal(za, zb), name
        else:
            # the 128-row kernel folds b1 / b2 into the MFMA accumulator (fp32 sum order): the
            # rows whose H1 / H2 round differently get a slightly different prediction, hence dy
            # (dZ2 = bf16(dy w3)); an H2 within fp32 noise of 0 may flip its ReLU mask
            a, b = za.float(), zb.float()
            print(f"{name}: dZ2 differs in {(a != b).float().mean().item():.4%}, rel-norm "
                  f"{((a - b).norm() / a.norm()).item():.2e}, mask flips {((a == 0) != (b == 0)).sum().item()}")
            assert (a != b).float().mean().item() < 0.01, name
            assert ((a - b).norm() / a.norm()).item() < 1e-3, name
            assert ((a == 0) != (b == 0)).float().mean().item() < 1e-5, name


def test_lstm_reads_resident_windows_in_place():
    """NativeLSTM.forward_backward(windows, y, rows=ids): the x-pack kernel reads the batch's
    windows straight from the resident row table (data/features.py SeriesWindows) — the same
    packed input, loss and gradients as the gathered [B][T][F] batch."""
    from wellflow.data.features import SeriesWindows
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    B, T, F, H = 512, 16, 16, 512
    g = torch.Generator(device=DEV).manual_seed(3)
    table = torch.randn(5000, F, device=DEV, generator=g)
    starts = torch.randint(0, 5000 - T + 1, (3000,), device=DEV, generator=g)
    win = SeriesWindows(table, starts, T)
    yall = torch.randn(3000, device=DEV, generator=g)
    ids = torch.randperm(3000, device=DEV, generator=g)[:B]
    out = []
    for inplace in (False, True):
        eng = NativeLSTM(F, H, T, B, device=DEV)
        eng.params.copy_(init_lstm_flat(F, H, seed=4).to(DEV))
        eng.sync_weights()
        if inplace:
            ls = eng.forward_backward(win, yall, 1.0 / B, rows=ids)
        else:
            ls = eng.forward_backward(win[ids], yall.index_select(0, ids), 1.0 / B)
        torch.cuda.synchronize()
        xb = eng.XH.view(T + 1, B, -1)[:T, :, : eng.lay.KX].clone()
        out.append((ls.item(), eng.grads.clone(), xb))
    (la, ga, xa), (lb, gb, xbb) = out
    assert torch.equal(xa, xbb)
    assert abs(la - lb) <= 1e-6 * abs(lb)
    assert _rel(gb, ga) < 1e-3
