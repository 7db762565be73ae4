"""The small-batch MLP path (csrc/mlp_small.hip, NativeMLP.fused_steps): K training steps
(forward, backward, Adam) in one persistent launch of 16 workgroups, at the job-default batch
(round-5 VERDICT item 3). Against fp32 autograd + torch.optim.Adam on the same batches, and
K fused steps against K single-step launches bit for bit."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(F=16, B=256, N=None, loss="mse", seed=5, clip=1.0):
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat
    from wellflow.optim.flat import FlatAdam

    N = N or 24 * B
    eng = NativeMLP(F, (256, 256), B, device=DEV, loss=loss, clip=clip)
    flat = init_mlp_flat(F, (256, 256), seed=seed)
    eng.params.copy_(flat.to(DEV))
    eng.sync_weights()
    opt = FlatAdam(eng.params, eng.grads, lr=1e-3, shadow=eng.shadow, zero_grads=True, shadow_t=eng.shadow_t)
    X, Y = synth_tabular_batch(N, F, seed=seed + 1)
    return eng, opt, flat, X.to(DEV).to(torch.bfloat16), Y.to(DEV)


def _state(eng, opt, acc):
    return [eng.params.clone(), opt.m.clone(), opt.v.clone(), opt.step_dev[:1].clone(), eng.shadow.clone(),
            None if eng.w2t is None else eng.w2t.clone(), acc.clone()]


@pytest.mark.parametrize("B", [256, 96])
def test_small_k_fused_equals_k_single(B):
    """One launch of K = 8 steps, eight launches of K = 1 and two of K = 4 from the same
    state: parameters, Adam moments, step counter, bf16 images and the loss sum bit-equal."""
    K = 8
    out = []
    for split in ([8], [1] * 8, [4, 4]):
        eng, opt, _, X, Y = _setup(B=B)
        g = torch.Generator(device=DEV)
        g.manual_seed(9)
        rows = torch.randperm(X.shape[0], generator=g, device=DEV)[: K * B]
        acc = torch.zeros(1, device=DEV)
        s = 0
        for k in split:
            eng.fused_steps(X, Y, B, k, opt, 1.0 / B, rows=rows[s * B : (s + k) * B], loss_into=acc)
            s += k
        torch.cuda.synchronize()
        eng.check_device_errors()
        out.append(_state(eng, opt, acc))
        assert opt.steps_taken == K
    for other in out[1:]:
        for a, b in zip(out[0], other):
            if a is not None:
                assert torch.equal(a, b)


def test_small_rows_equal_contiguous_slices():
    """Row ids into the dataset vs the same rows gathered into a contiguous buffer (the
    Trainer's sliced epoch): identical launches, identical results."""
    B, K = 256, 4
    res = []
    for mode in ("rows", "slices"):
        eng, opt, _, X, Y = _setup(B=B)
        rows = torch.randperm(X.shape[0], device="cpu", generator=torch.Generator().manual_seed(3))[: K * B].to(DEV)
        acc = torch.zeros(1, device=DEV)
        if mode == "rows":
            eng.fused_steps(X, Y, B, K, opt, 1.0 / B, rows=rows, loss_into=acc)
        else:
            eng.fused_steps(X.index_select(0, rows).contiguous(), Y.index_select(0, rows).contiguous(), B, K, opt,
                            1.0 / B, loss_into=acc)
        torch.cuda.synchronize()
        res.append(_state(eng, opt, acc))
    for a, b in zip(*res):
        if a is not None:
            assert torch.equal(a, b)


@pytest.mark.parametrize("loss", ["mse", "mae_clip"])
def test_small_trajectory_matches_fp32(loss):
    """20 steps at B = 256 on distinct batches against fp32 autograd + torch.optim.Adam on the
    same batches from the same initial parameters: per-step losses within the parity tolerance
    and the fp32 run learning."""
    from wellflow.models.base import per_element_loss
    from wellflow.models.mlp import MLPRegressor

    B, F, steps, clip = 256, 16, 20, 1.0
    eng, opt, flat, X, Y = _setup(F=F, B=B, N=steps * B, loss=loss, clip=clip)
    nat = []
    acc = torch.zeros(1, device=DEV)
    for k in range(steps):
        acc.zero_()
        eng.fused_steps(X[k * B : (k + 1) * B], Y[k * B : (k + 1) * B], B, 1, opt, 1.0 / B, loss_into=acc)
        nat.append(acc.item() / B)
    eng.check_device_errors()
    ref = MLPRegressor(F, (256, 256)).to(DEV)
    ref.load_flat(flat)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    fp = []
    Xf = X.float()
    for k in range(steps):
        ropt.zero_grad()
        L = per_element_loss(loss, ref(Xf[k * B : (k + 1) * B]).reshape(-1), Y[k * B : (k + 1) * B], clip).sum()
        (L / B).backward()
        ropt.step()
        fp.append(L.item() / B)
    rel = [abs(a - b) / b for a, b in zip(nat, fp)]
    dev = max(abs(a - b) for a, b in zip(nat, fp)) / fp[0]
    assert sum(rel) / len(rel) < 0.03 and dev < 0.03, (nat, fp)
    assert sum(fp[-5:]) < 0.9 * sum(fp[:5]), fp  # the reference learns on this data
    # the parameters after 20 updates: close to fp32's (bf16 compute, same Adam)
    p_ref = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    from wellflow.models.mlp import MlpLayout

    lay = MlpLayout(F, (256, 256))
    (w1, b1), (w2, b2) = lay.offsets()[0]
    _, hw, hb, _ = lay.offsets()
    p_nat = torch.cat([eng.params[w1 : w1 + 256 * F], eng.params[b1 : b1 + 256], eng.params[w2 : w2 + 65536],
                       eng.params[b2 : b2 + 256], eng.params[hw : hw + 256], eng.params[hb : hb + 1]])
    p0 = torch.cat([flat[w1 : w1 + 256 * F], flat[b1 : b1 + 256], flat[w2 : w2 + 65536], flat[b2 : b2 + 256],
                    flat[hw : hw + 256], flat[hb : hb + 1]]).to(DEV)
    d_nat, d_ref = p_nat - p0, p_ref - p0
    cos = torch.nn.functional.cosine_similarity(d_nat, d_ref, dim=0).item()
    assert cos > 0.98, cos


def test_small_one_step_matches_regular_step():
    """One fused step against the regular path (one-launch step kernel + dW2 + reduce +
    FlatAdam) on the same batch: the same update up to the fp32 summation order."""
    B = 256
    eng, opt, _, X, Y = _setup(B=B)
    acc = torch.zeros(1, device=DEV)
    p0 = eng.params.clone()
    eng.fused_steps(X[:B], Y[:B], B, 1, opt, 1.0 / B, loss_into=acc)
    torch.cuda.synchronize()
    d_small, l_small = eng.params - p0, acc.item()
    eng2, opt2, _, _, _ = _setup(B=B)
    ls = eng2.forward_backward(X[:B], Y[:B], 1.0 / B).item()
    opt2.step()
    torch.cuda.synchronize()
    assert abs(l_small - ls) <= 1e-3 * abs(ls), (l_small, ls)
    # the gradients, through Adam's first moment m = (1 - beta1) g (the first update itself is
    # ~lr sign(g), which flips on entries whose gradient is at rounding noise)
    rel = ((opt.m - opt2.m).norm() / opt2.m.norm()).item()
    assert rel < 2e-2, rel
    assert d_small.abs().max().item() <= 1.01e-3 and torch.count_nonzero(d_small).item() > 0


def test_small_spin_bound_fails_loudly():
    """A hand-off that cannot complete (spin bound 1: every wait trips) sets the sticky word,
    every workgroup still finishes, and check_device_errors raises; the next launch runs."""
    B = 64
    eng, opt, _, X, Y = _setup(B=B)
    os.environ["WELLFLOW_SPIN_LIMIT"] = "1"
    try:
        eng.fused_steps(X[: 4 * B], Y[: 4 * B], B, 4, opt, 1.0 / B)
        torch.cuda.synchronize()
    finally:
        del os.environ["WELLFLOW_SPIN_LIMIT"]
    with pytest.raises(RuntimeError, match="timed out"):
        eng.check_device_errors()
    eng.fused_steps(X[: 4 * B], Y[: 4 * B], B, 4, opt, 1.0 / B)
    torch.cuda.synchronize()
    eng.check_device_errors()


# ---------------------------------------------------------------------------- CNN (B = 20)
def _cnn_setup(B=20, N=None, seed=4, loss="mae_clip", dropout=0.5):
    from wellflow.models.cnn import CNN1DRegressor, CnnLayout, NativeCNN
    from wellflow.optim.flat import FlatSGD

    lay = CnnLayout()
    torch.manual_seed(seed)
    ref = CNN1DRegressor(lay.input_len, lay.in_ch, lay.filters, lay.kernel, lay.outputs).init_keras(seed)
    with torch.no_grad():
        ref.conv.bias.uniform_(-0.05, 0.05)
        ref.dense.bias.uniform_(-0.05, 0.05)
    flat = ref.to_flat()
    eng = NativeCNN(lay, B, DEV, dropout=dropout, loss=loss, seed=seed)
    eng.params.copy_(flat.to(DEV))
    eng.sync_weights()
    opt = FlatSGD(eng.params, eng.grads, zero_grads=True, writeback=eng)
    N = N or 24 * B
    g = torch.Generator(device="cpu").manual_seed(seed + 1)
    series = torch.randn(N, lay.input_len + lay.outputs, generator=g).cumsum(1) * 0.1
    X = series[:, : lay.input_len].contiguous().to(DEV)
    Y = series[:, lay.input_len:].contiguous().to(DEV)
    return eng, opt, ref, X, Y, lay


def test_cnn_small_k_fused_equals_k_single():
    B, K = 20, 8
    out = []
    for split in ([8], [1] * 8, [3, 5]):
        eng, opt, _, X, Y, _ = _cnn_setup(B=B)
        rows = torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(2))[: K * B].to(DEV)
        acc = torch.zeros(1, device=DEV)
        s = 0
        for k in split:
            eng.fused_steps(X, Y, B, k, opt, 1.0 / (B * 12), rows=rows[s * B : (s + k) * B], loss_into=acc)
            s += k
        torch.cuda.synchronize()
        eng.check_device_errors()
        out.append([eng.params.clone(), opt.vel.clone(), opt.step_dev[:1].clone(), eng.rng.clone(), acc.clone()])
        assert int(eng.rng.item()) == K and int(opt.step_dev[0].item()) == K
    for other in out[1:]:
        for a, b in zip(out[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("loss,dropout", [("mae_clip", 0.5), ("mse", 0.0)])
def test_cnn_small_trajectory_matches_fp32(loss, dropout):
    """20 Keras SGD-Nesterov steps at the reference's batch of 20 on distinct batches against
    fp32 autograd of CNN1DRegressor with the SAME dropout keep masks (cnn_dropout_mask of the
    engine's device step counter): the fused launch computes in fp32, so the per-step losses
    agree to rounding."""
    from wellflow.models.base import per_element_loss
    from wellflow.models.cnn import cnn_dropout_mask

    B, steps = 20, 20
    eng, opt, ref, X, Y, lay = _cnn_setup(B=B, N=steps * B, loss=loss, dropout=dropout)
    scale = 1.0 / (B * lay.outputs)
    step0, seed32 = int(eng.rng.item()), eng.seed32
    nat = []
    acc = torch.zeros(1, device=DEV)
    for k in range(steps):
        acc.zero_()
        eng.fused_steps(X[k * B : (k + 1) * B], Y[k * B : (k + 1) * B], B, 1, opt, scale, loss_into=acc)
        nat.append(acc.item() * scale)
    eng.check_device_errors()
    ref = ref.to(DEV)
    params = list(ref.parameters())
    vel = [torch.zeros_like(p) for p in params]
    lr, mu, decay = 0.001, 0.99, 1e-6
    fp = []
    for k in range(steps):
        for p in params:
            p.grad = None
        xc = X[k * B : (k + 1) * B].view(B, lay.input_len, 1)
        h = torch.relu(ref.conv(xc.transpose(1, 2))).transpose(1, 2)
        if dropout > 0:
            mask = cnn_dropout_mask(seed32, step0 + k, B, lay.lout, lay.Fp, device=DEV)
            h = h * mask[:, :, : lay.filters].float() * 2.0
        out = ref.dense(h.reshape(B, -1))
        L = per_element_loss(loss, out, Y[k * B : (k + 1) * B]).sum()
        (L * scale).backward()
        lr_t = lr / (1.0 + decay * k)
        with torch.no_grad():
            for p, v in zip(params, vel):
                v.mul_(mu).sub_(lr_t * p.grad)
                p.add_(mu * v - lr_t * p.grad)
        fp.append(L.item() * scale)
    rel = [abs(a - b) / b for a, b in zip(nat, fp)]
    assert max(rel) < 1e-3, (nat, fp)
    p_ref = ref.to_flat().to(DEV)
    assert ((eng.params - p_ref).norm() / p_ref.norm()).item() < 1e-4


def test_cnn_small_spin_bound_fails_loudly():
    B = 20
    eng, opt, _, X, Y, _ = _cnn_setup(B=B)
    os.environ["WELLFLOW_SPIN_LIMIT"] = "1"
    try:
        eng.fused_steps(X[: 4 * B], Y[: 4 * B], B, 4, opt, 1.0 / B)
        torch.cuda.synchronize()
    finally:
        del os.environ["WELLFLOW_SPIN_LIMIT"]
    with pytest.raises(RuntimeError, match="timed out"):
        eng.check_device_errors()
    eng.fused_steps(X[: 4 * B], Y[: 4 * B], B, 4, opt, 1.0 / B)
    torch.cuda.synchronize()
    eng.check_device_errors()


def test_online_job_stages_chunks_into_k_step_launches(tmp_path, monkeypatch):
    """mlp_online at its job default (256-row batches, one GPU): every stream chunk is one
    host -> HBM copy and its batches run as K-step launches (train/online.py _ChunkStage);
    the per-chunk training losses match the per-batch ring path (regular one-launch steps)."""
    from wellflow.models.mlp import NativeMLP
    from wellflow.train import online
    from wellflow.train.job import run_job

    used = []

    class Spy(online._ChunkStage):
        def __init__(self, *a, **k):
            used.append(1)
            super().__init__(*a, **k)

    monkeypatch.setattr(online, "_ChunkStage", Spy)
    names = "well,field,t,whp,choke,glr,temp,water_cut,dsp,flow"
    types = "string,string,int,float,float,float,float,float,float,float"

    def job(sub):
        args = [names, types, "flow", str(tmp_path / sub), "--epochs", "2", "--synth-wells", "8",
                "--synth-steps", "600", "--device", "cuda", "--online-chunk", "1024", "--seed", "3"]
        return run_job("mlp_online", args, log=lambda *a, **k: None)

    a = job("staged")
    assert used and a["native"] is True
    monkeypatch.setattr(NativeMLP, "small_steps_reason", lambda self, *args, **kw: "off")
    used.clear()
    b = job("ring")
    assert not used
    la, lb = a["history"]["loss"], b["history"]["loss"]
    assert len(la) == len(lb) >= 4
    for x, y in zip(la, lb):
        assert abs(x - y) <= 0.03 * abs(y) + 1e-4, (la, lb)
    assert abs(a["test_loss"] - b["test_loss"]) <= 0.05 * abs(b["test_loss"]) + 1e-4
