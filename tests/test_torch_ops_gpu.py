"""torch.library custom ops over the HIP kernels (ops/torch_ops.py) against fp32 PyTorch
autograd: forward values, input/parameter gradients, and plain nn.Module training loops
(loss.backward() + torch.optim.Adam) on the native ops."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-30)).item()


@pytest.mark.parametrize("M,K,N,act", [(300, 13, 12, 1), (1024, 64, 256, 1), (257, 40, 96, 0)])
def test_linear_act_matches_fp32_autograd(M, K, N, act):
    import wellflow.ops.torch_ops  # noqa: F401  (registers wellflow::*)

    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV, requires_grad=True)
    W = (torch.randn(N, K, device=DEV) / K ** 0.5).requires_grad_(True)
    b = torch.randn(N, device=DEV, requires_grad=True)
    y = torch.ops.wellflow.linear_act(x, W, b, act)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    g = torch.randn(M, N, device=DEV)
    (y.float() * g).sum().backward()
    # fp32 math on the bf16-rounded operands the MFMA sees: otherwise pre-activations within
    # bf16 rounding of 0 flip the ReLU mask and dominate the gradient comparison
    xr, Wr = (t.detach().to(torch.bfloat16).float().requires_grad_(True) for t in (x, W))
    br = b.detach().clone().requires_grad_(True)
    yr = xr @ Wr.t() + br
    if act:
        yr = torch.relu(yr)
    (yr * g).sum().backward()
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(W.grad, Wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


def test_regression_loss_op():
    from wellflow.ops.torch_ops import regression_loss

    torch.manual_seed(1)
    p = torch.randn(777, device=DEV, requires_grad=True)
    y = torch.randn(777, device=DEV) * 4
    for kind in ("mse", "mae_clip"):
        p.grad = None
        L = regression_loss(p, y, kind)
        L.backward()
        pr = p.detach().clone().requires_grad_(True)
        Lr = ((pr - y) ** 2).sum() if kind == "mse" else torch.clamp((y - pr).abs(), 0, 6).sum()
        Lr.backward()
        assert abs(L.item() - Lr.item()) <= 1e-4 * abs(Lr.item())
        assert _rel(p.grad, pr.grad) < 1e-5


def test_native_mlp_module_trains_like_fp32():
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import MLPRegressor
    from wellflow.ops.torch_ops import NativeMLPModule

    torch.manual_seed(2)
    F = 16
    ref = MLPRegressor(F, (256, 256)).to(DEV)
    mod = NativeMLPModule(F, (256, 256)).to(DEV)
    with torch.no_grad():
        for nl, rl in zip(mod.body, ref.linears()):
            nl.weight.copy_(rl.weight)
            nl.bias.copy_(rl.bias)
        mod.head.load_state_dict(ref.head.state_dict())
    x, y = synth_tabular_batch(8192, F, seed=3)
    x, y = x.to(DEV), y.to(DEV)
    losses = {}
    for name, m in (("native", mod), ("fp32", ref)):
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        ls = []
        for _ in range(30):
            opt.zero_grad()
            L = ((m(x) - y) ** 2).mean()
            L.backward()
            opt.step()
            ls.append(L.item())
        losses[name] = ls
    n, f = losses["native"], losses["fp32"]
    assert n[-1] < 0.5 * n[0]
    assert abs(n[-1] - f[-1]) <= 0.05 * f[-1] + 1e-3, (n[-1], f[-1])


def test_lstm_regressor_op_matches_engine_and_fp32():
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM
    from wellflow.ops.torch_ops import NativeLSTMModule

    B, T, F, H = 1024, 16, 16, 256
    mod = NativeLSTMModule(F, H, seed=4).to(DEV)
    x, y = synth_lstm_batch(B, T, F, seed=5)
    x, y = x.to(DEV), y.to(DEV)
    pred = mod(x)
    L = ((pred - y) ** 2).sum() / B
    L.backward()
    # the imperative engine on the same weights computes the same thing
    eng = NativeLSTM(F, H, T, B, device=DEV)
    eng.params.copy_(mod.flat.detach())
    eng.sync_weights()
    eng.forward_backward(x, y, grad_scale=1.0 / B)
    torch.cuda.synchronize()
    assert _rel(pred.detach(), eng.pred[:B]) < 1e-6
    assert _rel(mod.flat.grad, eng.grads) < 1e-3
    # and fp32 autograd of nn.LSTM (same flat layout through LSTMRegressor.load_flat)
    from wellflow.models.lstm import LSTMRegressor

    ref = LSTMRegressor(F, H)
    ref.load_flat(mod.flat.detach().cpu())
    ref = ref.to(DEV)
    Lr = ((ref(x) - y) ** 2).sum() / B
    Lr.backward()
    assert abs(L.item() - Lr.item()) <= 2e-2 * Lr.item()
    gr = torch.cat([p.grad.reshape(-1) for p in (ref.lstm.weight_ih_l0, ref.lstm.weight_hh_l0)])
    assert gr.norm().item() > 0
    # a few Adam steps through the op learn
    opt = torch.optim.Adam(mod.parameters(), lr=1e-3)
    ls = []
    for _ in range(10):
        opt.zero_grad()
        L = ((mod(x) - y) ** 2).mean()
        L.backward()
        opt.step()
        ls.append(L.item())
    assert ls[-1] < ls[0]


def test_fake_tensor_shapes():
    import wellflow.ops.torch_ops  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        x = torch.empty(64, 13, device=DEV)
        W = torch.empty(32, 13, device=DEV)
        b = torch.empty(32, device=DEV)
        y = torch.ops.wellflow.linear_act(x, W, b, 1)
        assert y.shape == (64, 32) and y.dtype == torch.bfloat16
