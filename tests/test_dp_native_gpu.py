"""DP pre-flight of the NATIVE engines on one GPU (round-3 VERDICT item 7 / weak #6).

Data parallelism over k ranks computes, per rank, the gradient of its shard of b rows with
grad_scale = 1 / (b k) and sums the k gradients in the flat all-reduce (train/step.py C2). On
one GPU the same arithmetic is k shard passes accumulated into one gradient bucket
(zero_grads only before the first): it must equal ONE pass over the concatenated batch with
grad_scale 1 / (b k) up to fp32 summation order. This pins the engines' grad_scale contract
under DP — the LSTM's sub-batched persistent launches, the MLP's spread-reduction scratch
(accumulating across calls), the CNN's per-workgroup partials — without an 8-GPU box. The
gloo tests (tests/test_dist_gloo.py) cover the collective itself on the fp32 engine.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _check(full_grads, shard_grads, full_loss, shard_loss, tol=1e-3):
    assert abs(full_loss - shard_loss) <= 1e-4 * abs(full_loss) + 1e-6, (full_loss, shard_loss)
    r = _rel(shard_grads, full_grads)
    assert r < tol, r


@pytest.mark.parametrize("k", [2, 8])
def test_lstm_dp_shards_equal_full_batch(k):
    from wellflow.data.synth import synth_lstm_batch
    from wellflow.models.lstm import NativeLSTM, init_lstm_flat

    B, T, F, H = 8192, 16, 16, 512
    b = B // k
    flat = init_lstm_flat(F, H, seed=1).to(DEV)
    x, y = synth_lstm_batch(B, T, F, seed=2)
    x, y = x.to(DEV), y.to(DEV)
    full = NativeLSTM(F, H, T, B, device=DEV)
    full.params.copy_(flat)
    full.sync_weights()
    lf = full.forward_backward(x, y, grad_scale=1.0 / B).item()
    shard = NativeLSTM(F, H, T, b, device=DEV)
    shard.params.copy_(flat)
    shard.sync_weights()
    ls = 0.0
    for r in range(k):
        ls += shard.forward_backward(x[r * b:(r + 1) * b].contiguous(), y[r * b:(r + 1) * b].contiguous(),
                                     grad_scale=1.0 / B, zero_grads=(r == 0)).item()
    torch.cuda.synchronize()
    assert full.last_forward_persistent and shard.last_forward_persistent
    assert full.last_backward_persistent and shard.last_backward_persistent
    full.check_device_errors()
    shard.check_device_errors()
    _check(full.grads, shard.grads, lf, ls)


@pytest.mark.parametrize("k", [2, 8])
def test_mlp_dp_shards_equal_full_batch(k):
    from wellflow.data.synth import synth_tabular_batch
    from wellflow.models.mlp import NativeMLP, init_mlp_flat

    B, F = 262144, 16
    b = B // k
    eng = NativeMLP(F, (256, 256), B, device=DEV)
    eng.params.copy_(init_mlp_flat(F, (256, 256), seed=3).to(DEV))
    eng.sync_weights()
    x, y = synth_tabular_batch(B, F, seed=4)
    x, y = x.to(DEV), y.to(DEV)
    lf = eng.forward_backward(x, y, grad_scale=1.0 / B).item()
    gf = eng.grads.clone()
    ls = 0.0
    for r in range(k):
        ls += eng.forward_backward(x[r * b:(r + 1) * b], y[r * b:(r + 1) * b], grad_scale=1.0 / B,
                                   zero_grads=(r == 0)).item()
    torch.cuda.synchronize()
    _check(gf, eng.grads, lf, ls)


@pytest.mark.parametrize("k", [2, 8])
def test_cnn_dp_shards_equal_full_batch(k):
    from wellflow.models.cnn import CNN1DRegressor, NativeCNN

    B = 65536
    b = B // k
    ref = CNN1DRegressor(dropout=0.0).init_keras(5)
    eng = NativeCNN(ref.layout, batch=B, device=DEV, dropout=0.0, loss="mae_clip")
    assert eng.fused
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()
    g = torch.Generator(device="cpu").manual_seed(6)
    series = torch.randn(B, 60, generator=g).cumsum(1) * 0.1
    x, y = series[:, :48].contiguous().to(DEV), series[:, 48:].contiguous().to(DEV)
    lf = eng.forward_backward(x, y, grad_scale=1.0 / (B * 12)).item()
    gf = eng.grads.clone()
    ls = 0.0
    for r in range(k):
        ls += eng.forward_backward(x[r * b:(r + 1) * b], y[r * b:(r + 1) * b], grad_scale=1.0 / (B * 12),
                                   zero_grads=(r == 0)).item()
    torch.cuda.synchronize()
    _check(gf, eng.grads, lf, ls)
