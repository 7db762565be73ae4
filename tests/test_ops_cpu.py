"""The torch.library op surface registers and traces without a GPU: schemas exist and the
fake (meta) implementations give the right output shapes / dtypes (ops/torch_ops.py)."""
import torch


def test_ops_registered_with_fake_impls():
    import wellflow.ops.torch_ops  # noqa: F401

    for name in ("linear_act", "regression_loss_fwd", "lstm_regressor_fwd", "lstm_regressor_bwd"):
        assert hasattr(torch.ops.wellflow, name), name
    x = torch.empty(64, 13, device="meta")
    W = torch.empty(32, 13, device="meta")
    b = torch.empty(32, device="meta")
    y = torch.ops.wellflow.linear_act(x, W, b, 1)
    assert y.shape == (64, 32) and y.dtype == torch.bfloat16
    ls, d = torch.ops.wellflow.regression_loss_fwd(torch.empty(10, device="meta"), torch.empty(10, device="meta"),
                                                   0, 6.0)
    assert ls.shape == (1,) and d.shape == (10,)
    from wellflow.models.lstm import LstmLayout

    lay = LstmLayout(16, 128)
    outs = torch.ops.wellflow.lstm_regressor_fwd(torch.empty(32, 8, 16, device="meta"),
                                                torch.empty(lay.numel, device="meta"), 128, lay.KX)
    assert outs[0].shape == (32,) and outs[1].numel() == 9 * 32 * lay.KA
