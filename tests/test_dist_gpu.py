"""Distributed tier on the GPU box (SURVEY.md §4 "Distributed (GPU): RCCL path at world=1"):
the same DistContext code the 8-GPU bench uses, with the backend "nccl" (= RCCL on ROCm),
a torchrun-style env, the per-attempt store prefix, and every collective the trainer calls."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_collectives_world1(monkeypatch):
    import torch.distributed as dist

    from wellflow.parallel.dist import DistContext

    for k, v in {"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(_port()), "TORCHELASTIC_RESTART_COUNT": "0"}.items():
        monkeypatch.setenv(k, v)
    ctx = DistContext.from_env(force_group=True)
    try:
        assert dist.is_initialized() and dist.get_backend() == "nccl"
        assert ctx.distributed and ctx.device.type == "cuda"
        g = torch.arange(1 << 20, device=ctx.device, dtype=torch.float32)
        ref = g.clone()
        ctx.all_reduce_sum_(g)
        torch.cuda.synchronize()
        assert torch.equal(g, ref)  # one rank: the sum is the tensor itself, bitwise
        p = torch.randn(4097, device=ctx.device)
        q = p.clone()
        ctx.broadcast_(p)
        assert torch.equal(p, q)
        a, b, c = ctx.sum_scalars(1.5, 2.0, 3)
        assert (a, b, c) == (1.5, 2.0, 3)
        assert ctx.max_scalar(0.25) == 0.25
        ctx.barrier()
    finally:
        ctx.shutdown()
