"""Data-parallel runtime: one process per GPU, RCCL over xGMI (gloo on CPU).

Replaces the reference's Spark/Hadoop layer (cnn.py:49 SparkSession; Readme.md:3) — the
reference has NO gradient communication at all. Call sites (§2.5 [design]):

  C1 ``broadcast_``      parameters from rank 0 once at start (identical init)
  C2 ``all_reduce_sum_`` the flat gradient bucket, once per step
  C3 ``all_reduce_sum_`` [loss_sum, count] per eval so early stopping agrees on all ranks
  C4 ``barrier``         around rank-0 checkpoint writes
  C5 ``broadcast_object`` feature vocabularies fitted on rank 0

Bucket policy for MI355X: every model here is <= ~1.2 M parameters (4.7 MB fp32), far
below the size where splitting the bucket to overlap with backward pays on a 7-link
xGMI mesh (a 4.7 MB ring all-reduce at 8 ranks is ~7-50 us, versus a ~10-30 us RCCL
launch/protocol floor): ONE flat bucket per step is the latency-optimal choice. Larger
models can set ``bucket_bytes`` to split the flat buffer into equal chunks that are
reduced back-to-back on a side stream (see :meth:`all_reduce_sum_`).

Gradient-comm precision (SURVEY.md §2.5 "bf16 halves them", §7.4 item 7 "an fp32 all-reduce
option"): ``comm_dtype`` "fp32" (default) reduces the fp32 bucket as is; "bf16" rounds it into a
preallocated bf16 twin, reduces that (half the bytes on every xGMI hop) and widens the sum back
into the fp32 bucket the optimizer reads. The twin lives as long as the context, so a captured
step graph replays the same cast / reduce / cast on the same addresses.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

COMM_DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16}


def _base_store(rank: int, world: int, timeout_s: float):
    """Client (or, outside the elastic agent, rank-0 server) of the MASTER_* TCP store."""
    from torch.distributed.rendezvous import _create_c10d_store
    return _create_c10d_store(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), rank, world,
                              datetime.timedelta(seconds=timeout_s))


class DistContext:
    def __init__(self, rank: int = 0, world_size: int = 1, local_rank: int = 0,
                 device: torch.device | None = None, backend: str | None = None,
                 bucket_bytes: int = 0, comm_dtype: str = "fp32"):
        self.rank, self.world_size, self.local_rank = rank, world_size, local_rank
        self.device = device or torch.device("cpu")
        self.backend = backend
        self.bucket_bytes = bucket_bytes
        if comm_dtype not in COMM_DTYPES:
            raise ValueError(f"comm_dtype must be one of {sorted(COMM_DTYPES)}, got {comm_dtype!r}")
        self.comm_dtype = comm_dtype
        self._lowp: dict = {}  # fp32 bucket (data_ptr, numel) -> its bf16 reduction twin
        self.forced = False

    # ---------------------------------------------------------------- bootstrap
    @classmethod
    def from_env(cls, backend: str | None = None, timeout_s: float = 600.0,
                 bucket_bytes: int = 0, device: str | None = None,
                 force_group: bool = False, comm_dtype: str = "fp32") -> "DistContext":
        """Read torchrun's RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and init the group.

        Device selection happens BEFORE any CUDA call so each rank pins its own GPU.
        ``force_group`` creates the process group even at world size 1 (tests of the
        RCCL path on a one-GPU box); otherwise a single process runs without one.
        """
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if device is None:
            use_gpu = torch.cuda.is_available()
        else:
            use_gpu = device.startswith("cuda")
        if use_gpu:
            torch.cuda.set_device(local)
            dev = torch.device("cuda", local)
        else:
            dev = torch.device("cpu")
        if (world > 1 or force_group) and not dist.is_initialized():
            backend = backend or ("nccl" if use_gpu else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = dev
            restart = os.environ.get("TORCHELASTIC_RESTART_COUNT")
            if restart is not None and "MASTER_PORT" in os.environ:
                # static rendezvous (--master-addr/--master-port) keeps ONE agent store across
                # torchrun restarts, so a restarted group would read the dead attempt's
                # transport addresses. Namespace every attempt's keys.
                kw["store"] = dist.PrefixStore(f"wellflow/attempt_{restart}", _base_store(rank, world, timeout_s))
            dist.init_process_group(**kw)
        ctx = cls(rank, world, local, dev, backend, bucket_bytes, comm_dtype)
        ctx.forced = bool(force_group)
        return ctx

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return dist.is_initialized() and (self.world_size > 1 or self.forced)

    # ---------------------------------------------------------------- collectives
    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.distributed:
            dist.broadcast(t, src=src)
        return t

    def all_reduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        """C2: in-place SUM over ranks, in ``comm_dtype`` (fp32 tensors only are narrowed)."""
        if not self.distributed:
            return t
        low = COMM_DTYPES[self.comm_dtype]
        if low != torch.float32 and t.dtype == torch.float32:
            key = (t.data_ptr(), t.numel())
            buf = self._lowp.get(key)
            if buf is None:
                buf = self._lowp[key] = torch.empty(t.numel(), dtype=low, device=t.device)
            buf.copy_(t.reshape(-1))
            self._reduce(buf)
            t.reshape(-1).copy_(buf)
            return t
        self._reduce(t)
        return t

    def _reduce(self, t: torch.Tensor) -> None:
        if self.bucket_bytes and t.numel() * t.element_size() > self.bucket_bytes:
            n = max(1, self.bucket_bytes // t.element_size())
            works = [dist.all_reduce(t[i : i + n], async_op=True) for i in range(0, t.numel(), n)]
            for w in works:
                w.wait()
        else:
            dist.all_reduce(t)

    def all_reduce_avg_(self, t: torch.Tensor) -> torch.Tensor:
        self.all_reduce_sum_(t)
        if self.distributed:
            t.div_(self.world_size)
        return t

    def max_scalar(self, x: float) -> float:
        if not self.distributed:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=self._coll_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_scalars(self, *xs: float) -> list:
        if not self.distributed:
            return [float(x) for x in xs]
        t = torch.tensor([float(x) for x in xs], dtype=torch.float64, device=self._coll_device())
        dist.all_reduce(t)
        return [float(v) for v in t.tolist()]

    def broadcast_object(self, obj, src: int = 0):
        if not self.distributed:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src)
        return box[0]

    def barrier(self) -> None:
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def shutdown(self) -> None:
        if dist.is_initialized():
            dist.destroy_process_group()

    def _coll_device(self):
        return self.device if self.backend == "nccl" else torch.device("cpu")
