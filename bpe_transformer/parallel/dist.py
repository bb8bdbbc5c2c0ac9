"""Process-group setup: one process per GPU, RCCL over xGMI.

Launch with ``torchrun --nproc-per-node N --master-addr 127.0.0.1 ...`` (or any
launcher that exports RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
MASTER_PORT).  On ROCm the ``"nccl"`` backend IS RCCL; CPU-only runs (tests)
use ``"gloo"``.  A hung collective fails after ``timeout_s`` instead of
hanging forever (async error handling is on by default in the RCCL backend).
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_distributed(device: str | None = None, backend: str | None = None, timeout_s: int = 900) -> DistInfo:
    """Initialise the default process group from the launcher environment.

    ``device``: "cuda" or "cpu" (default: cuda if available).  Returns a
    :class:`DistInfo`; single-process runs never touch ``torch.distributed``.
    """
    rank, world, local = env_world()
    use_cuda = (device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
    if use_cuda:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world <= 1:
        return DistInfo(0, 1, 0, dev, None)
    backend = backend or ("nccl" if use_cuda else "gloo")
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kwargs = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if use_cuda and backend == "nccl":
            kwargs["device_id"] = dev
        dist.init_process_group(**kwargs)
    return DistInfo(rank, world, local, dev, backend)


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float, device: torch.device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(dist.get_world_size())
    return t


def cleanup() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
