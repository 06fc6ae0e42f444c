"""Process-per-GPU runtime (replaces Hive's mapper fan-out + YARN).

One process per MI355X, ``torch.distributed`` over RCCL (backend ``"nccl"`` on ROCm) with
xGMI between the 8 GPUs of a node; ``gloo`` for CPU runs and CPU multi-process tests.
Rendezvous is env:// (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT) as set
by ``torch.distributed.run``.  Always 127.0.0.1 for single-node runs.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None

    @property
    def is_dist(self) -> bool:
        return self.world_size > 1 and dist.is_available() and dist.is_initialized()

    def barrier(self) -> None:
        if self.is_dist:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index or 0])
            else:
                dist.barrier()


_CTX: DistContext | None = None


def init_distributed(backend: str | None = None, timeout_s: float = 600.0,
                     device: str | None = None) -> DistContext:
    """Initialise the process group from the torchrun environment (idempotent).

    Single process (no WORLD_SIZE or WORLD_SIZE=1): no process group is created.
    """
    global _CTX
    if _CTX is not None:
        return _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() and device != "cpu"
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    # HM_DIST_BACKEND=gloo: rehearse the multi-rank GPU path with several ranks on one card
    # (RCCL refuses two ranks on the same GPU); production runs use RCCL
    be = backend or os.environ.get("HM_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    _CTX = DistContext(rank, world, local, dev, be if world > 1 else None)
    return _CTX


def context() -> DistContext:
    return _CTX or init_distributed()


def shutdown() -> None:
    global _CTX
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None
