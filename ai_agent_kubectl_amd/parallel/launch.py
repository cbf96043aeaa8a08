"""Process-group bootstrap for tensor / expert parallelism (one process per GPU).

Under `torchrun` (or the driver's `python -m torch.distributed.run`) every rank reads RANK /
WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT from the environment.  On GPUs the backend is
"nccl" — RCCL over xGMI on ROCm — bound to `cuda:LOCAL_RANK`; on CPU (tests) it is "gloo".
`HSA_ENABLE_IPC_MODE_LEGACY=0` must stay exported for RCCL's dmabuf IPC on this platform.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .comm import TorchComm, make_comm


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> Tuple[int, int, int]:
    """Initialise the default process group from the env; returns (rank, world_size, local_rank)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), local
    if backend is None:
        # KA_TP_BACKEND=gloo: several ranks on ONE GPU (tests on a 1-GPU box: RCCL refuses two ranks
        # on one device; the decode collectives still run as the one-shot IPC kernels)
        backend = os.environ.get("KA_TP_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    kw = {"backend": backend, "rank": rank, "world_size": world,
          "timeout": datetime.timedelta(seconds=timeout_s)}
    if backend == "nccl":
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device(f"cuda:{local}")
    dist.init_process_group(**kw)
    return rank, world, local


def init_tp(tp: int, backend: Optional[str] = None):
    """TP group = the whole world (single node, TP <= 8).  Returns (comm, rank)."""
    rank, world, _ = init_distributed(backend)
    if world != tp:
        raise ValueError(f"TP={tp} but WORLD_SIZE={world}: launch with torchrun --nproc-per-node {tp}")
    return make_comm(None), rank
