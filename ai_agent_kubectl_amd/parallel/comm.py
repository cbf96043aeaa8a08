"""Communicators for tensor / expert parallelism.

One process per GPU (`torch.distributed`, backend "nccl" = RCCL over xGMI on ROCm; "gloo" on CPU for
tests).  The model needs four collectives:

* `all_reduce(t)`   — sum, in place: row-parallel O-proj / down-proj outputs (A1, A2) and the
                      expert-parallel MoE combine;
* `all_gather(t)`   — vocab-parallel argmax winners (A3);
* `broadcast(t)`    — per-step metadata from the driver rank (A4);
* `all_to_all_single(t, out_splits, in_splits)` — Mixtral expert dispatch / combine (A5,
                      models/moe.py `moe_alltoall`, eager prefill).

All are issued on the current stream so that they are captured inside decode hipGraphs.
`LocalComm` is the TP=1 no-op.  `TorchComm` wraps a process group.  With KA_CUSTOM_AR=1 a
hand-written one-shot all-reduce over IPC-mapped peer buffers (csrc/allreduce.hip,
parallel/custom_allreduce.py) takes the small bf16 decode messages; RCCL keeps the rest.
"""
from __future__ import annotations

from typing import Optional

import torch


class LocalComm:
    world_size = 1
    rank = 0

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return t.unsqueeze(0)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return t

    def all_to_all_single(self, t: torch.Tensor, out_splits=None, in_splits=None) -> torch.Tensor:
        return t

    def barrier(self) -> None:
        return None


class TorchComm:
    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.custom_ar = None  # optional one-shot all-reduce (parallel/custom_allreduce.py)

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size == 1:
            return t
        if self.custom_ar is not None and self.custom_ar.should_use(t):
            return self.custom_ar.all_reduce(t)
        self.dist.all_reduce(t, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        flat = torch.empty(self.world_size * t.numel(), dtype=t.dtype, device=t.device)
        self.dist.all_gather_into_tensor(flat, t.contiguous().view(-1), group=self.group)
        return flat.view((self.world_size,) + tuple(t.shape))

    def all_to_all_single(self, t: torch.Tensor, out_splits=None, in_splits=None) -> torch.Tensor:
        """A5: rows of `t` grouped by destination rank (`in_splits[j]` rows to rank j); returns the
        rows received from every rank, grouped by source (`out_splits[j]` from rank j).  Without
        splits, t's first dim is divided evenly (used to exchange the split sizes themselves)."""
        rows = sum(out_splits) if out_splits is not None else t.shape[0]
        out = torch.empty((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        self.dist.all_to_all_single(out, t.contiguous(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                                    group=self.group)
        return out

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        self.dist.broadcast(t, src=self.dist.get_global_rank(self.group, src) if self.group else src,
                            group=self.group)
        return t

    def barrier(self) -> None:
        self.dist.barrier(group=self.group)


def make_comm(group=None):
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized():
        return LocalComm()
    if dist.get_world_size(group) == 1:
        return LocalComm()
    return TorchComm(group)
