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
`LocalComm` is the TP=1 no-op.  `TorchComm` wraps a process group.  On GPU TP groups hand-written
one-shot collectives over IPC-mapped peer buffers (csrc/allreduce.hip, parallel/custom_allreduce.py)
take the small decode messages — the all-reduce fused with the RMSNorm that follows it
(`all_reduce_rmsnorm`) and the argmax all-gather; RCCL keeps the large prefill messages.
"""
from __future__ import annotations

import os
import time
from typing import List, Optional

import torch


# TP decode: the row-parallel O / down projections hand their split-K partials to the fused all-reduce +
# RMSNorm (csrc/allreduce.hip reduces the slabs while staging its contribution).  0: reduce them first
# (splitk_reduce), as before round 6.
TP_SPLITK_NORM = os.environ.get("KA_TP_SPLITK_NORM", "1") == "1"


class CollectiveTimer:
    """Wall time of eager all-reduces for the `rccl_allreduce_seconds` histogram.
    Device tensors: a pair of timing events on the issuing stream, resolved later by `drain()`
    once the end event has completed (no host sync on the hot path); host tensors (gloo): host
    clock.  Collectives inside hipGraph capture are not timed (their replay has no per-node
    events); decode all-reduces therefore show up only in eager / prefill steps."""

    def __init__(self, max_pending: int = 4096):
        self.pending: List = []
        self.done: List[float] = []
        self.max_pending = max_pending

    def begin(self, t: torch.Tensor):
        if t.is_cuda:
            if torch.cuda.is_current_stream_capturing() or len(self.pending) >= self.max_pending:
                return None
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def end(self, tok) -> None:
        if tok is None:
            return
        if isinstance(tok, float):
            self.done.append(time.perf_counter() - tok)
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.pending.append((tok, e))

    def drain(self) -> List[float]:
        keep = []
        for a, b in self.pending:
            if b.query():
                self.done.append(a.elapsed_time(b) / 1e3)
            else:
                keep.append((a, b))
        self.pending = keep
        out, self.done = self.done, []
        return out


class LocalComm:
    world_size = 1
    rank = 0

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return t.unsqueeze(0)

    def all_reduce_rmsnorm(self, t, w, eps, residual=None):
        from .. import ops
        return ops.rmsnorm(t, w, eps, residual=residual)

    splitk_norm = True

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
        # RCCL collectives are ordered on the device stream (the host does not wait for them)
        self.device_ordered = dist.get_backend(group) == "nccl"
        self.custom_ar = None  # optional one-shot all-reduce (parallel/custom_allreduce.py)
        self.allreduce_calls = 0
        self.allreduce_bytes = 0
        self.timer = CollectiveTimer() if os.environ.get("KA_TIME_COLLECTIVES", "1") == "1" else None

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size == 1:
            return t
        self.allreduce_calls += 1
        self.allreduce_bytes += t.numel() * t.element_size()
        tok = self.timer.begin(t) if self.timer is not None else None
        if self.custom_ar is not None and self.custom_ar.should_use(t):
            self.custom_ar.all_reduce(t)
        else:
            self.dist.all_reduce(t, group=self.group)
        if tok is not None:
            self.timer.end(tok)
        return t

    def all_reduce_rmsnorm(self, t, w: torch.Tensor, eps: float, residual=None) -> torch.Tensor:
        """rmsnorm(all_reduce(t) (+ residual)) * w: one fused one-shot launch for decode-size rows
        (residual updated in place), else the all-reduce followed by the RMSNorm kernel.  t may be the
        split-K partials of the row-parallel projection (ops.SplitK): the one-shot kernel reduces them
        while staging its contribution; on the RCCL path they are reduced first."""
        from .. import ops
        if self.world_size > 1 and self.custom_ar is not None and self.custom_ar.can_fuse_norm(t):
            rows, hidden = t.shape
            self.allreduce_calls += 1
            self.allreduce_bytes += rows * hidden * 2
            return self.custom_ar.all_reduce_rmsnorm(t, w, eps, residual)
        if isinstance(t, ops.SplitK):
            t = ops.splitk_resolve(t)
        self.all_reduce(t)
        return ops.rmsnorm(t, w, eps, residual=residual)

    @property
    def splitk_norm(self) -> bool:
        """all_reduce_rmsnorm takes split-K partials (models/llama.py then defers the O / down reduce):
        with the one-shot kernel, unless KA_TP_SPLITK_NORM=0 (the A/B against splitk_reduce first)."""
        return self.custom_ar is not None and TP_SPLITK_NORM

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.custom_ar is not None and self.custom_ar.should_gather(t):
            return self.custom_ar.all_gather(t)
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


class VirtualRankComm:
    """One rank of a `world`-way TP / EP group run ALONE on one GPU, the collectives left out: every
    collective returns its input (all_gather replicates it `world` times, all_to_all returns what this
    rank would keep).  For timing one rank's share of a TP = 8 step (scripts/bench_virtual_rank.py)
    and for tuning the per-rank shard shapes' kernel plans on a single GPU — never for numerics (the
    partial sums are not reduced).  `allreduce_calls` / `allreduce_bytes` count what a real group
    would have exchanged."""

    device_ordered = True
    custom_ar = None
    # the persistent decode kernel (csrc/decode_persistent.hip) may serve this rank: its row-parallel
    # outputs are added to the residual unreduced, which is what every all-reduce here returns
    persistent_no_reduce = True

    def __init__(self, world: int, rank: int = 0):
        self.world_size, self.rank = world, rank
        self.allreduce_calls = 0
        self.allreduce_bytes = 0
        self.timer = None

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        self.allreduce_calls += 1
        self.allreduce_bytes += t.numel() * t.element_size()
        return t

    def all_reduce_rmsnorm(self, t, w: torch.Tensor, eps: float, residual=None) -> torch.Tensor:
        """t: bf16 rows or split-K partials (ops.SplitK, reduced inside the norm kernel as the fused
        one-shot kernel reduces them inside the collective)."""
        from .. import ops
        rows, hidden = t.shape
        self.allreduce_calls += 1
        self.allreduce_bytes += rows * hidden * 2
        return ops.rmsnorm(t, w, eps, residual=residual)

    @property
    def splitk_norm(self) -> bool:   # all_reduce_rmsnorm takes split-K partials (models/llama.py defers the reduce)
        return TP_SPLITK_NORM

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return t.unsqueeze(0).expand((self.world_size,) + tuple(t.shape)).contiguous()

    def all_to_all_single(self, t: torch.Tensor, out_splits=None, in_splits=None) -> torch.Tensor:
        rows = sum(out_splits) if out_splits is not None else t.shape[0]
        out = torch.zeros((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        n = min(rows, t.shape[0])
        out[:n].copy_(t[:n])
        return out

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return t

    def barrier(self) -> None:
        return None


def make_comm(group=None):
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized():
        return LocalComm()
    if dist.get_world_size(group) == 1:
        return LocalComm()
    return TorchComm(group)
