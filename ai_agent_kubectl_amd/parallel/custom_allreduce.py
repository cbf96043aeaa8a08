"""One-shot all-reduce for small tensor-parallel messages (csrc/allreduce.hip).

SURVEY.md §2.6: decode all-reduces are 8-16 KB x batch and latency-bound; RCCL's ring is per-link bound
on xGMI, a one-shot kernel reads every peer at once over its own link.  Setup (once per TP group):

1. every rank allocates one uncached device buffer ([2 x cap] bf16 data halves + per-block flags)
   with `ka_ar_alloc`; its epoch / done / error counters are a local int32 tensor;
2. the 64-byte hipIpc handles are exchanged over the process group (`all_gather_object`) and every
   peer buffer is mapped with `ka_ar_open_handle`;
3. `all_reduce(t)` launches `ka_allreduce_oneshot` on the current stream (graph-capturable: the
   epoch lives in device memory).

`should_use` routes bf16 tensors up to `cap` elements here; larger (prefill) messages stay on RCCL.
On by default for GPU TP groups (KA_CUSTOM_AR=0 disables it; parallel/comm.py `TorchComm`): the
decode all-reduces run fused with the following residual add + RMSNorm (`all_reduce_rmsnorm`), the
vocab-parallel argmax all-gather (`all_gather`) shares the buffers, so a TP decode hipGraph holds
every collective.  `err` is set by a kernel if a peer never arrived (bounded spin instead of a GPU
hang) and is checked by `check()`.
"""
from __future__ import annotations

import ctypes
import os
from typing import List

import torch

AR_MAX_RANKS = 8
AR_MAX_BLOCKS = 64
FLAG_BYTES = AR_MAX_BLOCKS * AR_MAX_RANKS * 4


def _lib():
    from ..ops._hip import check, require
    return require(), check


class OneShotAllReduce:
    def __init__(self, group=None, device=None, cap_elems: int = 4 << 20):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > AR_MAX_RANKS:
            raise ValueError(f"one-shot all-reduce supports up to {AR_MAX_RANKS} ranks")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cap = int(cap_elems) // 8 * 8
        lib, check = _lib()
        self.lib, self.check_rc = lib, check
        # + the persistent decode kernel's own exchange halves and flags (csrc/decode_persistent.hip
        # xreduce: a separate epoch sequence, so it never shares halves with the one-shot kernels)
        self.pd_off = 2 * self.cap * 2 + FLAG_BYTES
        self.bytes = self.pd_off + int(lib.ka_decode_persistent_xbytes())
        base = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.ka_ar_alloc(ctypes.byref(base), ctypes.c_size_t(self.bytes)), "ar_alloc")
            torch.cuda.synchronize(self.device)
        self.base = base.value
        handle = ctypes.create_string_buffer(64)
        check(lib.ka_ar_get_handle(ctypes.c_void_p(self.base), handle), "ar_get_handle")
        handles: List[bytes] = [None] * self.world  # type: ignore[list-item]
        dist.all_gather_object(handles, handle.raw, group=group)
        self.peers: List[int] = []
        self._opened: List[int] = []
        with torch.cuda.device(self.device):
            for p, h in enumerate(handles):
                if p == self.rank:
                    self.peers.append(self.base)
                    continue
                ptr = ctypes.c_void_p()
                check(lib.ka_ar_open_handle(ctypes.create_string_buffer(h, 64), ctypes.byref(ptr)), "ar_open_handle")
                self.peers.append(ptr.value)
                self._opened.append(ptr.value)
        flag_off = 2 * self.cap * 2
        self._data = (ctypes.c_void_p * self.world)(*self.peers)
        self._flags = (ctypes.c_void_p * self.world)(*[p + flag_off for p in self.peers])
        self.state = torch.zeros(4, dtype=torch.int32, device=self.device)   # ctr, done, err
        sp = self.state.data_ptr()
        self._ctr, self._done, self._err = sp, sp + 4, sp + 8
        pf = int(lib.ka_decode_persistent_xflag_offset())
        self._pd_data = (ctypes.c_void_p * 8)(*[p + self.pd_off for p in self.peers])
        self._pd_flags = (ctypes.c_void_p * 8)(*[p + self.pd_off + pf for p in self.peers])
        self.pd_ctr = torch.zeros(1, dtype=torch.int32, device=self.device)   # the kernel's epoch counter
        dist.barrier(group=group)

    def pd_exchange(self):
        """(world, rank, xdata, xflag, xctr) for ops.decode_persistent's in-kernel all-reduce."""
        return self.world, self.rank, self._pd_data, self._pd_flags, self.pd_ctr

    # ------------------------------------------------------------------------------------------
    def should_use(self, t: torch.Tensor) -> bool:
        return (t.dtype == torch.bfloat16 and t.is_cuda and t.is_contiguous() and t.numel() % 8 == 0
                and 0 < t.numel() <= self.cap)

    @staticmethod
    def blocks_for(n: int) -> int:
        return max(1, min(AR_MAX_BLOCKS, (n + 8 * 512 - 1) // (8 * 512)))

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        n = t.numel()
        stream = torch.cuda.current_stream(t.device).cuda_stream
        self.check_rc(self.lib.ka_allreduce_oneshot(
            ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()), self._data, self._flags,
            ctypes.c_void_p(self._ctr), ctypes.c_void_p(self._done), ctypes.c_void_p(self._err),
            self.rank, self.world, n, self.cap, self.blocks_for(n), ctypes.c_void_p(stream)), "allreduce_oneshot")
        return t

    def can_fuse_norm(self, t) -> bool:
        """t: a bf16 [rows, hidden] partial, or the `ops.SplitK` partial slabs of the producing GEMM."""
        from .. import ops
        if isinstance(t, ops.SplitK):
            rows, hidden = t.shape
            return (t.P.is_cuda and t.P.is_contiguous() and hidden % 8 == 0 and hidden <= 8192
                    and 0 < rows * hidden <= self.cap)
        return self.should_use(t) and t.dim() == 2 and t.shape[1] % 8 == 0 and t.shape[1] <= 8192

    def all_reduce_rmsnorm(self, t, w: torch.Tensor, eps: float, residual=None, out=None) -> torch.Tensor:
        """rmsnorm(sum_ranks(t) (+ residual)) * w in one launch (residual updated in place).  A SplitK
        input is reduced over its slabs inside the same launch (no splitk_reduce kernel)."""
        from .. import ops
        if isinstance(t, ops.SplitK):
            src, split, in_bf16 = t.P, t.split, int(t.is_bf16)
            rows, hidden = t.shape
        else:
            src, split, in_bf16 = t, 1, 1
            rows, hidden = t.shape
        out = torch.empty((rows, hidden), dtype=w.dtype, device=w.device) if out is None else out
        stream = torch.cuda.current_stream(src.device).cuda_stream
        self.check_rc(self.lib.ka_allreduce_rmsnorm(
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(src.data_ptr()),
            ctypes.c_void_p(residual.data_ptr() if residual is not None else 0), ctypes.c_void_p(w.data_ptr()),
            float(eps), self._data, self._flags, ctypes.c_void_p(self._ctr), ctypes.c_void_p(self._done),
            ctypes.c_void_p(self._err), self.rank, self.world, rows, hidden, self.cap, min(rows, AR_MAX_BLOCKS),
            split, in_bf16, ctypes.c_void_p(stream)), "allreduce_rmsnorm")
        return out

    def should_gather(self, t: torch.Tensor) -> bool:
        nb = t.numel() * t.element_size()
        return t.is_cuda and t.is_contiguous() and 0 < nb and (nb + 15) // 16 * 8 <= self.cap

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] (A3: vocab-parallel argmax winners); same buffers / epoch as all_reduce,
        graph-capturable.  Any dtype: moved as 16-byte units (padded)."""
        nb = t.numel() * t.element_size()
        n16 = (nb + 15) // 16 * 8
        src = t.contiguous().view(torch.uint8)
        if nb != n16 * 2:
            padded = torch.zeros(n16 * 2, dtype=torch.uint8, device=t.device)
            padded[:nb].copy_(src.view(-1))
            src = padded
        out = torch.empty((self.world, n16 * 2), dtype=torch.uint8, device=t.device)
        stream = torch.cuda.current_stream(t.device).cuda_stream
        self.check_rc(self.lib.ka_allgather_oneshot(
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(src.data_ptr()), self._data, self._flags,
            ctypes.c_void_p(self._ctr), ctypes.c_void_p(self._done), ctypes.c_void_p(self._err),
            self.rank, self.world, n16, self.cap, self.blocks_for(n16), ctypes.c_void_p(stream)), "allgather_oneshot")
        return out[:, :nb].contiguous().view(t.dtype).view((self.world,) + tuple(t.shape))

    def check(self) -> None:
        """Raise if any launch timed out waiting for a peer (the kernel's bounded spin)."""
        if int(self.state[2].item()):
            raise RuntimeError("one-shot all-reduce: a peer never arrived (spin timeout)")

    def close(self) -> None:
        if getattr(self, "base", None) is None:
            return
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.lib.ka_ar_close_handle(ctypes.c_void_p(p))
        self.lib.ka_ar_free(ctypes.c_void_p(self.base))
        self.base = None


def maybe_enable(comm, device) -> None:
    """Attach the one-shot collectives to a TorchComm whose ranks are on GPUs (default; KA_CUSTOM_AR=0
    keeps every collective on RCCL)."""
    if os.environ.get("KA_CUSTOM_AR", "1") != "1":
        return
    if getattr(comm, "world_size", 1) <= 1 or torch.device(device).type != "cuda":
        return
    if not hasattr(comm, "group"):   # not a torch.distributed comm (e.g. the virtual-TP test comm)
        return
    comm.custom_ar = OneShotAllReduce(comm.group, device, int(os.environ.get("KA_CUSTOM_AR_ELEMS", 4 << 20)))
