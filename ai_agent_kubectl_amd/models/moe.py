"""Mixtral sparse MoE block (K11 router + K12 expert GEMMs), expert-parallel.

Each rank owns `E / ep` experts.  Token activations arrive replicated across the TP/EP group (the
attention all-reduce already produced them).  Two ways to combine the experts:

* all-reduce combine (decode, graph-captured): every rank computes the contribution of its own
  experts for every token and the block output is summed by the all-reduce the caller issues
  right after (`LlamaModel.forward`).  Decode messages are a few KB-MB and latency-bound, and the
  collective is shape-static, so it sits inside the decode hipGraphs;
* all-to-all dispatch / combine (`moe_alltoall`, eager prefill when EP > 1 and
  MOE_DISPATCH=a2a, the default; `moe_alltoall_static` with fixed per-pair capacities and no host
  read, graph-capturable, everywhere when MOE_DISPATCH=a2a-static): each rank routes only its 1/ep token shard, sends every
  (token, slot) row to the rank owning its expert (A5 dispatch, `all_to_all_single` with exact
  split sizes), runs its local experts on what it received, sends the rows back (A5 combine),
  applies the router weights at the source and all-gathers the shards.  Per rank that moves
  2·k·T·H/ep (dispatch + combine) + T·H·(ep-1)/ep (all-gather) instead of the ring all-reduce's
  2·T·H·(ep-1)/ep, and the router / top-k work is divided by ep.  xGMI is point-to-point, so the
  all-to-all uses every link at once rather than one ring neighbour.

Execution shapes:
* `moe_hip` (decode, T*k <= 512): device-side routing lists, grouped weight-streaming MFMA GEMMs
  over only the routed rows and a weighted combine (csrc/moe.hip) — shape-static, captured in
  the decode hipGraphs, every local expert's weights streamed once per step;
* `moe_hip_grouped` (prefill on the GPU): the same device-side routing lists feeding the grouped
  LDS-DMA MFMA GEMM (csrc/gemm_mfma.hip, gathered X rows, scattered output rows) — no host sync,
  one launch per projection for all local experts;
* `moe_sorted` (CPU): rows sorted by expert, one host read of the counts per layer, one GEMM per
  contiguous expert segment;
* `moe_grouped`: per-expert nonzero() bucketing (one host sync per expert), kept as a reference;
* `moe_batched`: dense all-experts formulation, kept as a second reference.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import ops


def _dense_routing(x, L, cfg, ep_rank, ep_size):
    logits = F.linear(x, L["router"])                               # [T, E]
    w, ids = ops.moe_topk(logits, cfg.top_k)                        # [T, k] f32 / int32
    dense = torch.zeros((x.shape[0], cfg.num_experts), dtype=torch.float32, device=x.device)
    dense.scatter_(1, ids.long(), w)
    el = cfg.num_experts // ep_size
    return dense[:, ep_rank * el:(ep_rank + 1) * el]                # [T, E_local]


def moe_batched(x, L, cfg, ep_rank, ep_size):
    dw = _dense_routing(x, L, cfg, ep_rank, ep_size)                # [T, El]
    w13, w2 = L["w13"], L["w2"]                                     # [El, 2I, H], [El, H, I]
    El, two_i, H = w13.shape
    T = x.shape[0]
    gu = torch.matmul(x.unsqueeze(0), w13.transpose(1, 2))          # [El, T, 2I]
    act = ops.silu_mul(gu.view(El * T, two_i)).view(El, T, two_i // 2)
    y = torch.matmul(act, w2.transpose(1, 2))                       # [El, T, H]
    out = (y.float() * dw.t().unsqueeze(-1)).sum(0)
    return out.to(x.dtype)


def moe_grouped(x, L, cfg, ep_rank, ep_size):
    dw = _dense_routing(x, L, cfg, ep_rank, ep_size)                # [T, El]
    w13, w2 = L["w13"], L["w2"]
    out = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
    for e in range(w13.shape[0]):
        tok = torch.nonzero(dw[:, e] > 0, as_tuple=False).squeeze(1)
        if tok.numel() == 0:
            continue
        xe = x.index_select(0, tok)
        ye = F.linear(ops.silu_mul(F.linear(xe, w13[e])), w2[e])
        out.index_add_(0, tok, ye.float() * dw.index_select(0, tok)[:, e:e + 1])
    return out.to(x.dtype)


def moe_sorted(x, L, cfg, ep_rank, ep_size):
    """Prefill-sized MoE: (token, slot) rows sorted by local expert on the device, ONE host read
    of the per-expert counts per layer (hipBLASLt needs host shapes), then one contiguous segment
    per expert through hipBLASLt and a weighted index_add combine.  `moe_grouped` reads a nonzero()
    per expert instead — E host syncs per layer, each draining the GPU queue."""
    logits = F.linear(x, L["router"])
    w, ids = ops.moe_topk(logits, cfg.top_k)                        # [T, k] f32 / int32
    T, H = x.shape
    k = cfg.top_k
    w13, w2 = L["w13"], L["w2"]
    el = w13.shape[0]
    flat = ids.reshape(-1).long() - ep_rank * el                    # local expert id per (token, slot)
    key = torch.where((flat >= 0) & (flat < el), flat, torch.full_like(flat, el))   # others sort last
    order = torch.argsort(key, stable=True)
    counts = torch.bincount(key, minlength=el + 1)[:el].tolist()    # the layer's one host sync
    n = sum(counts)
    out = torch.zeros((T, H), dtype=torch.float32, device=x.device)
    if n == 0:
        return out.to(x.dtype)
    rows = order[:n]
    tok = torch.div(rows, k, rounding_mode="floor")
    xs = x.index_select(0, tok)
    ys = torch.empty_like(xs)
    off = 0
    for e, c in enumerate(counts):
        if c:
            ys[off:off + c] = F.linear(ops.silu_mul(F.linear(xs[off:off + c], w13[e])), w2[e])
            off += c
    out.index_add_(0, tok, ys.float() * w.reshape(-1).index_select(0, rows).unsqueeze(1))
    return out.to(x.dtype)


MOE_HIP_MAX_ROWS = 512   # T * top_k handled by the HIP grouped kernel (decode buckets); larger -> grouped hipBLASLt


def moe_hip(x, L, cfg, ep_rank, ep_size):
    """Device-resident MoE block: K11 top-k + K12 align / grouped GEMMs / combine (csrc/moe.hip)."""
    logits = ops.linear(x, L["router"])
    w, ids = ops.moe_topk(logits, cfg.top_k)
    el = cfg.num_experts // ep_size
    return ops.moe_experts(x, L["w13"], L["w2"], w, ids, ep_rank * el)


def moe_hip_grouped(x, L, cfg, ep_rank, ep_size):
    """Prefill-sized MoE block on the GPU without host syncs (ops.moe_experts_grouped)."""
    logits = ops.linear(x, L["router"])
    w, ids = ops.moe_topk(logits, cfg.top_k)
    el = cfg.num_experts // ep_size
    return ops.moe_experts_grouped(x, L["w13"], L["w2"], w, ids, ep_rank * el)


def _local_experts(xr, er, L, e0):
    """FFN_{er[r]}(xr[r]) for received rows whose expert id er[r] (global) is one of this rank's;
    unweighted (the source applies the router weight).  [R, H] in xr's dtype."""
    R = xr.shape[0]
    if R == 0:
        return xr.new_zeros((0, xr.shape[1]))
    w13, w2 = L["w13"], L["w2"]
    if xr.is_cuda and not ops._FORCE_REF:
        ones = torch.ones((R, 1), dtype=torch.float32, device=xr.device)
        fn = ops.moe_experts if R <= MOE_HIP_MAX_ROWS else ops.moe_experts_grouped
        return fn(xr, w13, w2, ones, er.view(R, 1).to(torch.int32), e0)
    out = torch.zeros_like(xr)
    el = er.long() - e0
    # rows of other ranks' experts / padding (id -1, moe_alltoall_static) sort last and stay zero
    el = torch.where((el >= 0) & (el < w13.shape[0]), el, torch.full_like(el, w13.shape[0]))
    order = torch.argsort(el, stable=True)
    counts = torch.bincount(el, minlength=w13.shape[0] + 1)[:w13.shape[0]].tolist()   # one host sync (hipBLASLt shapes)
    n = sum(counts)
    xs = xr.index_select(0, order[:n])
    ys = torch.empty_like(xs)
    off = 0
    for e, c in enumerate(counts):
        if c:
            ys[off:off + c] = F.linear(ops.silu_mul(F.linear(xs[off:off + c], w13[e])), w2[e])
            off += c
    out.index_copy_(0, order[:n], ys)
    return out


def moe_alltoall(x, L, cfg, comm):
    """Token-sharded MoE with all-to-all dispatch / combine (A5).  `x` [T, H] is replicated on every
    rank of `comm`; returns the full MoE output [T, H], replicated (the caller must NOT all-reduce).
    Split sizes are exchanged first (one small all-to-all + host read), so this is the eager path."""
    p, r = comm.world_size, comm.rank
    T, H = x.shape
    k, E = cfg.top_k, cfg.num_experts
    el = E // p
    ts = -(-T // p)                                                  # tokens per shard (last may be short)
    lo, hi = min(T, r * ts), min(T, (r + 1) * ts)
    xs = x[lo:hi]
    t_loc = hi - lo
    w, ids = ops.moe_topk(ops.linear(xs, L["router"]), k) if t_loc else (
        torch.zeros((0, k), dtype=torch.float32, device=x.device), torch.zeros((0, k), dtype=torch.int32,
                                                                               device=x.device))
    flat_ids = ids.reshape(-1).long()                                 # [t_loc * k]
    dest = torch.div(flat_ids, el, rounding_mode="floor")
    order = torch.argsort(dest, stable=True)                         # rows grouped by destination rank
    tok = torch.div(order, k, rounding_mode="floor")
    send_counts = torch.bincount(dest, minlength=p).to(torch.int64)
    recv_counts = comm.all_to_all_single(send_counts)
    sc, rc = send_counts.tolist(), recv_counts.tolist()              # host split sizes (eager path)
    send_x = xs.index_select(0, tok)
    send_e = flat_ids.index_select(0, order).to(torch.int32)
    recv_x = comm.all_to_all_single(send_x, rc, sc)                  # A5 dispatch
    recv_e = comm.all_to_all_single(send_e, rc, sc)
    y = _local_experts(recv_x, recv_e, L, r * el)
    back = comm.all_to_all_single(y, sc, rc)                         # A5 combine: rows return in `order`
    contrib = back.float() * w.reshape(-1).index_select(0, order).unsqueeze(1)
    out = torch.zeros((ts, H), dtype=torch.float32, device=x.device)
    out.index_add_(0, tok, contrib)
    full = comm.all_gather(out.to(x.dtype))                          # [p, ts, H]
    return full.reshape(p * ts, H)[:T]


def moe_alltoall_static(x, L, cfg, comm):
    """A5 with shape-static split sizes, so it can be captured in a hipGraph (no host read): every
    rank sends every rank exactly cap = ts * k rows (the most one destination can get from a shard of
    ts tokens), the rows placed by a device-side running count per destination and the unused slots
    carrying expert id -1 (computed as zero by the receiver).  Same result as `moe_alltoall`; moves
    p * cap rows each way instead of the exact counts -- the price of static shapes, small at decode
    batch sizes where the messages are latency-bound."""
    p, r = comm.world_size, comm.rank
    T, H = x.shape
    k, E = cfg.top_k, cfg.num_experts
    el = E // p
    ts = -(-T // p)
    cap = ts * k
    lo, hi = min(T, r * ts), min(T, (r + 1) * ts)
    xs = x[lo:hi]
    t_loc = hi - lo
    dev = x.device
    if t_loc:
        w, ids = ops.moe_topk(ops.linear(xs, L["router"]), k)
    else:
        w, ids = (torch.zeros((0, k), dtype=torch.float32, device=dev), torch.zeros((0, k), dtype=torch.int32, device=dev))
    flat_ids = ids.reshape(-1).long()                                 # [n = t_loc * k]
    dest = torch.div(flat_ids, el, rounding_mode="floor")
    onehot = (dest.unsqueeze(1) == torch.arange(p, device=dev).unsqueeze(0)).to(torch.int64)   # [n, p]
    pos = (onehot.cumsum(0) - 1).gather(1, dest.unsqueeze(1)).squeeze(1)   # row's index within its destination
    slot = dest * cap + pos                                           # unique in [0, p * cap)
    tok = torch.div(torch.arange(flat_ids.shape[0], device=dev), k, rounding_mode="floor")
    send_x = x.new_zeros((p * cap, H))
    send_x.index_copy_(0, slot, xs.index_select(0, tok))
    send_e = torch.full((p * cap,), -1, dtype=torch.int32, device=dev)
    send_e.index_copy_(0, slot, flat_ids.to(torch.int32))
    recv_x = comm.all_to_all_single(send_x)                           # A5 dispatch, equal splits
    recv_e = comm.all_to_all_single(send_e)
    y = _local_experts(recv_x, recv_e, L, r * el)
    back = comm.all_to_all_single(y)                                  # A5 combine: rows return to `slot`
    contrib = back.index_select(0, slot).float() * w.reshape(-1).unsqueeze(1)
    out = torch.zeros((ts, H), dtype=torch.float32, device=dev)
    out.index_add_(0, tok, contrib)
    full = comm.all_gather(out.to(x.dtype))                          # [p, ts, H]
    return full.reshape(p * ts, H)[:T]


def moe_dispatch_mode() -> str:
    return os.environ.get("MOE_DISPATCH", "a2a")


def moe_forward(x, L, cfg, ep_rank, ep_size, is_decode: bool, comm=None):
    """Returns (out, combined): `combined` is True when the output is already summed over the EP
    group (all-to-all path) and the caller's all-reduce must be skipped."""
    mode = moe_dispatch_mode()
    if comm is not None and ep_size > 1:
        capturing = x.is_cuda and torch.cuda.is_current_stream_capturing()
        # MOE_DISPATCH=a2a (default): exact-count all-to-all for prefill, the all-reduce combine in
        # the decode graphs; a2a-static: the shape-static all-to-all everywhere (graph-capturable)
        if mode == "a2a-static":
            return moe_alltoall_static(x, L, cfg, comm), True
        if mode == "a2a" and not is_decode and not capturing:
            return moe_alltoall(x, L, cfg, comm), True
    if x.is_cuda and not ops._FORCE_REF:
        if x.shape[0] * cfg.top_k <= MOE_HIP_MAX_ROWS:
            return moe_hip(x, L, cfg, ep_rank, ep_size), False
        return moe_hip_grouped(x, L, cfg, ep_rank, ep_size), False
    return moe_sorted(x, L, cfg, ep_rank, ep_size), False
