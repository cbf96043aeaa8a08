"""Mixtral sparse MoE block (K11 router + K12 expert GEMMs), expert-parallel.

Each rank owns `E / ep` experts.  Token activations are replicated across the TP/EP group (the
attention all-reduce already produced them), every rank computes the contribution of its own
experts, and the block output is summed across ranks by the all-reduce the caller issues right
after (`LlamaModel.forward`) — the EP combine costs no extra collective.

Execution shapes:
* `moe_hip` (decode, T*k <= 512): device-side routing lists, grouped weight-streaming MFMA GEMMs
  over only the routed rows and a weighted combine (csrc/moe.hip) — shape-static, captured in
  the decode hipGraphs, every local expert's weights streamed once per step;
* `moe_grouped` (prefill / CPU reference): tokens bucketed by expert on the host, hipBLASLt GEMMs
  per expert (ragged, eager);
* `moe_batched`: dense all-experts formulation, kept as a second reference.
"""
from __future__ import annotations

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


MOE_HIP_MAX_ROWS = 512   # T * top_k handled by the HIP grouped kernel (decode buckets); larger -> grouped hipBLASLt


def moe_hip(x, L, cfg, ep_rank, ep_size):
    """Device-resident MoE block: K11 top-k + K12 align / grouped GEMMs / combine (csrc/moe.hip)."""
    logits = ops.linear(x, L["router"])
    w, ids = ops.moe_topk(logits, cfg.top_k)
    el = cfg.num_experts // ep_size
    return ops.moe_experts(x, L["w13"], L["w2"], w, ids, ep_rank * el)


def moe_forward(x, L, cfg, ep_rank, ep_size, is_decode: bool):
    if x.is_cuda and not ops._FORCE_REF and x.shape[0] * cfg.top_k <= MOE_HIP_MAX_ROWS:
        return moe_hip(x, L, cfg, ep_rank, ep_size)
    return moe_grouped(x, L, cfg, ep_rank, ep_size)
