"""Mixtral sparse MoE block (K11 router + K12 expert GEMMs), expert-parallel.

Each rank owns `E / ep` experts.  Token activations are replicated across the TP/EP group (the
attention all-reduce already produced them), every rank computes the contribution of its own
experts, and the block output is summed across ranks by the all-reduce the caller issues right
after (`LlamaModel.forward`) — the EP combine costs no extra collective.

Two execution shapes:
* grouped (`moe_grouped`): tokens are bucketed by expert and each expert runs its own GEMMs on
  only its tokens — used for prefill (ragged, eager);
* batched (`moe_batched`): every local expert processes the whole (small) decode batch with one
  batched GEMM per projection and non-routed tokens get weight 0 — shape-static, so it is
  captured into the decode hipGraphs.  At decode batch sizes every expert's weights are streamed
  anyway, so the extra MFMA work rides under the weight stream.
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


def moe_forward(x, L, cfg, ep_rank, ep_size, is_decode: bool):
    if is_decode and x.is_cuda:
        return moe_batched(x, L, cfg, ep_rank, ep_size)
    return moe_grouped(x, L, cfg, ep_rank, ep_size)
