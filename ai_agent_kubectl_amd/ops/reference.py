"""Plain-PyTorch fp32 reference implementations of every engine op.

These define the semantics the HIP kernels (`csrc/*.hip`) must match; the GPU numerics tests
compare kernel output against them, and CPU-only runs (tests, no GPU) execute the engine through
them.  Layouts are documented in `csrc/elementwise.hip` / `csrc/attention.hip`.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x @ w.T computed in fp32 (the reference for every projection), returned in x's dtype."""
    return torch.nn.functional.linear(x.float(), w.float()).to(x.dtype)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    if residual is not None:
        r = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(r)
        x = r
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq: int, hkv: int, d: int):
    T = qkv.shape[0]
    half = d // 2
    q = qkv[:, : hq * d].view(T, hq, d).float()
    k = qkv[:, hq * d: (hq + hkv) * d].view(T, hkv, d).float()
    v = qkv[:, (hq + hkv) * d:].view(T, hkv, d)
    cs = cos_sin[positions.long()]
    cos, sin = cs[:, None, :half], cs[:, None, half:]

    def rot(x):
        x1, x2 = x[..., :half], x[..., half:]
        return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)

    q_out = rot(q).to(qkv.dtype)
    k_rot = rot(k).to(qkv.dtype)
    bs = k_cache.shape[2]
    slots = slot_mapping.long()
    valid = slots >= 0
    if valid.any():
        s = slots[valid]
        blk, off = s // bs, s % bs
        k_cache[blk, :, off, :] = k_rot[valid].to(k_cache.dtype)
        v_cache[blk, :, :, off] = v[valid].to(v_cache.dtype)
    return q_out


def _gather_kv(k_cache, v_cache, table_row, ctx: int):
    bs = k_cache.shape[2]
    nb = (ctx + bs - 1) // bs
    blocks = table_row[:nb].long()
    k = k_cache[blocks]                       # [nb, Hkv, bs, D]
    v = v_cache[blocks].transpose(-1, -2)     # [nb, Hkv, bs, D]
    k = k.permute(1, 0, 2, 3).reshape(k.shape[1], nb * bs, -1)[:, :ctx]
    v = v.permute(1, 0, 2, 3).reshape(v.shape[1], nb * bs, -1)[:, :ctx]
    return k.float(), v.float()               # [Hkv, ctx, D]


def attention_prefill(q, k_cache, v_cache, block_tables, q_starts, ctx_lens, scale: float):
    T, hq, d = q.shape
    hkv = k_cache.shape[1]
    G = hq // hkv
    out = torch.zeros_like(q)
    qs = q_starts.tolist()
    cl = ctx_lens.tolist()
    for s in range(len(cl)):
        q0, q1, ctx = qs[s], qs[s + 1], cl[s]
        qlen = q1 - q0
        if qlen == 0 or ctx == 0:      # ctx 0 = padding row of a bucketed decode batch
            continue
        k, v = _gather_kv(k_cache, v_cache, block_tables[s], ctx)
        k = k.repeat_interleave(G, dim=0)
        v = v.repeat_interleave(G, dim=0)
        qq = q[q0:q1].float().transpose(0, 1)            # [Hq, qlen, D]
        sc = torch.matmul(qq, k.transpose(-1, -2)) * scale  # [Hq, qlen, ctx]
        qpos = torch.arange(ctx - qlen, ctx, device=q.device)
        kpos = torch.arange(ctx, device=q.device)
        sc = sc.masked_fill(kpos[None, None, :] > qpos[None, :, None], float("-inf"))
        p = torch.softmax(sc, dim=-1)
        out[q0:q1] = torch.matmul(p, v).transpose(0, 1).to(q.dtype)
    return out


def attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale: float):
    B = q.shape[0]
    starts = torch.arange(B + 1, dtype=torch.int32, device=q.device)
    return attention_prefill(q, k_cache, v_cache, block_tables, starts, ctx_lens, scale)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    i = gu.shape[-1] // 2
    g, u = gu[..., :i].float(), gu[..., i:].float()
    return (F.silu(g) * u).to(gu.dtype)


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_offset: int = 0) -> torch.Tensor:
    local = ids.long() - vocab_offset
    valid = (local >= 0) & (local < table.shape[0])
    out = table[local.clamp(0, table.shape[0] - 1)]
    return out * valid[:, None].to(out.dtype)


def masked_argmax(logits, mask_bits, mask_idx, vocab_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    lf = logits.float().clone()
    V = lf.shape[1]
    if mask_bits is not None and mask_idx is not None:
        gid = torch.arange(V, device=logits.device) + vocab_offset
        words = mask_bits[:, gid // 32].long()                      # [M, V]
        allowed = ((words >> (gid % 32)) & 1).bool()
        mi = mask_idx.long().to(logits.device)
        rows = allowed[mi.clamp(min=0)] | (mi < 0)[:, None]
        lf = lf.masked_fill(~rows, float("-inf"))
    idx = torch.argmax(lf, dim=-1)   # documented: first index of the maximum (= kernel tie-break)
    val = lf.gather(1, idx[:, None]).squeeze(1)
    return (idx + vocab_offset).to(torch.int32), val


def moe_topk(router_logits: torch.Tensor, k: int):
    p = torch.softmax(router_logits.float(), dim=-1)
    w, ids = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, ids.to(torch.int32)


def argmax_combine(vals: torch.Tensor, idxs: torch.Tensor) -> torch.Tensor:
    """[ranks, S] (value, global id) pairs -> [S] int32: the largest value, the lowest id on ties."""
    v = vals.float()
    best = v.max(dim=0, keepdim=True).values
    big = torch.iinfo(torch.int32).max
    cand = torch.where(v == best, idxs.to(torch.int64), torch.full_like(idxs, big, dtype=torch.int64))
    return cand.min(dim=0).values.to(torch.int32)
