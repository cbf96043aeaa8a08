"""Engine ops: one implementation per op on the GPU (hand-written HIP, `csrc/`), the fp32 torch
reference (`ops/reference.py`) for CPU tensors.

Dispatch is by tensor device only: a CUDA (HIP) tensor always goes to the HIP kernel and raises if
the kernel library is missing; CPU tensors (tests, no-GPU development) go to the reference.
GEMMs that are plain library GEMMs use `torch.nn.functional.linear` (hipBLASLt) except where a
hand-written kernel wins (decode GEMV, MoE grouped GEMM).
"""
from __future__ import annotations

import bisect
import os
from typing import NamedTuple, Optional, Tuple

import torch

from . import reference as ref
from ._hip import check, require


_FORCE_REF = False
_REF_FP32 = False


class force_reference:
    """Test-only context: run the fp32 torch references even on GPU tensors (model-level parity).
    fp32=True: the model also carries its activations and residual stream in fp32 between the ops
    (models/llama.py), so only the weights and the KV cache are bf16 — the fp32 truth a greedy token
    is compared against; fp32=False: every op rounds its output to bf16 as the engine's kernels do."""

    def __init__(self, fp32: bool = False):
        self.fp32 = fp32

    def __enter__(self):
        global _FORCE_REF, _REF_FP32
        self._old = (_FORCE_REF, _REF_FP32)
        _FORCE_REF, _REF_FP32 = True, self.fp32

    def __exit__(self, *exc):
        global _FORCE_REF, _REF_FP32
        _FORCE_REF, _REF_FP32 = self._old


def reference_fp32() -> bool:
    """Inside force_reference(fp32=True)."""
    return _FORCE_REF and _REF_FP32


def _ref(t: torch.Tensor) -> bool:
    return _FORCE_REF or not t.is_cuda


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream() -> int:
    """Current HIP stream handle (the capture stream inside hipGraph capture).  The raw C accessor
    costs ~0.3 us; torch.cuda.current_stream() ~8 us, paid per kernel launch in eager steps."""
    if _raw_stream is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream().cuda_stream


class SplitK(NamedTuple):
    """Split-K partials of a projection whose reduction is deferred to the consumer (rmsnorm,
    decode_attention_rope, rope_kv_write, silu_mul).  P is fp32, or bf16 when the producer was
    asked for `bf16_partials` (only rmsnorm and the fused decode attention read those)."""
    P: torch.Tensor          # [split, M, N] fp32 | bf16
    split: int

    @property
    def is_bf16(self) -> bool:
        return self.P.dtype == torch.bfloat16

    @property
    def shape(self):
        return self.P.shape[1:]

    def fp32(self) -> "SplitK":
        """The fp32 partials a consumer without a bf16 path (RoPE, attention, SiLU) needs."""
        if self.is_bf16:
            raise TypeError("bf16 split-K partials are only consumed by rmsnorm and decode_attention_rope")
        return self

    def resolve(self) -> torch.Tensor:
        """bf16 [M, N] (for consumers without a fused path)."""
        return self.P.float().sum(0).to(torch.bfloat16)


def splitk_resolve(t: SplitK) -> torch.Tensor:
    """bf16 [M, N] sum of split-K partials (the RCCL all-reduce path of a TP rank, which cannot read
    the slabs itself)."""
    return t.resolve()


def rmsnorm(x, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = rmsnorm(x (+ residual)) * w; when `residual` is given it is updated in place to x + residual.
    `x` may be a `SplitK` (partials of the producing GEMM): the reduction is fused into the norm."""
    if isinstance(x, SplitK):
        lib = require()
        rows, hidden = x.shape
        out = torch.empty((rows, hidden), dtype=w.dtype, device=w.device) if out is None else out
        check(lib.ka_rmsnorm_splitk(_p(out), _p(residual), _p(x.P), x.split, int(x.is_bf16), _p(w), rows, hidden,
                                    float(eps), _stream()), "rmsnorm_splitk")
        return out
    if _ref(x):
        return ref.rmsnorm(x, w, eps, residual)
    lib = require()
    out = torch.empty_like(x) if out is None else out
    rows, hidden = x.shape[0], x.shape[-1]
    check(lib.ka_rmsnorm(_p(out), _p(residual), _p(x), _p(w), rows, hidden, float(eps), _stream()), "rmsnorm")
    return out


def kv_block_copy(k_cache: torch.Tensor, v_cache: torch.Tensor, src: torch.Tensor, dst: torch.Tensor) -> None:
    """k_cache[:, dst] = k_cache[:, src] and the same for v_cache ([L, NB, ...] paged caches; src/dst
    int32 device tensors of equal length) — the sub-block prefix-reuse copy."""
    if _ref(k_cache):
        s, d = src.long(), dst.long()
        k_cache[:, d] = k_cache[:, s]
        v_cache[:, d] = v_cache[:, s]
        return
    lib = require()
    L, NB = k_cache.shape[0], k_cache.shape[1]
    block_elems = k_cache[0, 0].numel()
    check(lib.ka_kv_block_copy(_p(k_cache), _p(v_cache), _p(src), _p(dst), src.shape[0], L, NB * block_elems,
                               block_elems, _stream()), "kv_block_copy")


def rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq: int, hkv: int, d: int,
                  q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """RoPE on q/k + paged KV append.  `qkv` may be a `SplitK` (the QKV projection's fp32 partials):
    the reduction then happens inside this kernel (bit-identical to reduce-then-rope)."""
    if isinstance(qkv, SplitK):
        lib = require()
        qkv = qkv.fp32()
        T = qkv.shape[0]
        q_out = torch.empty((T, hq, d), dtype=k_cache.dtype, device=k_cache.device) if q_out is None else q_out
        check(lib.ka_rope_kv_splitk(_p(q_out), _p(k_cache), _p(v_cache), _p(qkv.P), qkv.split, _p(positions),
                                    _p(cos_sin), _p(slot_mapping), T, hq, hkv, d, k_cache.shape[2], _stream()),
              "rope_kv_splitk")
        return q_out
    if _ref(qkv):
        return ref.rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, d)
    lib = require()
    T = qkv.shape[0]
    q_out = torch.empty((T, hq, d), dtype=qkv.dtype, device=qkv.device) if q_out is None else q_out
    check(lib.ka_rope_kv(_p(q_out), _p(k_cache), _p(v_cache), _p(qkv), _p(positions), _p(cos_sin),
                         _p(slot_mapping), T, hq, hkv, d, k_cache.shape[2], _stream()), "rope_kv")
    return q_out


def attention_prefill(q, k_cache, v_cache, block_tables, q_starts, ctx_lens, max_q_len: int, scale: float,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _ref(q):
        r = ref.attention_prefill(q, k_cache, v_cache, block_tables, q_starts, ctx_lens, scale)
        if out is None:
            return r
        for i in range(ctx_lens.shape[0]):   # only this call's sequences' rows, like the kernel
            out[int(q_starts[i]):int(q_starts[i + 1])] = r[int(q_starts[i]):int(q_starts[i + 1])]
        return out
    lib = require()
    out = torch.empty_like(q) if out is None else out
    S = ctx_lens.shape[0]
    check(lib.ka_paged_prefill(_p(out), _p(q), _p(k_cache), _p(v_cache), _p(block_tables), block_tables.shape[1],
                               _p(q_starts), _p(ctx_lens), S, int(max_q_len), q.shape[1], k_cache.shape[1],
                               q.shape[2], k_cache.shape[2], float(scale), _stream()), "paged_prefill")
    return out


def attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale: float,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _ref(q):
        r = ref.attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale)
        if out is None:
            return r
        out.copy_(r)
        return out
    lib = require()
    out = torch.empty_like(q) if out is None else out
    check(lib.ka_paged_decode(_p(out), _p(q), _p(k_cache), _p(v_cache), _p(block_tables), block_tables.shape[1],
                              _p(ctx_lens), q.shape[0], q.shape[1], k_cache.shape[1], q.shape[2], k_cache.shape[2],
                              float(scale), _stream()), "paged_decode")
    return out


_CASCADE_WS = {}


def cascade_ok(B: int, hq: int, hkv: int) -> bool:
    g = hq // hkv
    return hq % hkv == 0 and g in (1, 2, 4, 8)


def decode_attention_rope(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, block_tables, ctx_lens,
                          hq: int, hkv: int, d: int, scale: float, out: Optional[torch.Tensor] = None,
                          shared_blocks: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One decode token per sequence: RoPE + paged-KV append + paged attention in ONE kernel
    (attention.hip, paged_decode_kernel<true>): the rotated queries never leave the chip and the new
    token is merged from LDS.  `qkv` may be a `SplitK` (the QKV projection's fp32 or bf16 partials).
    shared_blocks (device int32 [1]): the number of leading block-table entries the whole batch
    shares (prefix cache); > 0 runs the cascade (the shared blocks attended once per kv head and 16
    query rows by cascade_prefix_kernel, merged with each sequence's own part).  Equivalent to
    `attention_decode(rope_kv_write(qkv, ...), ...)` (the CPU path)."""
    lead = qkv.P if isinstance(qkv, SplitK) else qkv
    if _ref(lead) or d != 128 or k_cache.shape[2] != 16 or hq % hkv or hq // hkv > 15:
        if isinstance(qkv, SplitK) and qkv.is_bf16:
            qkv = qkv.resolve()
        q = rope_kv_write(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, hq, hkv, d)
        return attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, out=out)
    lib = require()
    B = ctx_lens.shape[0]
    out = torch.empty((B, hq, d), dtype=k_cache.dtype, device=k_cache.device) if out is None else out
    if isinstance(qkv, SplitK):   # fp32 or bf16 partials: the prologue reduces either
        src, P, split, pb = None, _p(qkv.P), qkv.split, int(qkv.is_bf16)
    else:
        src, P, split, pb = _p(qkv), None, 1, 0
    if shared_blocks is not None and cascade_ok(B, hq, hkv):
        key = (k_cache.device, B, hq)
        ws = _CASCADE_WS.get(key)
        if ws is None:   # allocated by the eager warm-up before graph capture
            ws = torch.empty(int(lib.ka_decode_cascade_ws(B, hq)), dtype=torch.uint8, device=k_cache.device)
            _CASCADE_WS[key] = ws
        check(lib.ka_paged_decode_rope_cascade(_p(out), src, P, split, pb, _p(k_cache), _p(v_cache), _p(positions),
                                               _p(cos_sin), _p(slot_mapping), _p(block_tables), block_tables.shape[1],
                                               _p(ctx_lens), B, hq, hkv, d, k_cache.shape[2], float(scale),
                                               _p(shared_blocks), _p(ws), _stream()), "paged_decode_rope_cascade")
        return out
    check(lib.ka_paged_decode_rope(_p(out), src, P, split, pb, _p(k_cache), _p(v_cache), _p(positions), _p(cos_sin),
                                   _p(slot_mapping), _p(block_tables), block_tables.shape[1], _p(ctx_lens), B, hq,
                                   hkv, d, k_cache.shape[2], float(scale), _stream()), "paged_decode_rope")
    return out


def silu_mul(gu, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up of the fused gate_up output; `gu` may be a `SplitK` (reduction fused in)."""
    if isinstance(gu, SplitK):
        lib = require()
        gu = gu.fp32()
        T, two_i = gu.shape
        out = torch.empty((T, two_i // 2), dtype=torch.bfloat16, device=gu.P.device) if out is None else out
        check(lib.ka_silu_mul_splitk(_p(out), _p(gu.P), gu.split, T, two_i // 2, _stream()), "silu_mul_splitk")
        return out
    if _ref(gu):
        return ref.silu_mul(gu)
    lib = require()
    T, two_i = gu.shape
    out = torch.empty((T, two_i // 2), dtype=gu.dtype, device=gu.device) if out is None else out
    check(lib.ka_silu_mul(_p(out), _p(gu), T, two_i // 2, _stream()), "silu_mul")
    return out


def prefetch(t: torch.Tensor, nbytes: int = 0, blocks: int = 0) -> None:
    """Read the first `nbytes` (default: all) of `t` once and discard them: pulls a weight into the
    Infinity Cache ahead of the kernel that streams it (csrc/elementwise.hip prefetch_kernel).  No-op
    on CPU tensors."""
    if _ref(t):
        return
    lib = require()
    n = t.numel() * t.element_size()
    n = min(n, nbytes) if nbytes > 0 else n
    check(lib.ka_prefetch(_p(t), n, int(blocks), None, _stream()), "prefetch")


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_offset: int = 0,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _ref(table):
        return ref.embedding(ids, table, vocab_offset)
    lib = require()
    T = ids.shape[0]
    out = torch.empty((T, table.shape[1]), dtype=table.dtype, device=table.device) if out is None else out
    check(lib.ka_embedding(_p(out), _p(ids), _p(table), T, table.shape[1], table.shape[0], int(vocab_offset),
                           _stream()), "embedding")
    return out


def masked_argmax(logits: torch.Tensor, mask_bits: Optional[torch.Tensor], mask_idx: Optional[torch.Tensor],
                  vocab_offset: int = 0, out_idx: Optional[torch.Tensor] = None,
                  out_val: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Greedy token per row among tokens allowed by mask row `mask_idx[r]` (-1 = all)."""
    if _ref(logits):
        return ref.masked_argmax(logits, mask_bits, mask_idx, vocab_offset)
    lib = require()
    B, V = logits.shape
    out_idx = torch.empty(B, dtype=torch.int32, device=logits.device) if out_idx is None else out_idx
    out_val = torch.empty(B, dtype=torch.float32, device=logits.device) if out_val is None else out_val
    words = mask_bits.shape[1] if mask_bits is not None else 0
    slices = lib.ka_argmax_slices(B, V)   # small batches: the row is split over workgroups
    ws = torch.empty(2 * B * slices, dtype=torch.float32, device=logits.device) if slices > 1 else None
    check(lib.ka_masked_argmax(_p(out_idx), _p(out_val), _p(logits), _p(mask_bits),
                               _p(mask_idx) if mask_bits is not None else None, B, V, words, int(vocab_offset),
                               _p(ws), slices, _stream()), "masked_argmax")
    return out_idx, out_val


def argmax_combine(vals: torch.Tensor, idxs: torch.Tensor) -> torch.Tensor:
    """TP vocab-parallel greedy combine: vals / idxs [ranks, S] (every rank's best value and global token
    id) -> [S] int32 id of the largest value, the lowest id on ties (csrc/sampling.hip)."""
    if _ref(vals):
        return ref.argmax_combine(vals, idxs)
    lib = require()
    t, S = vals.shape
    out = torch.empty(S, dtype=torch.int32, device=vals.device)
    vals, idxs = vals.float().contiguous(), idxs.to(torch.int32).contiguous()
    check(lib.ka_argmax_combine(_p(out), _p(vals), _p(idxs), S, t, _stream()), "argmax_combine")
    return out


def decode_persistent(h0: torch.Tensor, layer_ptrs: torch.Tensor, L: int, hq: int, hkv: int, I: int, eps: float,
                      scale: float, k_cache: torch.Tensor, v_cache: torch.Tensor, positions: torch.Tensor,
                      slot_mapping: torch.Tensor, block_table: torch.Tensor, ctx_lens: torch.Tensor,
                      cos_sin: torch.Tensor, ws: torch.Tensor, stamps: Optional[torch.Tensor] = None,
                      tp=None) -> torch.Tensor:
    """Every decoder layer of a decode step of B = 1 or 2 sequences in one persistent launch
    (csrc/decode_persistent.hip): h0 [B, H] bf16 embeddings -> the residual streams after the last
    layer [B, H] bf16.  layer_ptrs: int64 [L, 6] device pointers (wqkv, wo, w13, w2, ln1, ln2); caches
    [L, NB, hkv, ...]; positions / slot_mapping / ctx_lens [>= B]; block_table [>= B, max_blocks]
    (a 1-D table is the single sequence's).  tp: None, or (world, rank, xdata, xflag, xctr) of a tensor-
    parallel group (parallel/custom_allreduce.py OneShotAllReduce.pd_exchange): the row-parallel O /
    down outputs are then all-reduced inside the kernel."""
    lib = require()
    B, H = h0.shape
    out = torch.empty_like(h0)
    bt_stride = block_table.stride(0) if block_table.dim() == 2 else block_table.shape[0]
    world, rank, xdata, xflag, xctr = tp if tp is not None else (0, 0, None, None, None)
    check(lib.ka_decode_persistent_tp(_p(out), _p(h0), _p(layer_ptrs), L, H, hq, hkv, I, float(eps), float(scale),
                                      _p(k_cache), _p(v_cache), k_cache[0].numel(), _p(positions), _p(slot_mapping),
                                      _p(block_table), _p(ctx_lens), _p(cos_sin), _p(ws), _p(stamps), B, bt_stride,
                                      world, rank, xdata, xflag, _p(xctr), _stream()),
          "decode_persistent")
    return out


def decode_persistent_max_b(H: int, hq: int, I: int, gq: int = 4) -> int:
    """Largest batch (0, 1 or 2) csrc/decode_persistent.hip takes for a model (its LDS budget; gq =
    hq / hkv: the GQA-8 attention scratch takes more of it)."""
    return int(require().ka_decode_persistent_max_b2(H, hq, I, gq))


GB_BN = 256   # csrc/gemm_big.hip output tile (weight rows)


def lm_head_argmax(x: torch.Tensor, w: torch.Tensor, mask_bits: Optional[torch.Tensor],
                   mask_idx: Optional[torch.Tensor], vocab_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused LM head + greedy SAFE_DECODE sampling (csrc/gemm_big.hip EPI_ARGMAX): the [M, V] logits
    are never written; each 256-token tile's per-row (max, lowest index) of the bf16-rounded allowed
    logits goes to a small workspace and argmax_finish picks the winner.  Same result as
    `masked_argmax(linear(x, w), ...)` (ties: lowest token id)."""
    if _ref(x):
        return ref.masked_argmax(ref.linear(x, w), mask_bits, mask_idx, vocab_offset)
    lib = require()
    M, K = x.shape
    N = w.shape[0]
    out_idx = torch.empty(M, dtype=torch.int32, device=x.device)
    out_val = torch.empty(M, dtype=torch.float32, device=x.device)
    ws = torch.empty(2 * M * ((N + GB_BN - 1) // GB_BN), dtype=torch.float32, device=x.device)
    words = mask_bits.shape[1] if mask_bits is not None else 0
    check(lib.ka_gemm_big_argmax(_p(out_idx), _p(out_val), _p(x), _p(w), M, N, K, x.stride(0), _p(mask_bits),
                                 _p(mask_idx) if mask_bits is not None else None, words, int(vocab_offset),
                                 _p(ws), _stream()), "gemm_big_argmax")
    return out_idx, out_val


def lm_head_argmax_ok(x: torch.Tensor, w: torch.Tensor, vocab_offset: int = 0) -> bool:
    return (x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.shape[1] % 128 == 0
            and w.shape[0] % 128 == 0 and w.is_contiguous() and vocab_offset % 4 == 0)


# Fused LM head per row count M: filled at engine start by ModelRunner.tune_lm_head (timed against
# the plan's GEMM + masked_argmax on the model's own LM head); row counts not timed (prefill / mixed
# steps sample S rows) use the fused kernel from LM_HEAD_FUSED_MIN_M rows up.
# KA_FUSED_LM_HEAD: auto (default) | 1 (always, where the shape allows) | 0 (never).
LM_HEAD_MODE = os.environ.get("KA_FUSED_LM_HEAD", "auto")
LM_HEAD_FUSED: dict = {}
LM_HEAD_FUSED_MIN_M = 64


def use_fused_lm_head(x: torch.Tensor, w: torch.Tensor, vocab_offset: int = 0) -> bool:
    if _ref(x) or LM_HEAD_MODE == "0" or not lm_head_argmax_ok(x, w, vocab_offset):
        return False
    if LM_HEAD_MODE == "1":
        return True
    M = x.shape[0]
    fused = LM_HEAD_FUSED.get(M)
    return fused if fused is not None else M >= LM_HEAD_FUSED_MIN_M


def moe_topk(router_logits: torch.Tensor, k: int):
    if _ref(router_logits):
        return ref.moe_topk(router_logits, k)
    lib = require()
    T, E = router_logits.shape
    w = torch.empty((T, k), dtype=torch.float32, device=router_logits.device)
    ids = torch.empty((T, k), dtype=torch.int32, device=router_logits.device)
    check(lib.ka_moe_topk(_p(w), _p(ids), _p(router_logits), T, E, k, _stream()), "moe_topk")
    return w, ids


# ---- decode GEMM (K13): hand-written weight-streaming split-K MFMA kernel for M <= 256 ----
SKINNY_MAX_M = 256
SKINNY_TARGET_WGS = int(os.environ.get("KA_SKINNY_WGS", "512"))


def skinny_split(M: int, N: int, K: int, target_wgs: int = 0) -> int:
    target = target_wgs or SKINNY_TARGET_WGS
    tiles = (N + 63) // 64
    split = max(1, min(target // max(tiles, 1), K // 256))
    return split


# (M, N, K) -> ("skinny", split) | ("gm", split, cfg) | ("rows", split, rows per wave) | ("big", 0, 0)
# (csrc/gemm_big.hip) | ("blas", 0);
# filled by ops.autotune at engine start for the decode batch buckets.  PLAN_CHOICES is the set
# `linear` dispatches on (tests and the autotuner check plans against it).
PLAN_CHOICES = ("skinny", "gm", "rows", "big", "blas")
BIG_PLAN_MIN_M = 128   # smallest M the autotuner times csrc/gemm_big.hip at (256 x 256 tiles)
GEMM_PLAN: dict = {}
TILE_MAX_M = 512      # largest M the autotuner plans for (decode buckets and small mixed steps)
_PLAN_MS: dict = {}   # (N, K) -> sorted planned M, rebuilt when GEMM_PLAN changes size
_PLAN_MS_SIZE = [-1]


def plan_for(M: int, N: int, K: int):
    """GEMM_PLAN entry for (M, N, K); a row count no bucket was timed at (a mixed step of, say, 300
    rows) takes the plan of the smallest planned M above it, so it stays on the hand-written kernel
    that bucket measured fastest (every plan's kernels take any M up to their bucket)."""
    plan = GEMM_PLAN.get((M, N, K))
    if plan is not None:
        return plan
    if _PLAN_MS_SIZE[0] != len(GEMM_PLAN):
        _PLAN_MS.clear()
        for (m, n, k) in GEMM_PLAN:
            _PLAN_MS.setdefault((n, k), []).append(m)
        for v in _PLAN_MS.values():
            v.sort()
        _PLAN_MS_SIZE[0] = len(GEMM_PLAN)
    ms = _PLAN_MS.get((N, K))
    if not ms:
        return None
    i = bisect.bisect_left(ms, M)
    if i == len(ms):
        return None
    plan = GEMM_PLAN.get((ms[i], N, K))
    if plan is None:   # an entry replaced by another of the same count: rebuild on the next call
        _PLAN_MS_SIZE[0] = -1
        return None
    if plan[0] == "rows" and not rows_ok(M, K, plan[1]):
        return None
    return plan


def linear(x: torch.Tensor, w: torch.Tensor, split: int = 0, defer_reduce: bool = False,
           bf16_partials: bool = False):
    """y = x @ w.T (w is [out, in]).  M <= TILE_MAX_M (decode buckets, small mixed steps): the kernel
    the per-(M, N, K) plan (GEMM_PLAN, ops/tuned/gemm_plan_mi355x.json or timed at engine start by
    ops.autotune) measured fastest — row GEMV ("rows", csrc/gemm_skinny.hip), split-K weight
    streaming ("skinny"), the LDS-DMA ring kernels ("gm", csrc/gemm_mfma.hip), csrc/gemm_big.hip
    ("big") or hipBLASLt ("blas"); an M no bucket planned takes the next larger bucket's plan, and
    without any plan M <= SKINNY_MAX_M streams through gemm_skinny.  Prefill / mixed steps
    (M > TILE_MAX_M) go to csrc/gemm_big.hip (`linear_big`) under KA_PREFILL_GEMM=big where the shape
    allows, else hipBLASLt via F.linear.
    defer_reduce: when the chosen kernel splits K, return its partials as a `SplitK` for a consumer
    that fuses the reduction instead of running the reduce kernel.
    bf16_partials: with defer_reduce, a gemm_mfma plan stores those partials as bf16
    (half the slab write + read).  Consumers that read bf16 partials (summing them in fp32):
    rmsnorm (O-proj / down, `KA_BF16_PARTIALS`) and the fused decode attention
    decode_attention_rope (QKV, `KA_BF16_QKV_PARTIALS`); RoPE / SiLU need fp32 partials."""
    M, K = x.shape
    N = w.shape[0]
    if _ref(x):
        return ref.linear(x, w)
    if M > TILE_MAX_M and use_big_gemm(x, w):
        return linear_big(x, w)
    if M > TILE_MAX_M or K % 64 != 0 or N % 4 != 0 or not x.is_contiguous():
        return torch.nn.functional.linear(x, w)
    if not split:
        plan = plan_for(M, N, K)
        if plan is None:
            if M > SKINNY_MAX_M:
                return torch.nn.functional.linear(x, w)
        elif plan[0] == "blas":
            return torch.nn.functional.linear(x, w)
        elif plan[0] == "gm":
            return linear_gm(x, w, plan[2], plan[1], defer_reduce, bf16_partials)
        elif plan[0] == "rows":
            return linear_rows(x, w, plan[1], plan[2], defer_reduce)
        elif plan[0] == "big":
            return linear_big(x, w)
        else:
            split = plan[1]
    if M > SKINNY_MAX_M:
        return torch.nn.functional.linear(x, w)
    lib = require()
    split = split or skinny_split(M, N, K)
    kps = ((K // split + 63) // 64) * 64
    split = (K + kps - 1) // kps
    ws = torch.empty((split, M, N), dtype=torch.float32, device=x.device) if split > 1 else None
    if defer_reduce and split > 1:
        check(lib.ka_gemm_skinny(None, _p(x), _p(w), _p(ws), M, N, K, split, _stream()), "gemm_skinny")
        return SplitK(ws, split)
    y = torch.empty((M, N), dtype=x.dtype, device=x.device)
    check(lib.ka_gemm_skinny(_p(y), _p(x), _p(w), _p(ws), M, N, K, split, _stream()), "gemm_skinny")
    return y


# Prefill / mixed-step gate_up with the SwiGLU epilogue (csrc/gemm_big.hip EPI_SWIGLU): the [M, 2I]
# gate_up output never exists and the separate SiLU·mul pass goes away.  Every M > TILE_MAX_M (513+)
# rows (profiles/r3/gemm_big: 565 us vs hipBLASLt 550 us + SiLU·mul at M = 2944, 691 vs 620 + 122
# at M = 4096, Llama-3-8B; the split tail of round 4 takes the short last round of tiles at smaller
# M).  KA_PREFILL_SWIGLU=0 restores hipBLASLt + silu_mul.
PREFILL_SWIGLU = os.environ.get("KA_PREFILL_SWIGLU", "1") == "1"
PREFILL_SWIGLU_MIN_M = int(os.environ.get("KA_PREFILL_SWIGLU_MIN_M", "513"))
# Prefill / mixed-step QKV, O and down projections (M > TILE_MAX_M): KA_PREFILL_GEMM=big runs them all
# on csrc/gemm_big.hip (split tail, 192-wide tiles where they fill the rounds), blas all on hipBLASLt
# (F.linear), auto (default) per shape and row-count bucket from PREFILL_PLAN: ModelRunner.tune_prefill
# times both on the model's own weights at engine start (persisted in the plan file, section prefill)
# and keeps gemm_big where it is within PREFILL_MARGIN of hipBLASLt.
PREFILL_GEMM = os.environ.get("KA_PREFILL_GEMM", "auto")
PREFILL_PLAN: dict = {}          # (M bucket, N, K) -> True: gemm_big
PREFILL_BUCKETS = (1024, 2048, 3072, 4096, 6144, 8192)


def prefill_bucket(M: int) -> int:
    i = bisect.bisect_left(PREFILL_BUCKETS, M)
    return PREFILL_BUCKETS[min(i, len(PREFILL_BUCKETS) - 1)]


def use_big_gemm(x: torch.Tensor, w: torch.Tensor) -> bool:
    if PREFILL_GEMM == "blas" or _ref(x) or x.shape[0] <= TILE_MAX_M or not big_gemm_ok(x, w):
        return False
    if PREFILL_GEMM == "big":
        return True
    return PREFILL_PLAN.get((prefill_bucket(x.shape[0]), w.shape[0], w.shape[1]), False)
GB_EPI_SWIGLU = 3


def swiglu_gemm_ok(x: torch.Tensor, w13: torch.Tensor) -> bool:
    """Shapes csrc/gemm_big.hip's SwiGLU epilogue takes: K % 128, I % 128, 16-B aligned rows."""
    M, K = x.shape
    N = w13.shape[0]
    return (x.stride(1) == 1 and x.stride(0) % 8 == 0 and K % 128 == 0 and N % 256 == 0
            and w13.is_contiguous() and w13.shape[1] == K)


def use_prefill_swiglu(x: torch.Tensor, w13: torch.Tensor) -> bool:
    return (PREFILL_SWIGLU and not _ref(x) and x.shape[0] >= PREFILL_SWIGLU_MIN_M
            and x.shape[0] > TILE_MAX_M and swiglu_gemm_ok(x, w13))


def linear_swiglu(x: torch.Tensor, w13: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) for w13 = [gate; up] ([2I, K]): [M, I] bf16.  GPU: one
    gemm_big launch (256 x 256 tiles whose W rows alternate 16-row gate / up chunks, so each lane
    holds gate and up of the same outputs); CPU: the fp32 reference."""
    if _ref(x):
        return ref.silu_mul(ref.linear(x, w13))
    if not swiglu_gemm_ok(x, w13):
        raise ValueError(f"gemm_big SwiGLU needs K % 128 == 0, 2I % 256 == 0, aligned rows: {tuple(x.shape)} "
                         f"x {tuple(w13.shape)}")
    lib = require()
    M, K = x.shape
    N = w13.shape[0]
    out = torch.empty((M, N // 2), dtype=x.dtype, device=x.device) if out is None else out
    ws = gemm_big_ws(x.device)
    check(lib.ka_gemm_big(_p(out), None, _p(x), _p(w13), M, N, K, x.stride(0), out.stride(0), GB_EPI_SWIGLU, 0,
                          _p(ws), ws.numel() if ws is not None else 0, _stream()), "gemm_big_swiglu")
    return out


# csrc/gemm_big.hip split tail: a zero-filled workspace per device (counters + fp32 slabs; the kernel
# leaves the counters zeroed).  KA_GEMM_BIG_TAIL=0: no split tail.
GEMM_BIG_TAIL = os.environ.get("KA_GEMM_BIG_TAIL", "1") == "1"
_GB_WS: dict = {}


def gemm_big_ws(device) -> Optional[torch.Tensor]:
    if not GEMM_BIG_TAIL:
        return None
    ws = _GB_WS.get(device)
    if ws is None:
        ws = _GB_WS[device] = torch.zeros(int(require().ka_gemm_big_ws_bytes()), dtype=torch.uint8, device=device)
    return ws


def gemm_big_err(device) -> int:
    """The split tail's error word (a slice that waited ~0.1 s for the others; 0 in a correct run),
    cleared by the read.  Synchronises the stream."""
    ws = _GB_WS.get(device)
    return 0 if ws is None else int(require().ka_gemm_big_err(_p(ws), _stream()))


def linear_big(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ w.T through csrc/gemm_big.hip (prefill / mixed-step projections, M > TILE_MAX_M):
    256 x 256 tiles, one workgroup per CU, the partial last round split over K (split tail)."""
    if _ref(x):
        return ref.linear(x, w)
    if not big_gemm_ok(x, w):
        raise ValueError(f"gemm_big needs K % 128 == 0, N % 128 == 0, aligned rows: {tuple(x.shape)} x {tuple(w.shape)}")
    lib = require()
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty((M, N), dtype=x.dtype, device=x.device) if out is None else out
    ws = gemm_big_ws(x.device)
    check(lib.ka_gemm_big(_p(out), None, _p(x), _p(w), M, N, K, x.stride(0), out.stride(0), 0, 0, _p(ws),
                          ws.numel() if ws is not None else 0, _stream()), "gemm_big")
    return out


def big_gemm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    M, K = x.shape
    N = w.shape[0]
    return (x.stride(1) == 1 and x.stride(0) % 8 == 0 and K % 128 == 0 and N % 128 == 0 and w.is_contiguous()
            and w.shape[1] == K and M * x.stride(0) * 2 < 2 ** 31 - 4096 and N * K * 2 < 2 ** 31 - 4096)


# Decode gate_up with the SwiGLU epilogue in the csrc/gemm_mfma.hip ring kernel, per decode bucket
# M -> configuration: filled at engine start by ModelRunner.tune_swiglu where it beats the GEMM plan's
# gate_up + SiLU·mul (profiles/r3/decode_swiglu: 72.9 vs 77.4 us at M = 256, 51.9 vs 58.4 at 128,
# Llama-3-8B).  KA_DECODE_SWIGLU=0 disables it.
DECODE_SWIGLU = os.environ.get("KA_DECODE_SWIGLU", "auto")
DECODE_SWIGLU_CFG: dict = {}
DECODE_SWIGLU_CFGS = (2, 3, 4, 5, 12)
# DECODE_SWIGLU_CFG value for "csrc/gemm_big.hip's SwiGLU epilogue" (ops.linear_swiglu): its 256 x 256
# tiles with one wave per SIMD read a quarter of the ring kernel's LDS bytes per MFMA, which pays from
# M ~ 256 up (the fused LM head's measurement)
DECODE_SWIGLU_BIG = 100


def decode_swiglu_ok(x: torch.Tensor, w13: torch.Tensor) -> bool:
    """Rows the ring kernel's SwiGLU epilogue takes: any M up to TILE_MAX_M (rows past M re-read the
    distinct rows r % M: a clamp to row M - 1 triggered LDS-DMA corruption, profiles/r5/gemm_big_clamp/); below 8 rows ModelRunner.tune_swiglu weighs it against the GEMV path with the activation in
    the down projection's staging (ops.swiglu_linear), down projection included."""
    M, K = x.shape
    return (x.is_contiguous() and w13.is_contiguous() and w13.shape[1] == K and K % 64 == 0
            and w13.shape[0] % 32 == 0 and 1 <= M <= TILE_MAX_M)


def decode_swiglu_cfg(x: torch.Tensor, w13: torch.Tensor) -> int:
    """The gemm_mfma configuration for this decode gate_up + SwiGLU, 0 for the unfused path.  A row
    count no bucket was timed at (a mixed step's pruned last layer, e.g. 282 sequences) takes the
    decision of the smallest timed bucket above it, as ops.plan_for does for the GEMM plan."""
    if DECODE_SWIGLU == "0" or _ref(x):
        return 0
    M = x.shape[0]
    cfg = DECODE_SWIGLU_CFG.get(M)
    if cfg is None:
        ms = sorted(DECODE_SWIGLU_CFG)
        i = bisect.bisect_left(ms, M)
        cfg = DECODE_SWIGLU_CFG[ms[i]] if i < len(ms) else 0
    if cfg == DECODE_SWIGLU_BIG and not swiglu_gemm_ok(x, w13):
        return 0
    return cfg if cfg and decode_swiglu_ok(x, w13) else 0


# Row-streaming GEMV (csrc/gemm_skinny.hip gemv_rows_kernel) for M <= 4: each wave streams a
# contiguous block of weight rows 1 KB per load, non-temporal (profiles/r3/gemv_rows: Llama-3-8B
# batch 1 gate_up 46.8 -> 38.6 us, down with SwiGLU staging 24.1 -> 21.8, QKV 13.3 -> 12.1, LM head
# 201 -> 164).  Planned per shape by ops.autotune ("rows", split, rows per wave).
ROWS_MAX_M = 16                 # csrc/gemm_skinny.hip stages up to 16 X rows per workgroup
ROWS_NT = 4                     # ka_gemv_rows flag: non-temporal weight loads
ROWS_SWIGLU = os.environ.get("KA_GEMV_ROWS_SWIGLU", "1") == "1"
ROWS_SWIGLU_SPLIT, ROWS_SWIGLU_RW = 4, 4


def rows_mr(M: int) -> int:
    return 1 if M == 1 else 2 if M == 2 else 4 if M <= 4 else 8 if M <= 8 else 16


def rows_ok(M: int, K: int, split: int) -> bool:
    return (M <= ROWS_MAX_M and split >= 1 and K % (512 * split) == 0
            and rows_mr(M) * (K // split) * 2 <= 65536)


def linear_rows(x: torch.Tensor, w: torch.Tensor, split: int, rw: int, defer_reduce: bool = False):
    """y = x @ w.T for M <= 16 through the row-streaming GEMV (`rw` weight rows per wave, K split
    `split` ways); split > 1 with defer_reduce returns the fp32 partials as a `SplitK`."""
    M, K = x.shape
    N = w.shape[0]
    if _ref(x):
        return ref.linear(x, w)
    if not rows_ok(M, K, split) or not x.is_contiguous():
        raise ValueError(f"gemv_rows needs M <= 16, K % (512*split) == 0: M={M} K={K} split={split}")
    lib = require()
    ws = torch.empty((split, M, N), dtype=torch.float32, device=x.device) if split > 1 else None
    if defer_reduce and split > 1:
        check(lib.ka_gemv_rows(None, _p(x), _p(w), _p(ws), M, N, K, split, rw, ROWS_NT, _stream()), "gemv_rows")
        return SplitK(ws, split)
    y = torch.empty((M, N), dtype=x.dtype, device=x.device)
    check(lib.ka_gemv_rows(_p(y), _p(x), _p(w), _p(ws), M, N, K, split, rw, ROWS_NT, _stream()), "gemv_rows")
    return y


GEMV_SWIGLU_MAX_M = 4   # csrc/gemm_skinny.hip GEMV_SWIGLU_MAX_M


def swiglu_linear(gu, w: torch.Tensor, defer_reduce: bool = False, bf16_partials: bool = False):
    """y = (silu(gu[:, :I]) * gu[:, I:]) @ w.T — the MLP down projection fed directly by the fused
    gate_up output (a bf16 tensor; a `SplitK` goes through silu_mul's fused reduce).

    * M <= 4 (batch-1..4 decode, the model's path): the GEMV computes the activation while staging
      its X slice once per workgroup (ka_gemv_swiglu, bit-identical to SiLU·mul + GEMV): one kernel
      and one launch boundary less per layer;
    * otherwise SiLU·mul then `linear` (an activation computed inside a tiled GEMM's X staging
      measured 138 us vs 47 + 6 us unfused at M=256, Llama-3-8B down: every one of the N/BN
      column tiles re-stages X and so recomputes it)."""
    if isinstance(gu, SplitK) or _ref(gu) or not gu.is_contiguous():
        return linear(silu_mul(gu), w, defer_reduce=defer_reduce, bf16_partials=bf16_partials)
    M, I2 = gu.shape
    I = I2 // 2
    N = w.shape[0]
    if ROWS_SWIGLU and rows_ok(M, I, ROWS_SWIGLU_SPLIT):
        lib = require()
        sp = ROWS_SWIGLU_SPLIT
        ws = torch.empty((sp, M, N), dtype=torch.float32, device=gu.device)
        if defer_reduce:
            check(lib.ka_gemv_rows(None, _p(gu), _p(w), _p(ws), M, N, I, sp, ROWS_SWIGLU_RW, ROWS_NT | 1, _stream()),
                  "gemv_rows_swiglu")
            return SplitK(ws, sp)
        y = torch.empty((M, N), dtype=gu.dtype, device=gu.device)
        check(lib.ka_gemv_rows(_p(y), _p(gu), _p(w), _p(ws), M, N, I, sp, ROWS_SWIGLU_RW, ROWS_NT | 1, _stream()),
              "gemv_rows_swiglu")
        return y
    if M <= GEMV_SWIGLU_MAX_M and I % 64 == 0 and N % 4 == 0:
        lib = require()
        split = skinny_split(M, N, I, 256)
        kps = ((I // split + 63) // 64) * 64
        split = (I + kps - 1) // kps
        if M * kps * 2 <= 65536:
            ws = torch.empty((split, M, N), dtype=torch.float32, device=gu.device) if split > 1 else None
            if defer_reduce and split > 1:
                check(lib.ka_gemv_swiglu(None, _p(gu), _p(w), _p(ws), M, N, I, split, _stream()), "gemv_swiglu")
                return SplitK(ws, split)
            y = torch.empty((M, N), dtype=gu.dtype, device=gu.device)
            check(lib.ka_gemv_swiglu(_p(y), _p(gu), _p(w), _p(ws), M, N, I, split, _stream()), "gemv_swiglu")
            return y
    return linear(silu_mul(gu), w, defer_reduce=defer_reduce, bf16_partials=bf16_partials)


# csrc/gemm_mfma.hip configurations (LDS-DMA staged MFMA GEMM family; ka_gm_bn / ka_gm_bm give the
# tile): 2-5, 12 ring kernels, 19 the 2-phase 256 x 256 ping-pong kernel
GM_CFGS = (2, 3, 4, 5, 12, 19)
GM_EPI_BF16, GM_EPI_P32, GM_EPI_P16, GM_EPI_SWIGLU = 0, 1, 2, 3
# grouped (MoE prefill) configuration: the 256 x 256 ping-pong kernel (profiles/r2/bench_moe_prefill.txt)
MOE_GROUPED_CFG = int(os.environ.get("KA_MOE_GROUPED_CFG", "19"))


def gm_shape(cfg: int):
    """(BN, BM) of a gemm_mfma configuration."""
    lib = require()
    return lib.ka_gm_bn(cfg), lib.ka_gm_bm(cfg)


def linear_gm(x: torch.Tensor, w: torch.Tensor, cfg: int, split: int = 1, defer_reduce: bool = False,
              bf16_partials: bool = False):
    """y = x @ w.T through csrc/gemm_mfma.hip (configuration `cfg`, split-K `split`; K must be a
    multiple of 64 * split).  split > 1 with defer_reduce returns the fp32 (or bf16) partial slabs
    as a `SplitK` for a fused consumer; without it the slabs are reduced by splitk_reduce."""
    M, K = x.shape
    N = w.shape[0]
    if K % (64 * split) or N % 16 or x.stride(0) % 8:
        raise ValueError(f"gemm_mfma needs K % (64*split) == 0, N % 16 == 0: N={N} K={K} split={split}")
    lib = require()
    st = _stream()
    if split == 1:
        y = torch.empty((M, N), dtype=x.dtype, device=x.device)
        check(lib.ka_gemm_mfma(_p(y), None, _p(x), _p(w), M, N, K, x.stride(0), N, 1, cfg, GM_EPI_BF16, 0, st),
              "gemm_mfma")
        return y
    pb = defer_reduce and bf16_partials
    ws = torch.empty((split, M, N), dtype=torch.bfloat16 if pb else torch.float32, device=x.device)
    if defer_reduce:
        check(lib.ka_gemm_mfma(None, _p(ws), _p(x), _p(w), M, N, K, x.stride(0), N, split, cfg,
                               GM_EPI_P16 if pb else GM_EPI_P32, 0, st), "gemm_mfma")
        return SplitK(ws, split)
    y = torch.empty((M, N), dtype=x.dtype, device=x.device)
    check(lib.ka_gemm_mfma(_p(y), _p(ws), _p(x), _p(w), M, N, K, x.stride(0), N, split, cfg, GM_EPI_P32, 0, st),
          "gemm_mfma")
    return y


def linear_gm_swiglu(x: torch.Tensor, w13: torch.Tensor, cfg: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) for w13 = [gate; up] through csrc/gemm_mfma.hip configuration
    `cfg` with the SwiGLU epilogue (the DMA sources gather gate / up in 16-row chunks): [M, I] bf16.
    cfg DECODE_SWIGLU_BIG: csrc/gemm_big.hip's SwiGLU epilogue instead (ops.linear_swiglu)."""
    M, K = x.shape
    I = w13.shape[0] // 2
    if _ref(x):
        return ref.silu_mul(ref.linear(x, w13))
    if cfg == DECODE_SWIGLU_BIG:
        return linear_swiglu(x, w13, out)
    lib = require()
    out = torch.empty((M, I), dtype=x.dtype, device=x.device) if out is None else out
    check(lib.ka_gemm_mfma_swiglu(_p(out), _p(x), _p(w13), M, I, K, x.stride(0), out.stride(0), int(cfg), _stream()),
          "gemm_mfma_swiglu")
    return out


def linear_grouped(x: torch.Tensor, w: torch.Tensor, counts: torch.Tensor, lists: torch.Tensor, rows: int,
                   src_div: int = 1, cfg: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Y[r] = x[r // src_div] @ w[e].T for every row r listed for group e (lists [G, stride], counts
    [G], device-side: no host read) through csrc/gemm_mfma.hip's grouped ring kernel.  Y is
    [rows, N]; rows listed for no group are left unwritten."""
    G, N, K = w.shape
    cfg = MOE_GROUPED_CFG if cfg is None else cfg
    if K % 64 or N % 16 or x.stride(0) % 8:
        raise ValueError(f"grouped gemm_mfma needs K % 64 == 0 and N % 16 == 0: N={N} K={K}")
    out = torch.empty((rows, N), dtype=x.dtype, device=x.device) if out is None else out
    lib = require()
    check(lib.ka_gemm_mfma_grouped(_p(out), None, _p(x), _p(w), _p(counts), _p(lists), lists.shape[1], src_div, G,
                                   rows, N, K, x.stride(0), N, 1, cfg, GM_EPI_BF16, _stream()), "gemm_mfma_grouped")
    return out


# ---- Mixtral MoE (K12): device-side routing lists + grouped weight-streaming GEMM + combine ----
def moe_split(rows: int, n_experts_local: int, N: int, K: int, target_wgs: int = 0) -> int:
    """Split-K factor for the grouped expert GEMM: at decode row counts only min(El, rows) experts
    are active, so (N / 64 column tiles) x (active experts) workgroups can leave most CUs idle
    (w2 at batch 1: 128 on 256 CUs).  Split K until ~target_wgs workgroups stream weights; the
    default target per row count is the best of a 1024/2048/4096/8192 sweep at the Mixtral-8x7B
    geometry (profiles/moe_split_sweep.txt: T=1 block 304 -> 161 us)."""
    if target_wgs <= 0:
        target_wgs = 4096 if rows <= 2 else 2048 if rows >= 256 else 1024
    active = max(1, min(n_experts_local, rows))
    wgs = (N + 63) // 64 * active * ((rows + 127) // 128)
    split = 1
    while split < 16 and wgs * split * 2 <= target_wgs and K % (64 * split * 2) == 0:
        split *= 2
    return split


def moe_experts(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                topk_ids: torch.Tensor, e0: int) -> torch.Tensor:
    """sum_j topk_w[t,j] * FFN_{e(t,j)}(x[t]) over this rank's experts [e0, e0 + El); [T, H] bf16."""
    lib = require()
    T, H = x.shape
    k = topk_ids.shape[1]
    El, two_i, _ = w13.shape
    R = T * k
    dev = x.device
    counts = torch.empty(El, dtype=torch.int32, device=dev)
    lists = torch.empty((El, R), dtype=torch.int32, device=dev)
    st = _stream()
    check(lib.ka_moe_align(_p(counts), _p(lists), _p(topk_ids), R, e0, El, st), "moe_align")
    s1 = moe_split(R, El, two_i, H)
    if s1 > 1:   # fp32 partials; silu_mul_splitk reduces them
        p1 = torch.empty((s1, R, two_i), dtype=torch.float32, device=dev)
        check(lib.ka_moe_gemm(None, _p(x), _p(w13), _p(counts), _p(lists), R, El, two_i, H, k, R, s1, _p(p1), st),
              "moe_gemm1")
        act = silu_mul(SplitK(p1, s1))
    else:
        y1 = torch.empty((R, two_i), dtype=x.dtype, device=dev)
        check(lib.ka_moe_gemm(_p(y1), _p(x), _p(w13), _p(counts), _p(lists), R, El, two_i, H, k, R, 1, None, st),
              "moe_gemm1")
        act = silu_mul(y1)
    I = two_i // 2
    s2 = moe_split(R, El, H, I)
    out = torch.empty((T, H), dtype=x.dtype, device=dev)
    if s2 > 1:
        p2 = torch.empty((s2, R, H), dtype=torch.float32, device=dev)
        check(lib.ka_moe_gemm(None, _p(act), _p(w2), _p(counts), _p(lists), R, El, H, I, 1, R, s2, _p(p2), st),
              "moe_gemm2")
        check(lib.ka_moe_combine(_p(out), None, _p(p2), s2, _p(topk_w), _p(topk_ids), T, k, H, e0, El, st),
              "moe_combine")
    else:
        y2 = torch.empty((R, H), dtype=x.dtype, device=dev)
        check(lib.ka_moe_gemm(_p(y2), _p(act), _p(w2), _p(counts), _p(lists), R, El, H, I, 1, R, 1, None, st),
              "moe_gemm2")
        check(lib.ka_moe_combine(_p(out), _p(y2), None, 1, _p(topk_w), _p(topk_ids), T, k, H, e0, El, st),
              "moe_combine")
    return out


# MoE prefill expert GEMMs (KA_MOE_PREFILL): "big" = expert-sorted rows through csrc/gemm_big.hip's
# grouped mode (256 x 256 tiles, SwiGLU epilogue), "gm" = the grouped gemm_mfma ring kernel over
# gathered rows (MOE_GROUPED_CFG), "auto" (default) = big from MOE_BIG_MIN_ROWS routed rows up, gm
# below.  Mixtral block, profiles/r5/gemm_big_clamp/replan/moe_prefill.log: T = 1024 (2048 rows) gm
# 1.12 vs big 1.31 ms; T = 4096 big 3.02 vs gm 3.16; T = 8192 big 5.24 vs gm 5.88 (sorted hipBLASLt
# 1.51 / 3.40 / 5.66).
MOE_PREFILL = os.environ.get("KA_MOE_PREFILL", "auto")
MOE_BIG_MIN_ROWS = int(os.environ.get("KA_MOE_BIG_MIN_ROWS", "6144"))


def moe_big_ok(H: int, I: int, El: int, R: int = 0) -> bool:
    """Shapes the grouped gemm_big path takes (ka_gemm_big_grouped / ka_moe_sort requirements).  R: the
    routed rows (tokens x top-k); the [R, max(H, I)] activations must fit a 32-bit buffer descriptor
    (Mixtral's [R, 14336] act passes 2^31 bytes at R ~ 75k), else the gm path takes the block."""
    return (H % 256 == 0 and I % 128 == 0 and El <= 64
            and El * 2 * I * H * 2 < 2 ** 31 - 4096 and El * H * I * 2 < 2 ** 31 - 4096
            and R * max(H, I) * 2 < 2 ** 31 - 4096)


def moe_experts_grouped(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                        topk_ids: torch.Tensor, e0: int) -> torch.Tensor:
    """Prefill-sized MoE block, device-resident end to end (no host sync): routing lists
    (moe_align), then either (KA_MOE_PREFILL=big, or auto at >= MOE_BIG_MIN_ROWS rows) the routed rows sorted by expert
    (moe_sort) -> grouped gemm_big gate_up with the SwiGLU epilogue -> grouped gemm_big down
    scattering each row back to its slot, or (gm) the grouped ring-kernel gate_up over gathered token
    rows -> SiLU·mul -> grouped down; then the weighted combine.  Same contract as `moe_experts`."""
    lib = require()
    T, H = x.shape
    k = topk_ids.shape[1]
    El, two_i, _ = w13.shape
    R = T * k
    st = _stream()
    counts = torch.empty(El, dtype=torch.int32, device=x.device)
    lists = torch.empty((El, R), dtype=torch.int32, device=x.device)
    check(lib.ka_moe_align(_p(counts), _p(lists), _p(topk_ids), R, e0, El, st), "moe_align")
    I = two_i // 2
    big = MOE_PREFILL == "big" or (MOE_PREFILL == "auto" and R >= MOE_BIG_MIN_ROWS)
    if big and moe_big_ok(H, I, El, R) and x.is_contiguous():
        chunks = (R + 255) // 256 + El
        xs = torch.empty((R, H), dtype=x.dtype, device=x.device)
        slot = torch.empty(R, dtype=torch.int32, device=x.device)
        tab = torch.empty(chunks * 4, dtype=torch.int32, device=x.device)
        check(lib.ka_moe_sort(_p(xs), _p(slot), _p(tab), _p(x), _p(counts), _p(lists), R, k, H, El, chunks, st),
              "moe_sort")
        act = torch.empty((R, I), dtype=x.dtype, device=x.device)   # expert-sorted rows
        check(lib.ka_gemm_big_grouped(_p(act), _p(xs), _p(w13), _p(tab), chunks, None, R, two_i, H, H, I, El,
                                      3, st), "gemm_big_grouped(w13)")
        y2 = torch.empty((R, H), dtype=x.dtype, device=x.device)    # slot rows (others never read)
        check(lib.ka_gemm_big_grouped(_p(y2), _p(act), _p(w2), _p(tab), chunks, _p(slot), R, H, I, I, H, El,
                                      0, st), "gemm_big_grouped(w2)")
        out = torch.empty((T, H), dtype=x.dtype, device=x.device)
        check(lib.ka_moe_combine(_p(out), _p(y2), None, 1, _p(topk_w), _p(topk_ids), T, k, H, e0, El, st),
              "moe_combine")
        return out
    y1 = linear_grouped(x, w13, counts, lists, R, src_div=k)          # slot rows of local experts
    y2 = linear_grouped(silu_mul(y1), w2, counts, lists, R)          # other rows: never read
    out = torch.empty((T, H), dtype=x.dtype, device=x.device)
    check(lib.ka_moe_combine(_p(out), _p(y2), None, 1, _p(topk_w), _p(topk_ids), T, k, H, e0, El, st),
          "moe_combine")
    return out


rope_cos_sin = ref.rope_cos_sin
