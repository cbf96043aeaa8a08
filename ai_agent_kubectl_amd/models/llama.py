"""Llama-3 decoder (8B / 70B) and Mixtral-8x7B (MoE MLP) over the engine ops.

This is what replaces the remote `ChatOpenAI` call (`/root/reference/app.py:117,184`): the
forward pass of SURVEY.md §3.6 —
  K1 embed -> per layer: K2 norm, K3 QKV GEMM, K4 RoPE+KV append, K5/K6 paged attention,
  K7 O-proj (+A1 all-reduce), K2 norm, K8 gate_up GEMM + SiLU*mul (or K11/K12 MoE), K9 down
  (+A2 all-reduce) -> final norm -> K10 vocab-parallel LM head -> masked greedy argmax (+A3).

Tensor parallelism is Megatron-style (column-parallel QKV / gate_up, row-parallel O / down,
vocab-parallel LM head); Mixtral experts are sharded over the same group (EP = TP group) and
combined by the all-reduce that follows the MoE block (decode) or by the all-to-all dispatch /
combine of `moe_alltoall` (eager prefill, models/moe.py).  Every op is shape-static for a given
token count, so decode steps can be captured into hipGraphs by the runner.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..parallel.comm import LocalComm
from .config import ModelConfig
from .moe import moe_forward


def persistent_default() -> bool:
    """KA_PERSISTENT_DECODE: 0 off, 1 on, auto (default) on unless the GPU is shared with another
    engine (KA_GPU_MEM_SHARE < 1): co-residency of the persistent grid is not guaranteed there."""
    mode = os.environ.get("KA_PERSISTENT_DECODE", "auto")
    if mode in ("0", "1"):
        return mode == "1"
    return float(os.environ.get("KA_GPU_MEM_SHARE", "1")) >= 1.0


@dataclass
class AttnMeta:
    """Per-step metadata (device int32 tensors unless noted)."""
    positions: torch.Tensor            # [T]
    slot_mapping: torch.Tensor         # [T]   -1 = padding token
    block_tables: torch.Tensor         # [S, max_blocks]
    ctx_lens: torch.Tensor             # [S]   KV length after this step
    logits_indices: torch.Tensor       # [S]   int64, row of each sequence's last token in [T]
    is_decode: bool                    # all sequences contribute exactly one token
    q_starts: Optional[torch.Tensor] = None   # [S+1] (prefill)
    max_q_len: int = 1
    num_decode: int = 0                # mixed step: the first num_decode sequences are 1-token decode rows
    num_tokens: int = 0                # real tokens when the step is padded (rows beyond are padding)
    shared_blocks: Optional[torch.Tensor] = None   # decode: [1] leading blocks shared by every row (cascade)


class LlamaModel:
    def __init__(self, cfg: ModelConfig, weights: Dict[str, torch.Tensor], comm=None, tp_rank: int = 0,
                 tp_size: int = 1, ep_rank: int = 0, ep_size: int = 1):
        self.cfg = cfg
        self.W = weights
        self.comm = comm or LocalComm()
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self._local_comm = isinstance(self.comm, LocalComm)   # no all-reduce between GEMM and norm
        self.ep_rank, self.ep_size = ep_rank, ep_size
        self.hq = cfg.num_heads // tp_size
        self.hkv = cfg.num_kv_heads // tp_size
        self.D = cfg.head_dim
        self.scale = cfg.head_dim ** -0.5
        self.vocab_local = weights["lm_head"].shape[0]
        self.vocab_offset = tp_rank * self.vocab_local
        dev = weights["embed"].device
        self.device = dev
        self.cos_sin = ops.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta, device=dev)
        self.fuse_decode_rope = os.environ.get("KA_FUSE_DECODE_ROPE", "1") == "1"
        # split-K partials of the norm-feeding projections (o_proj, down) stored as bf16: half the
        # slab traffic; the fused reduce + RMSNorm still accumulates them in fp32
        self.bf16_partials = os.environ.get("KA_BF16_PARTIALS", "1") == "1"
        # the QKV projection's split-K partials for the fused decode attention (its prologue sums
        # them in fp32): a separate switch so the two can be A/B'd independently
        self.bf16_qkv_partials = os.environ.get("KA_BF16_QKV_PARTIALS", "1") == "1"
        self.layers = [self._layer(i) for i in range(cfg.num_layers)]
        # this rank's MLP width (the TP shard of the intermediate size)
        w13 = self.layers[0].get("w13") if self.layers else None
        self.i_local = w13.shape[-2] // 2 if w13 is not None else cfg.intermediate // tp_size
        # prefill / mixed steps: the last layer's rows other than each sequence's last token feed
        # nothing (only the last rows reach the final norm and the LM head), so after that layer's
        # QKV + RoPE + KV append (which every row needs for later steps) it continues on the S
        # last-token rows only: attention as S one-query rows, O-proj, norm and MLP on S rows
        self.prune_last_layer = os.environ.get("KA_PRUNE_LAST_LAYER", "1") == "1"
        # eager steps only: record `mark_event` when layer `mark_layer` starts (-1: never)
        self.mark_layer = -1
        self.mark_event = None
        # small-batch decode: while attention, O-proj and the second norm run (HBM mostly idle), a
        # side stream reads the first KA_DECODE_PREFETCH_MB of this layer's gate_up weights into the
        # Infinity Cache so the gate_up GEMV starts on cache hits (fork / join inside the captured
        # graph).  0 (default): off.
        self.prefetch_bytes = int(float(os.environ.get("KA_DECODE_PREFETCH_MB", "0")) * (1 << 20))
        self.prefetch_max_b = int(os.environ.get("KA_DECODE_PREFETCH_MAX_B", "4"))
        self.prefetch_blocks = int(os.environ.get("KA_DECODE_PREFETCH_BLOCKS", "64"))
        self._side = None
        # batch-1 decode: every layer in ONE persistent launch (csrc/decode_persistent.hip) instead of
        # ~7 kernels per layer (2.85 vs 3.44 ms/step for Llama-3-8B, profiles/r4/persistent_decode/,
        # profiles/r4/zero_cijk_decode/), wherever the geometry allows.  Its grid barriers need every
        # workgroup resident, which only holds when this engine owns the GPU: KA_PERSISTENT_DECODE=auto
        # (default) turns it off when several replicas / ranks share the device (KA_GPU_MEM_SHARE < 1,
        # parallel/dp.py), 1 forces it on, 0 keeps the kernel chain.
        self.persistent = persistent_default()
        self._pd = None   # (layer pointer table, workspace)
        # decode batches the persistent kernel serves (1 or 2: B = 2 streams the weights once for both
        # sequences' rows)
        self.persistent_max_b = int(os.environ.get("KA_PERSISTENT_MAX_B", "2"))
        self._pd_max_b = None
        self.persistent_stamps = None   # diagnostics: int64 [CUs, L, 16] phase timestamps (scripts/)

    def _layer(self, i):
        p = f"layers.{i}."
        return {k: self.W[p + k] for k in ("wqkv", "wo", "ln1", "ln2", "w13", "w2", "router") if p + k in self.W}

    # ------------------------------------------------------------------------------------------
    def forward(self, input_ids: torch.Tensor, meta: AttnMeta, k_cache: torch.Tensor,
                v_cache: torch.Tensor) -> torch.Tensor:
        """Returns the final-normed hidden state of each sequence's last token: [S, H]."""
        cfg = self.cfg
        eps = cfg.norm_eps
        h = ops.embedding(input_ids, self.W["embed"])
        if ops.reference_fp32():   # test-only fp32 truth: activations / residual in fp32 (ops.force_reference)
            h = h.float()
        if meta.is_decode and not ops._ref(h) and self.persistent_ok(input_ids.shape[0]):
            return self._forward_persistent(h, meta, k_cache, v_cache)
        residual = None
        pending = False   # h holds this rank's partial of a row-parallel output (TP all-reduce due)
        T = input_ids.shape[0]
        mark = self.mark_layer
        last_li = len(self.layers) - 1
        pruned = False   # rows cut down to the sequences' last tokens (last layer, prefill / mixed)
        for li, L in enumerate(self.layers):
            if li == mark and input_ids.is_cuda:   # progress marker (engine lookahead timing)
                self.mark_event = torch.cuda.Event()
                self.mark_event.record()
            if residual is None:
                residual = h
                x = ops.rmsnorm(h, L["ln1"], eps)
            else:
                x = self._reduce_norm(h, L["ln1"], eps, residual, pending)
            # column-parallel projections: no all-reduce before their consumer, so a split-K plan
            # hands its partials to the RoPE / attention / SiLU kernels, which reduce them on the fly
            fused = meta.is_decode and self.fuse_decode_rope
            # the fused decode attention reduces bf16 QKV partials too (KA_BF16_QKV_PARTIALS);
            # rope_kv_write needs fp32 ones
            qkv = ops.linear(x, L["wqkv"], defer_reduce=True, bf16_partials=fused and self.bf16_qkv_partials)
            side = self._fork_prefetch(L, T) if meta.is_decode else None
            if fused:
                # RoPE + KV append + attention in one kernel (the rotated q never goes to HBM)
                a = ops.decode_attention_rope(qkv, meta.positions, self.cos_sin, meta.slot_mapping, k_cache[li],
                                              v_cache[li], meta.block_tables, meta.ctx_lens, self.hq, self.hkv,
                                              self.D, self.scale, shared_blocks=meta.shared_blocks)
            else:
                q = ops.rope_kv_write(qkv, meta.positions, self.cos_sin, meta.slot_mapping, k_cache[li],
                                      v_cache[li], self.hq, self.hkv, self.D)
                if li == last_li and not meta.is_decode and self.prune_last_layer:
                    # every sequence's last token as a one-query decode row over its whole context
                    # (this step's keys were just appended); the residual stream follows those rows
                    idx = meta.logits_indices
                    a = ops.attention_decode(q.index_select(0, idx), k_cache[li], v_cache[li], meta.block_tables,
                                             meta.ctx_lens, self.scale)
                    residual = residual.index_select(0, idx)
                    pruned = True
                else:
                    a = self._attention(q, meta, k_cache[li], v_cache[li])
            if 0 < meta.num_tokens < T and not meta.is_decode and not pruned:
                a[meta.num_tokens:].zero_()   # padding rows: no sequence's attention writes them
            # the projections feeding a norm leave their split-K partials to the consumer
            # (ops.SplitK): TP = 1 the fused reduce + residual + RMSNorm kernel; a TP rank's decode
            # step the one-shot all-reduce + RMSNorm kernel, which reduces the slabs while staging its
            # contribution (comm.all_reduce_rmsnorm, A1 / A2; comm.splitk_norm)
            fuse = self._local_comm or (meta.is_decode and getattr(self.comm, "splitk_norm", False))
            h = ops.linear(a.reshape(a.shape[0], self.hq * self.D), L["wo"], defer_reduce=fuse,
                           bf16_partials=self.bf16_partials)
            x = self._reduce_norm(h, L["ln2"], eps, residual, True)
            if side is not None:   # join: the gate_up GEMV reads what the side stream prefetched
                torch.cuda.current_stream(self.device).wait_stream(side)
            combined = False
            if cfg.is_moe:
                h, combined = moe_forward(x, L, cfg, self.ep_rank, self.ep_size, meta.is_decode, self.comm)
            elif ops.use_prefill_swiglu(x, L["w13"]):
                # prefill / mixed steps: gate_up with the SwiGLU epilogue (no [T, 2I] intermediate)
                h = ops.linear(ops.linear_swiglu(x, L["w13"]), L["w2"], defer_reduce=fuse,
                               bf16_partials=self.bf16_partials)
            elif sw := ops.decode_swiglu_cfg(x, L["w13"]):
                # decode buckets where the ring kernel's SwiGLU epilogue won (ModelRunner.tune_swiglu)
                h = ops.linear(ops.linear_gm_swiglu(x, L["w13"], sw), L["w2"], defer_reduce=fuse,
                               bf16_partials=self.bf16_partials)
            else:
                # batch <= 4: SiLU·mul computed inside the down GEMV's X staging (ops.swiglu_linear)
                h = ops.swiglu_linear(ops.linear(x, L["w13"], defer_reduce=True), L["w2"], defer_reduce=fuse,
                                      bf16_partials=self.bf16_partials)
            pending = not combined   # A2: reduced together with the next norm
        if meta.is_decode:   # every row is its sequence's last token (logits_indices = arange)
            return self._reduce_norm(h, self.W["norm"], eps, residual, pending)
        if pending and not self._local_comm:
            self.comm.all_reduce(h)
        if pruned:   # h and residual already hold only the sequences' last rows
            return ops.rmsnorm(h, self.W["norm"], eps, residual=residual)
        if isinstance(h, ops.SplitK):
            x = ops.rmsnorm(h, self.W["norm"], eps, residual=residual)
            return x.index_select(0, meta.logits_indices)
        # prefill: only the sequences' last rows are sampled, so only they are normed
        idx = meta.logits_indices
        return ops.rmsnorm(h.index_select(0, idx), self.W["norm"], eps, residual=residual.index_select(0, idx))

    def persistent_ok(self, B: int = 1) -> bool:
        """The persistent all-layers kernel takes a decode step of B sequences: B <= KA_PERSISTENT_MAX_B
        (default 2) and within the kernel's LDS budget for this geometry (ops.decode_persistent_max_b)."""
        cfg = self.cfg
        # TP = 1 (LocalComm), a virtual rank (parallel/comm.py VirtualRankComm, whose all-reduces are
        # no-ops by definition), or a real TP group with the one-shot IPC buffers, whose O / down
        # all-reduces the kernel then runs itself (KA_PERSISTENT_TP=1: opt-in until an 8-GPU node has
        # measured it; the 2-rank-on-one-GPU test covers the protocol)
        comm_ok = (self._local_comm or getattr(self.comm, "persistent_no_reduce", False)
                   or self._tp_exchange() is not None)
        I = self.i_local
        if not (self.persistent and self.device.type == "cuda" and comm_ok and not cfg.is_moe
                and self.D == 128 and self.hq % self.hkv == 0 and self.hq // self.hkv <= 8
                and cfg.hidden % 512 == 0 and I % 512 == 0 and (self.hq * self.D) % 512 == 0
                and cfg.hidden <= 16384 and 1 <= B <= self.persistent_max_b):
            return False
        if self._pd_max_b is None:
            self._pd_max_b = ops.decode_persistent_max_b(cfg.hidden, self.hq, I, self.hq // self.hkv)
        return B <= self._pd_max_b

    def _tp_exchange(self):
        """The in-kernel all-reduce's buffers of a real TP group (None: TP = 1, virtual, or not enabled)."""
        car = getattr(self.comm, "custom_ar", None)
        if car is None or self.tp_size <= 1 or os.environ.get("KA_PERSISTENT_TP", "0") != "1":
            return None
        return car.pd_exchange()

    def _forward_persistent(self, h0, meta: AttnMeta, k_cache, v_cache) -> torch.Tensor:
        """Batch-1 / 2 decode through the persistent all-layers kernel; returns the final-normed hidden
        states [B, H] like `forward`."""
        if self._pd is None:
            ptrs = [[L[k].data_ptr() for k in ("wqkv", "wo", "w13", "w2", "ln1", "ln2")] for L in self.layers]
            table = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
            lib = ops._hip.require()
            ws = torch.zeros(int(lib.ka_decode_persistent_ws(self.cfg.hidden, self.hq, self.hkv, self.i_local)),
                             dtype=torch.uint8, device=self.device)
            self._pd = (table, ws)
        table, ws = self._pd
        assert k_cache.shape[3] == 16, "persistent decode needs KV block 16"   # [L, NB, hkv, 16, 128]
        hout = ops.decode_persistent(h0, table, len(self.layers), self.hq, self.hkv, self.i_local,
                                     self.cfg.norm_eps, self.scale, k_cache, v_cache, meta.positions,
                                     meta.slot_mapping, meta.block_tables, meta.ctx_lens, self.cos_sin, ws,
                                     self.persistent_stamps, tp=self._tp_exchange())
        return ops.rmsnorm(hout, self.W["norm"], self.cfg.norm_eps)

    def persistent_err_word(self) -> Optional[torch.Tensor]:
        """The persistent kernel's error word in its workspace (int32 [1], cleared by every launch),
        for the runner's per-step readback; None before the first launch."""
        if self._pd is None:
            return None
        off = int(ops._hip.require().ka_decode_persistent_err_offset())
        return self._pd[1][off:off + 4].view(torch.int32)

    def persistent_err(self) -> int:
        """Error word of the last persistent launch (a grid wait that ran out; 0 in a correct run)."""
        if self._pd is None:
            return 0
        return int(ops._hip.require().ka_decode_persistent_err(self._pd[1].data_ptr(), ops._stream()))

    def _fork_prefetch(self, L, T: int):
        """Start the side-stream prefetch of this layer's gate_up weights (see __init__); returns the
        stream to join before gate_up, or None."""
        if not self.prefetch_bytes or T > self.prefetch_max_b or not self.device.type == "cuda" or "w13" not in L:
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        side = self._side
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            ops.prefetch(L["w13"], self.prefetch_bytes, self.prefetch_blocks)
        return side

    def _reduce_norm(self, h, w, eps, residual, pending: bool):
        """residual += all_reduce(h) (when `pending`); return rmsnorm(residual) * w.  TP = 1: h may be
        split-K partials (the reduction is fused into the norm kernel); TP > 1: the all-reduce is
        fused with the norm for decode-size rows (one-shot kernel) or runs before it."""
        if not pending or self._local_comm:
            return ops.rmsnorm(h, w, eps, residual=residual)
        return self.comm.all_reduce_rmsnorm(h, w, eps, residual)

    def _attention(self, q, meta: AttnMeta, kc: torch.Tensor, vc: torch.Tensor) -> torch.Tensor:
        if meta.is_decode:
            return ops.attention_decode(q, kc, vc, meta.block_tables, meta.ctx_lens, self.scale)
        if meta.num_decode:
            # mixed step: prompt rows through the varlen prefill kernel, the leading decode rows
            # through the decode kernel (a 1-row query would waste a 64-row prefill tile)
            nd = meta.num_decode
            a = ops.attention_prefill(q, kc, vc, meta.block_tables[nd:], meta.q_starts[nd:], meta.ctx_lens[nd:],
                                      meta.max_q_len, self.scale, out=torch.empty_like(q))
            ops.attention_decode(q[:nd], kc, vc, meta.block_tables[:nd], meta.ctx_lens[:nd], self.scale, out=a[:nd])
            return a
        return ops.attention_prefill(q, kc, vc, meta.block_tables, meta.q_starts, meta.ctx_lens, meta.max_q_len,
                                     self.scale)

    def logits(self, hidden_last: torch.Tensor) -> torch.Tensor:
        """Vocab-parallel logits of this rank: [S, V / tp] (bf16)."""
        return ops.linear(hidden_last, self.W["lm_head"])

    def sample(self, hidden_last: torch.Tensor, mask_bits: Optional[torch.Tensor],
               mask_idx: Optional[torch.Tensor]) -> torch.Tensor:
        """Greedy (temperature 0, app.py:109) next tokens under the SAFE_DECODE mask: [S] int32.
        Where it measured faster (ops.use_fused_lm_head), the LM head GEMM and the masked argmax are
        one kernel and the logits are never written."""
        lm = self.W["lm_head"]
        if ops.use_fused_lm_head(hidden_last, lm, self.vocab_offset):
            idx, val = ops.lm_head_argmax(hidden_last, lm, mask_bits, mask_idx, vocab_offset=self.vocab_offset)
        else:
            logits = self.logits(hidden_last)
            idx, val = ops.masked_argmax(logits, mask_bits, mask_idx, vocab_offset=self.vocab_offset)
        if self.tp_size == 1:
            return idx
        vals = self.comm.all_gather(val)                       # [t, S]
        idxs = self.comm.all_gather(idx)                       # [t, S]
        return ops.argmax_combine(vals, idxs)                  # lowest id (= lowest rank) on ties
