"""Model runner: KV cache ownership, step metadata, eager prefill, hipGraph decode, TP fan-out.

Decode steps dominate the request latency (one replay per output token, SURVEY.md §3.6 hot loop 1),
so they are captured once per batch bucket (`HIPGRAPH_BUCKETS`) with `torch.cuda.CUDAGraph` (a
hipGraph on ROCm): embedding -> 32 x (norm, QKV GEMM, RoPE+KV append, paged decode attention, O
GEMM [+ all-reduce], norm, gate_up GEMM, SiLU*mul, down GEMM [+ all-reduce]) -> norm -> LM head ->
masked argmax [+ all-gather].  All per-step inputs live in ONE device staging tensor at fixed
offsets so a step is: one pinned host->device copy, one graph replay, one 4*B-byte readback.

With TP > 1 the driver rank (rank 0) owns the scheduler; every step it broadcasts a small header
and the packed metadata and all ranks run the same forward, the collectives
inside it synchronising them.  Worker ranks sit in `worker_loop()`.
"""
from __future__ import annotations

import bisect
import logging
import os
import time
from typing import Dict, List, NamedTuple, Optional

import numpy as np
import torch

from ..models.config import ModelConfig
from .. import ops
from ..models.llama import AttnMeta, LlamaModel

logger = logging.getLogger("app.engine")
from ..parallel.comm import LocalComm
from .safe_decode import mask_index_for
from .scheduler import Batch
from .sequence import PLACEHOLDER

KIND_STOP, KIND_DECODE, KIND_PREFILL = 0, 1, 2
HDR = 8


class CollectiveTimeout(RuntimeError):
    """A one-shot TP collective gave up waiting for a peer (csrc/allreduce.hip's bounded spin set its
    error word): the step's reduced values are stale, so its tokens must not be used.  Fatal for
    the process (the TP group's collective epochs are out of step): engine.py fails the in-flight
    requests with 503 and marks the engine unhealthy / exits for the supervisor to restart it."""


def shared_prefix_len(bt: np.ndarray, lim: int) -> int:
    """Length of the common prefix of the rows of `bt` ([B, max_blocks]) within the first `lim` columns."""
    if lim <= 0 or bt.shape[0] == 0:
        return 0
    eq = (bt[:, :lim] == bt[0:1, :lim]).all(axis=0)
    return lim if bool(eq.all()) else int(np.argmin(eq))


class PersistentStall(RuntimeError):
    """The batch-1 persistent decode kernel (csrc/decode_persistent.hip) gave up a grid-wide wait:
    some workgroup never ran (the GPU shared with another kernel), so the step's hidden state is
    stale.  Recoverable: the engine fails the in-flight requests and recovers; the runner has
    already switched batch-1 decode back to the per-kernel chain."""


class StepHandle(NamedTuple):
    """A step queued on the device and not yet read back (`collect`)."""
    event: Optional["torch.cuda.Event"]   # recorded after the step's token readback copy
    host_out: torch.Tensor                # pinned host buffer the sampled tokens land in
    rows: int
    t0: float                             # perf_counter at launch
    prefill_tokens: int = 0               # > 0: a prefill step (launch_prefill_async)
    progress: Optional["torch.cuda.Event"] = None   # recorded KA_LOOKAHEAD_LAYERS layers before the end
    err_host: Optional[torch.Tensor] = None   # pinned copy of the one-shot collectives' error word

class ModelRunner:
    def __init__(self, cfg: ModelConfig, weights: Dict[str, torch.Tensor], device: torch.device,
                 num_blocks: int, block_size: int = 16, max_model_len: int = 4096, graph_buckets=(1, 2, 4, 8),
                 mask_bits: Optional[np.ndarray] = None, comm=None, tp_rank: int = 0, tp_size: int = 1,
                 ep_rank: int = 0, ep_size: int = 1, use_graphs: bool = True):
        self.cfg = cfg
        self.device = torch.device(device)
        self.comm = comm or LocalComm()
        # mixed steps: decode rows through the decode kernel (KA_SPLIT_MIXED_ATTN=0: all varlen)
        self.split_mixed_attention = os.environ.get("KA_SPLIT_MIXED_ATTN", "1") == "1"
        self.prefill_pad = int(os.environ.get("KA_PREFILL_PAD", "256"))
        self.prefill_pad_min = int(os.environ.get("KA_PREFILL_PAD_MIN", "1024"))
        # an async prefill / mixed step records a progress event this many layers before its end: the
        # engine schedules the step after it once that event has passed (engine._lookahead_step)
        self.lookahead_layers = int(os.environ.get("KA_LOOKAHEAD_LAYERS", "10"))
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.model = LlamaModel(cfg, weights, self.comm, tp_rank, tp_size, ep_rank, ep_size)
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.max_blocks = (max_model_len + block_size - 1) // block_size
        hkv = cfg.num_kv_heads // tp_size
        L, D = cfg.num_layers, cfg.head_dim
        dt = weights["embed"].dtype
        # zero-filled: stale slots read by masked lanes must be finite (attention.hip contract)
        self.k_cache = torch.zeros((L, num_blocks, hkv, block_size, D), dtype=dt, device=self.device)
        self.v_cache = torch.zeros((L, num_blocks, hkv, D, block_size), dtype=dt, device=self.device)
        self.mask_bits = (torch.from_numpy(mask_bits.view(np.int32)).to(self.device)
                          if mask_bits is not None else None)
        self.buckets = sorted(set(int(b) for b in graph_buckets))
        self.bmax = self.buckets[-1] if self.buckets else 1
        self.use_graphs = use_graphs and self.device.type == "cuda"
        # ---- decode staging: [ids | pos | slots | ctx | mask | block_tables] at fixed offsets ----
        B = self.bmax
        # nsh: the leading block-table entries every row shares (cascade decode attention, 16-int slot)
        self._off = {"ids": 0, "pos": B, "slots": 2 * B, "ctx": 3 * B, "mask": 4 * B, "nsh": 5 * B, "bt": 5 * B + 16}
        self._stage_len = 5 * B + 16 + B * self.max_blocks
        # cascade decode attention from this bucket up (KA_CASCADE_MIN_B; 0 = off, the default): the
        # shared prefix blocks attended once per kv head and 16 query rows instead of once per row.
        # Measured slower at B = 64 / 256 with a 5-block shared prefix (+0.23 / +0.14 ms per step,
        # profiles/r4/cascade/): the per-row kernel's prefix reads are L2 hits, and the partials'
        # round trip plus the second launch cost more than they save.
        self.cascade_min_b = int(os.environ.get("KA_CASCADE_MIN_B", "0"))
        self.d_stage = torch.zeros(self._stage_len, dtype=torch.int32, device=self.device)
        pin = self.device.type == "cuda"
        self.h_stage = torch.zeros(self._stage_len, dtype=torch.int32, pin_memory=pin)
        self.h_np = self.h_stage.numpy()
        # overlapped decode (launch_decode_async): second pinned staging / output buffers so step
        # t+1 can be packed and queued while step t's copies are still in flight
        self._h_stages = [self.h_stage, torch.zeros(self._stage_len, dtype=torch.int32, pin_memory=pin)]
        self._h_outs = [torch.zeros(B, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._flip = 0
        self.d_logits_idx = torch.arange(B, dtype=torch.int64, device=self.device)
        self.d_out = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.h_out = torch.zeros(B, dtype=torch.int32, pin_memory=pin)
        # steps queued ahead of a readback (engine._lookahead_step): prefill / mixed staging in grown
        # pinned buffers and token outputs, each double-buffered (a buffer is reused two launches
        # later, when the step that used it has been read back), and the placeholder fixups of a
        # decode step ([dst rows | src rows] of d_out)
        self._h_pre: List[Optional[torch.Tensor]] = [None, None]
        self._sflip = 0
        self._h_pouts = [torch.zeros(B, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._pflip = 0
        self._h_fix = [torch.zeros(2 * B, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.d_fix = torch.zeros(2 * B, dtype=torch.int32, device=self.device)
        self.d_hdr = torch.zeros(HDR, dtype=torch.int32, device=self.device)
        self._h_hdrs = [torch.zeros(HDR, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._hflip = 0
        # the one-shot TP collectives' error word rides back with every step's tokens (a pinned
        # 4-byte copy behind them on the same stream: no extra synchronisation), one slot per launch
        # parity like the token outputs
        self._h_errs = [torch.zeros(2, dtype=torch.int32, pin_memory=pin) for _ in range(4)]
        self._eflip = 0
        # TP decode overlap: rank 0 queues step t+1 (header + staging broadcast + graph) before
        # reading step t back.  Needs collectives that are stream-ordered on the device (RCCL):
        # with a host-synchronous transport (gloo) the step still works, it just does not overlap.
        ov = os.environ.get("KA_TP_OVERLAP", "1")
        self.tp_overlap = tp_size > 1 and (ov == "force" or (ov == "1" and getattr(self.comm, "device_ordered", False)))
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_pool = None
        self.stats = {"decode_steps": 0, "prefill_steps": 0, "graph_replays": 0, "decode_ms": 0.0,
                      "prefill_ms": 0.0, "prefill_tokens": 0, "persistent_stalls": 0}
        # bucket -> the captured graph holds the persistent decode kernel (its error word must be read
        # back on every replay of that graph, whatever model.persistent says now)
        self.graph_persistent: Dict[int, bool] = {}
        # graphs taken out of service while a replay may still be queued (freed by health_check)
        self._retired_graphs: List[object] = []

    # ------------------------------------------------------------------------------------------
    def _view(self, name: str, n: int) -> torch.Tensor:
        o = self._off[name]
        if name == "bt":
            return self.d_stage[o:o + n * self.max_blocks].view(n, self.max_blocks)
        return self.d_stage[o:o + n]

    def _cascade(self, B: int) -> bool:
        return self.cascade_min_b > 0 and B >= self.cascade_min_b and self.device.type == "cuda"

    def _decode_forward(self, B: int) -> None:
        meta = AttnMeta(positions=self._view("pos", B), slot_mapping=self._view("slots", B),
                        block_tables=self._view("bt", B), ctx_lens=self._view("ctx", B),
                        logits_indices=self.d_logits_idx[:B], is_decode=True,
                        shared_blocks=self._view("nsh", 1) if self._cascade(B) else None)
        h = self.model.forward(self._view("ids", B), meta, self.k_cache, self.v_cache)
        mask_idx = self._view("mask", B) if self.mask_bits is not None else None
        tok = self.model.sample(h, self.mask_bits, mask_idx)
        self.d_out[:B].copy_(tok)

    def autotune(self) -> dict:
        """Pick hipBLASLt vs the hand-written decode GEMM per (bucket, N, K) on this model's weights."""
        if self.device.type != "cuda":
            return {}
        from ..ops.autotune import tune_linear
        groups = {}
        norm_fed = set()
        # O / down partials feed the norm directly at TP = 1, and in a TP rank's decode step when the
        # collective reduces them (models/llama.py `fuse`): timed with that consumer
        local = getattr(self.model, "_local_comm", False) or getattr(self.model.comm, "splitk_norm", False)
        for L in self.model.layers:
            for k in ("wqkv", "wo", "w13", "w2"):
                w = L.get(k)
                if w is not None and w.dim() == 2:
                    groups.setdefault(tuple(w.shape), []).append(w)
                    if local and k in ("wo", "w2"):   # llama.py defers their split-K reduce into the norm
                        norm_fed.add(tuple(w.shape))
        lm = self.model.W["lm_head"]
        groups.setdefault(tuple(lm.shape), []).append(lm)
        consumers = {}
        m = self.model
        if m.fuse_decode_rope and m.D == 128 and self.block_size == 16 and "wqkv" in m.layers[0]:
            # QKV is timed with its real consumer, the fused RoPE + KV append + decode attention
            # on a synthetic 128-token context (a norm stand-in picked a split plan whose partials
            # then slowed the attention prologue: profiles/phase_profile_c256_qkv_proxy_negative.txt)
            consumers[tuple(m.layers[0]["wqkv"].shape)] = (self._attention_consumer(), m.bf16_qkv_partials)
        bf16 = getattr(self.model, "bf16_partials", False)
        ctx_of = {nk: ("attn" + ("-bf16" if consumers[nk][1] else "")) if nk in consumers else
                  ("norm" + ("-bf16" if bf16 else "")) if nk in norm_fed else "plain" for nk in groups}
        from ..ops import TILE_MAX_M
        from ..ops.autotune import DEFAULT_PLAN_FILE, load_plan, save_plan
        wanted = {(M, N, K): ctx_of[(N, K)] for (N, K) in groups for M in set(self.buckets) if M <= TILE_MAX_M}
        mode = os.environ.get("KA_GEMM_PLAN", "file")
        path = os.environ.get("KA_GEMM_PLAN_FILE", DEFAULT_PLAN_FILE)
        Ms = self.buckets
        if mode == "file":
            missing = load_plan(path, wanted)
            if not missing:
                return {"from": path}
            Ms = sorted({M for (M, _, _) in missing})
            groups = {nk: ws for nk, ws in groups.items() if any((M,) + nk in missing for M in Ms)}
        report = tune_linear(groups, Ms, norm_fed, bf16, consumers)
        if mode == "write":
            save_plan(path, report, ctx_of)
        return report

    @torch.inference_mode()
    def tune_lm_head(self) -> dict:
        """Per decode bucket: the fused LM head + masked argmax (csrc/gemm_big.hip) against the
        GEMM plan's LM head + masked_argmax, on the model's own LM head and a SAFE_DECODE mask row;
        fills ops.LM_HEAD_FUSED and the threshold for untimed row counts."""
        m = self.model
        lm = m.W["lm_head"]
        if self.device.type != "cuda" or ops.LM_HEAD_MODE != "auto":
            return {}
        from ..ops.autotune import _time, load_section, plan_mode, save_section
        K = lm.shape[1]
        report = {}
        # persisted with the GEMM plan (ops/tuned/gemm_plan_mi355x.json, section lm_head): the same
        # decision on every box and run unless KA_GEMM_PLAN=tune / write re-times it
        mode, path = plan_mode()
        key = lambda M: f"{M},{lm.shape[0]},{K},{int(self.mask_bits is not None)}"   # noqa: E731
        saved = load_section(path, "lm_head") if mode == "file" else {}
        for M in sorted(set(self.buckets)):
            x = torch.randn(M, K, device=self.device, dtype=lm.dtype)
            if not ops.lm_head_argmax_ok(x, lm, m.vocab_offset):
                return {}
            if key(M) in saved:
                fused, t_fu, t_un = saved[key(M)]
            else:
                midx = (torch.zeros(M, dtype=torch.int32, device=self.device) if self.mask_bits is not None else None)
                t_un = _time(lambda w: ops.masked_argmax(ops.linear(x, w), self.mask_bits, midx, m.vocab_offset), [lm])
                t_fu = _time(lambda w: ops.lm_head_argmax(x, w, self.mask_bits, midx, m.vocab_offset), [lm])
                # within the plan's margin the hand-written fused kernel is taken over a hipBLASLt plan
                # (ops/autotune.py BLAS_MARGIN), as for the GEMM plan and the decode SwiGLU
                from ..ops.autotune import BLAS_MARGIN
                plan = ops.GEMM_PLAN.get((M, lm.shape[0], K), ("blas",))
                fused = t_fu < t_un * (1.0 + (BLAS_MARGIN if plan[0] == "blas" else 0.0))
            ops.LM_HEAD_FUSED[M] = bool(fused)
            report[M] = {"fused_us": round(t_fu, 1), "unfused_us": round(t_un, 1), "fused": bool(fused)}
        if mode == "write":
            save_section(path, "lm_head", {key(M): [r["fused"], r["fused_us"], r["unfused_us"]]
                                          for M, r in report.items()})
        wins = sorted(M for M, f in ops.LM_HEAD_FUSED.items() if f)
        # untimed row counts: fused from the smallest bucket above which every timed bucket won
        ops.LM_HEAD_FUSED_MIN_M = next((M for M in wins if all(ops.LM_HEAD_FUSED[b] for b in ops.LM_HEAD_FUSED
                                                                  if b >= M)), 1 << 30)
        logger.info("lm head plan: %s (fused from %d rows)", report, ops.LM_HEAD_FUSED_MIN_M)
        return report

    @torch.inference_mode()
    def tune_prefill(self) -> dict:
        """Prefill / mixed-step projections (ops.PREFILL_GEMM auto): csrc/gemm_big.hip against hipBLASLt
        per (N, K) of the model's QKV / O / down at the row-count buckets of ops.PREFILL_BUCKETS, on
        the model's own weights rotated over layers (the persisted decision in the plan file, section
        prefill, unless KA_GEMM_PLAN=tune / write).  Fills ops.PREFILL_PLAN: gemm_big where it is within
        KA_PREFILL_MARGIN (default 0.02) of hipBLASLt."""
        m = self.model
        ops.PREFILL_PLAN.clear()
        if self.device.type != "cuda" or ops.PREFILL_GEMM != "auto":
            return {}
        from ..ops.autotune import _time, load_section, plan_mode, save_section
        margin = float(os.environ.get("KA_PREFILL_MARGIN", "0.02"))
        groups = {}
        for L in m.layers:
            for k in ("wqkv", "wo", "w2"):
                w = L.get(k)
                if w is not None and w.dim() == 2:
                    groups.setdefault(tuple(w.shape), []).append(w)
        mode, path = plan_mode()
        saved = load_section(path, "prefill") if mode == "file" else {}
        report = {}
        for (N, K), ws in groups.items():
            ws = ws[:4]
            for M in ops.PREFILL_BUCKETS:
                key = f"{M},{N},{K}"
                if key in saved:
                    big, t_big, t_blas = saved[key]
                else:
                    x = torch.randn(M, K, device=self.device, dtype=ws[0].dtype)
                    if not ops.big_gemm_ok(x, ws[0]):
                        break
                    t_blas = _time(lambda w: torch.nn.functional.linear(x, w), ws, reps=6)
                    t_big = _time(lambda w: ops.linear_big(x, w), ws, reps=6)
                    big = t_big <= t_blas * (1.0 + margin)
                    del x
                ops.PREFILL_PLAN[(M, N, K)] = bool(big)
                report[key] = [bool(big), round(float(t_big), 1), round(float(t_blas), 1)]
        if mode == "write":
            save_section(path, "prefill", report)
        logger.info("prefill gemm plan: %s", report)
        return report

    @torch.inference_mode()
    def tune_swiglu(self) -> dict:
        """Per decode bucket: gate_up with the ring kernel's SwiGLU epilogue (ops.linear_gm_swiglu,
        each configuration) against the GEMM plan's gate_up + SiLU·mul, on the model's own w13
        rotated over layers; fills ops.DECODE_SWIGLU_CFG with the winners."""
        m = self.model
        ops.DECODE_SWIGLU_CFG.clear()
        if self.device.type != "cuda" or ops.DECODE_SWIGLU == "0" or getattr(m.cfg, "is_moe", False):
            return {}
        ws = [L["w13"] for L in m.layers if L.get("w13") is not None and L["w13"].dim() == 2][:8]
        if not ws:
            return {}
        w2s = [L["w2"] for L in m.layers if L.get("w2") is not None and L["w2"].dim() == 2][:8]
        from ..ops.autotune import _time, load_section, plan_mode, save_section
        report = {}
        mode, path = plan_mode()   # persisted like the GEMM plan (section decode_swiglu)
        key = lambda M: f"{M},{ws[0].shape[0]},{ws[0].shape[1]}"   # noqa: E731
        saved = load_section(path, "decode_swiglu") if mode == "file" else {}
        for M in sorted(set(self.buckets)):
            x = torch.randn(M, ws[0].shape[1], device=self.device, dtype=ws[0].dtype)
            if not ops.decode_swiglu_ok(x, ws[0]):
                continue
            if key(M) in saved:
                cfg, t_fu, t_un = saved[key(M)]
                best = (int(cfg), t_fu if int(cfg) else t_un)
                fused = (int(cfg), t_fu)
            else:
                small = M <= ops.GEMV_SWIGLU_MAX_M and len(w2s) == len(ws)
                if small:
                    # the unfused path at these rows computes SiLU·mul inside the down GEMV's staging
                    # (ops.swiglu_linear): compare gate_up + down, both ways (indices pair w13 / w2)
                    pair = {id(a): b for a, b in zip(ws, w2s)}
                    t_un = _time(lambda w: ops.swiglu_linear(ops.linear(x, w, defer_reduce=True), pair[id(w)]), ws)
                else:
                    t_un = _time(lambda w: ops.silu_mul(ops.linear(x, w, defer_reduce=True)), ws)
                fused = (0, float("inf"))
                cands = list(ops.DECODE_SWIGLU_CFGS)
                if M >= ops.BIG_PLAN_MIN_M and ops.swiglu_gemm_ok(x, ws[0]):
                    cands.append(ops.DECODE_SWIGLU_BIG)   # csrc/gemm_big.hip's SwiGLU epilogue
                for cfg in cands:
                    if small:
                        t = _time(lambda w: ops.linear(ops.linear_gm_swiglu(x, w, cfg), pair[id(w)]), ws)
                    else:
                        t = _time(lambda w: ops.linear_gm_swiglu(x, w, cfg), ws)
                    if t < fused[1]:
                        fused = (cfg, t)
                # the unfused path's gate_up is a hipBLASLt plan: the hand-written fused kernel is
                # taken within the plan's margin too (ops/autotune.py BLAS_MARGIN)
                from ..ops.autotune import BLAS_MARGIN
                plan = ops.GEMM_PLAN.get((M, ws[0].shape[0], ws[0].shape[1]), ("blas",))
                margin = BLAS_MARGIN if plan[0] == "blas" else 0.0
                best = fused if fused[1] < t_un * (1.0 + margin) else (0, t_un)
            ops.DECODE_SWIGLU_CFG[M] = best[0]   # 0 (unfused) is kept too: un-timed M take the next bucket
            # fused_us: the fastest SwiGLU-epilogue configuration's time, whether or not it was taken
            report[M] = {"cfg": best[0], "fused_us": round(fused[1], 1), "unfused_us": round(t_un, 1)}
        if mode == "write":
            save_section(path, "decode_swiglu", {key(M): [r["cfg"], r["fused_us"], r["unfused_us"]]
                                                for M, r in report.items()})
        logger.info("decode swiglu plan: %s", report)
        return report

    def _attention_consumer(self, ctx: int = 128):
        """fn(qkv, M): decode_attention_rope over M synthetic sequences of `ctx` cached tokens in
        layer 0's cache (autotune runs before serving: the KV written here is never read)."""
        m, bs = self.model, self.block_size
        nb = (ctx + bs - 1) // bs
        memo = {}

        def consume(qkv, M):
            if M not in memo:
                bt = (torch.arange(M * nb, dtype=torch.int32, device=self.device) % self.num_blocks).view(M, nb)
                pos = torch.full((M,), ctx - 1, dtype=torch.int32, device=self.device)
                slots = (bt[:, -1] * bs + (ctx - 1) % bs).to(torch.int32)
                lens = torch.full((M,), ctx, dtype=torch.int32, device=self.device)
                memo[M] = (pos, slots, bt.contiguous(), lens)
            pos, slots, bt, lens = memo[M]
            return ops.decode_attention_rope(qkv, pos, m.cos_sin, slots, self.k_cache[0], self.v_cache[0], bt, lens,
                                             m.hq, m.hkv, m.D, m.scale)
        return consume

    @torch.inference_mode()
    def capture_graphs(self, autotune: bool = True) -> float:
        """Capture one decode graph per bucket (largest first, sharing a memory pool)."""
        if not self.use_graphs:
            return 0.0
        t0 = time.perf_counter()
        if self.device.type == "cuda":
            ops.gemm_big_ws(self.device)   # allocated (and zeroed) outside any capture
        if autotune:
            self.gemm_plan = self.autotune()
            self.lm_head_plan = self.tune_lm_head()
            self.swiglu_plan = self.tune_swiglu()
            self.prefill_plan = self.tune_prefill()
        self.h_np[:] = 0
        o = self._off
        for name in ("slots",):
            self.h_np[o[name]:o[name] + self.bmax] = -1
        self.h_np[o["mask"]:o["mask"] + self.bmax] = -1
        self.d_stage.copy_(self.h_stage)
        stream = torch.cuda.Stream(self.device)
        stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(stream):
            for B in reversed(self.buckets):
                self._decode_forward(B)  # warm-up (hipBLASLt heuristics, allocator)
        torch.cuda.current_stream(self.device).wait_stream(stream)
        torch.cuda.synchronize(self.device)
        for B in reversed(self.buckets):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.graph_pool):
                self._decode_forward(B)
            if self.graph_pool is None:
                self.graph_pool = g.pool()
            self.graphs[B] = g
            self.graph_persistent[B] = self.model.persistent_ok(B)
        torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0

    # ------------------------------------------------------------------------------------------
    def _slot(self, table: List[int], pos: int) -> int:
        return table[pos // self.block_size] * self.block_size + pos % self.block_size

    def _pack_decode(self, batch: Batch, Bp: int, h: Optional[np.ndarray] = None, ahead: int = 0) -> None:
        """Fill the decode staging image.  ahead = 1: for the step after the one in flight (its token
        is not appended yet; ids then come from the device, launch_decode_async)."""
        h = self.h_np if h is None else h
        o, mb = self._off, self.max_blocks
        B = len(batch.seqs)
        for i, s in enumerate(batch.seqs):
            if not s.block_table:   # a freed (finished) sequence: its slots would alias block 0
                raise RuntimeError(f"decode row {i} (seq {s.seq_id}) has no KV blocks")
            L = s.total_len + ahead
            pos = L - 1
            h[o["ids"] + i] = s.all_ids[-1] if not ahead else 0
            h[o["pos"] + i] = pos
            h[o["slots"] + i] = self._slot(s.block_table, pos)
            h[o["ctx"] + i] = L
            h[o["mask"] + i] = mask_index_for(s.num_generated + ahead, s.params.safe_decode)
            row = o["bt"] + i * mb
            n = len(s.block_table)
            h[row:row + n] = s.block_table
        if Bp > B:  # padding rows: no cache write, empty context
            for name, val in (("ids", 0), ("pos", 0), ("slots", -1), ("ctx", 0), ("mask", -1)):
                h[o[name] + B:o[name] + Bp] = val
        h[o["nsh"]] = self._shared_prefix_blocks(batch, h, ahead) if self._cascade(Bp) else 0

    def _shared_prefix_blocks(self, batch: Batch, h: np.ndarray, ahead: int) -> int:
        """Leading block-table entries that every row shares, counting only blocks full of cached
        tokens (the new token's block is each row's own)."""
        o, mb, B = self._off, self.max_blocks, len(batch.seqs)
        lim = min((s.total_len + ahead - 1) // self.block_size for s in batch.seqs)
        return shared_prefix_len(h[o["bt"]:o["bt"] + B * mb].reshape(B, mb), lim)

    def can_overlap(self, B: int) -> bool:
        """A decode step of B rows can be queued before the previous one is read back.
        (on CPU the "async" launch simply runs synchronously: same code path, testable)"""
        return (self.tp_size == 1 or self.tp_overlap) and B <= self.bmax

    def can_overlap_prefill(self, B: int) -> bool:
        return (self.tp_size == 1 or self.tp_overlap) and B <= self.bmax

    def can_lookahead(self) -> bool:
        """Steps can be scheduled and queued ahead of the in-flight step's readback.  With TP, rank 0
        applies the placeholder fixups on the device BEFORE the staging broadcast (every rank samples
        the same tokens into its d_out, but only rank 0 knows the fixup list), so the other ranks
        receive final inputs; needs stream-ordered collectives (tp_overlap) to actually overlap."""
        return self.tp_size == 1 or self.tp_overlap

    @torch.inference_mode()
    def launch_decode_async(self, batch: Batch, chained: bool = False, fix: Optional[List[tuple]] = None):
        """Queue one decode step without waiting for it.  chained: `batch` is the step after the one
        in flight (same sequences, same row order): its input ids are copied on the device from the
        previous step's sampled tokens (with TP, on rank 0 before the staging broadcast, so the other
        ranks receive them; every rank samples the same token).  fix: (row, src) pairs of rows whose
        input is a PLACEHOLDER: their ids are the in-flight step's sampled tokens d_out[src] (a step
        scheduled ahead, engine._lookahead_step).  Returns a handle for `collect`."""
        B = len(batch.seqs)
        i = bisect.bisect_left(self.buckets, B)
        Bp = self.buckets[i] if i < len(self.buckets) else B
        t0 = time.perf_counter()
        k = self._flip
        self._flip ^= 1
        hs, ho = self._h_stages[k], self._h_outs[k]
        self._pack_decode(batch, Bp, hs.numpy(), ahead=1 if chained else 0)
        n_copy = self._off["bt"] + Bp * self.max_blocks
        self._bcast_header_async(KIND_DECODE, Bp, n_copy)
        self.d_stage[:n_copy].copy_(hs[:n_copy], non_blocking=True)
        if chained:
            o = self._off["ids"]
            self.d_stage[o:o + B].copy_(self.d_out[:B])
        if fix:
            nf = len(fix)
            hf = self._h_fix[k]
            hf.numpy()[:2 * nf] = np.asarray(fix, dtype=np.int32).T.reshape(-1)
            self.d_fix[:2 * nf].copy_(hf[:2 * nf], non_blocking=True)
            o = self._off["ids"]
            self.d_stage[o:o + Bp].index_copy_(0, self.d_fix[:nf].long(),
                                               self.d_out.index_select(0, self.d_fix[nf:2 * nf].long()))
        self._launch_decode(Bp, n_copy)
        ho[:B].copy_(self.d_out[:B], non_blocking=True)
        eh = self._copy_err(persistent=self._persistent_step(Bp))
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        return StepHandle(ev, ho, B, t0, err_host=eh)

    @torch.inference_mode()
    def launch_prefill_async(self, batch: Batch):
        """Queue a prefill or mixed step without waiting for its tokens (at most `bmax` rows; with TP,
        rank 0 broadcasts the header and the fixed-up metadata, stream-ordered):
        the sampled tokens are also left in `d_out`, in batch row order, so the next step can be
        queued right behind it with its inputs taken on the device (`launch_decode_async(chained=
        True)` for the same rows, or the PLACEHOLDER fixups of a step scheduled ahead).  Rows whose
        input is a PLACEHOLDER (this batch was scheduled ahead of the in-flight step's readback) get
        it from `d_out` before the forward.  Returns a handle for `collect`."""
        t0 = time.perf_counter()
        host, nf = self._pack_prefill(batch, pad=True, with_fix=True)
        T, S, max_q, nc = self.padded_tokens(batch.num_tokens), len(batch.seqs), max(batch.num_query), len(batch.copies)
        nd = S - len(batch.prefill_seqs) if self.split_mixed_attention else 0
        buf = self._stage_prefill(host)
        if nf:   # trailing [dst positions | src rows]
            n = buf.shape[0]
            buf[:T].index_copy_(0, buf[n - 2 * nf:n - nf].long(), self.d_out.index_select(0, buf[n - nf:].long()))
            buf = buf[:n - 2 * nf]
        if self.tp_size > 1:   # the other ranks get the fixed-up metadata (worker_loop KIND_PREFILL)
            self._bcast_header_async(KIND_PREFILL, T, S, max_q, buf.shape[0], nc, nd, batch.num_tokens)
            self.comm.broadcast(buf, src=0)
        self.model.mark_layer = max(0, self.cfg.num_layers - self.lookahead_layers)
        self.model.mark_event = None
        try:
            tok = self._run_prefill(buf, T, S, max_q, nc, nd, batch.num_tokens)
        finally:
            self.model.mark_layer = -1
        progress, self.model.mark_event = self.model.mark_event, None
        self.d_out[:S].copy_(tok)
        ho = self._h_pouts[self._pflip]
        self._pflip ^= 1
        ho[:S].copy_(tok, non_blocking=True)
        eh = self._copy_err()
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        return StepHandle(ev, ho, S, t0, prefill_tokens=T, progress=progress, err_host=eh)

    def _stage_prefill(self, host: np.ndarray) -> torch.Tensor:
        """Packed prefill metadata -> device without a host sync: through one of two pinned buffers
        (grown on demand; the one being refilled served the launch before last, already read back)."""
        if self.device.type != "cuda":
            return torch.from_numpy(host)
        n = host.shape[0]
        k = self._sflip = self._sflip ^ 1
        hb = self._h_pre[k]
        if hb is None or hb.numel() < n:
            hb = torch.empty(max(n, 2 * (hb.numel() if hb is not None else 0), 1 << 16), dtype=torch.int32,
                             pin_memory=True)
            self._h_pre[k] = hb
        hb.numpy()[:n] = host
        return hb[:n].to(self.device, non_blocking=True)

    @torch.inference_mode()
    def health_check(self) -> None:
        """Raise if the device no longer answers: a tiny kernel through the stream and a sync."""
        probe = self.d_out[:1] + 0
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        int(probe[0].item())
        # nothing queued before the synchronize can still be replaying a retired graph
        self._retired_graphs.clear()

    def _err_word(self) -> Optional[torch.Tensor]:
        car = getattr(self.comm, "custom_ar", None)
        return car.state[2:3] if car is not None else None

    def _persistent_step(self, Bp: int) -> bool:
        """The decode step of bucket Bp runs the persistent kernel (its error word is read back): the
        captured graph decides when there is one (a graph captured with the kernel keeps launching it
        after model.persistent is turned off), the model's current setting otherwise."""
        if Bp in self.graphs:
            return self.graph_persistent.get(Bp, False)
        return self.model.persistent_ok(Bp)

    def _copy_err(self, persistent: bool = False) -> Optional[torch.Tensor]:
        """Queue the error word's readback behind the step just launched: [one-shot collectives,
        persistent decode kernel] (None when the step has neither)."""
        src = self._err_word()
        psrc = self.model.persistent_err_word() if persistent else None
        if src is None and psrc is None:
            return None
        h = self._h_errs[self._eflip]
        self._eflip = (self._eflip + 1) % len(self._h_errs)
        h.zero_()
        if src is not None:
            h[0:1].copy_(src, non_blocking=True)
        if psrc is not None:
            h[1:2].copy_(psrc, non_blocking=True)
        return h

    def _check_err(self, h: Optional[torch.Tensor]) -> None:
        if h is None:
            return
        if int(h[0]):
            raise CollectiveTimeout("one-shot TP collective: a peer never arrived (spin timeout); "
                                    "the step's results are stale")
        if int(h[1]):
            self.model.persistent = False   # the chain from now on: co-residency cannot be relied on
            # a graph captured with the persistent kernel would keep replaying it: take those graphs
            # out of service (their buckets run eagerly, the kernel chain, from the next step on).  The
            # engine may already have queued a chained step that replays one of them, so the graph
            # objects are only retired here; health_check() frees them after a device synchronize
            # (destroying a hipGraphExec with a launch still pending is not defined)
            for b in [b for b, p in self.graph_persistent.items() if p]:
                g = self.graphs.pop(b, None)
                if g is not None:
                    self._retired_graphs.append(g)
                self.graph_persistent.pop(b, None)
            self.stats["persistent_stalls"] += 1
            logger.error("persistent decode kernel: a grid wait ran out; batch-1 decode falls back to "
                         "the kernel chain (stall #%d)", self.stats["persistent_stalls"])
            raise PersistentStall("persistent decode: a workgroup never ran (grid wait timeout); "
                                  "the step's results are stale")

    def collect(self, handle: "StepHandle") -> List[int]:
        ev, ho, B, t0 = handle.event, handle.host_out, handle.rows, handle.t0
        if handle.prefill_tokens:   # launch_prefill_async
            if ev is not None:
                ev.synchronize()
            now = time.perf_counter()
            self.stats["prefill_steps"] += 1
            self.stats["prefill_tokens"] += handle.prefill_tokens
            self.stats["prefill_ms"] += (now - t0) * 1e3
            self._last_collect = now
            self._check_err(handle.err_host)
            return ho[:B].tolist()
        if ev is not None:
            ev.synchronize()
        self._check_err(handle.err_host)
        now = time.perf_counter()
        # wall time attributed to this step: from its launch (or the previous collect, if later)
        self.stats["decode_ms"] += (now - max(t0, getattr(self, "_last_collect", t0))) * 1e3
        self._last_collect = now
        self.stats["decode_steps"] += 1
        return ho[:B].tolist()

    def _launch_decode(self, Bp: int, n_copy: int) -> None:
        if self.tp_size > 1:
            self.comm.broadcast(self.d_stage[:n_copy], src=0)
        g = self.graphs.get(Bp)
        if g is not None:
            g.replay()
            self.stats["graph_replays"] += 1
        else:
            self._decode_forward(Bp)

    def padded_tokens(self, T: int) -> int:
        """Prefill steps of >= 1024 tokens run padded to a multiple of KA_PREFILL_PAD (256): hipBLASLt
        is up to ~10% faster per token on whole 256-row tiles (scripts/bench_prefill_gemm.py: M=4000
        1.31 PFLOP/s vs M=4096 1.45).  Padding rows write no KV (slot -1) and are never sampled."""
        q = self.prefill_pad
        return T if q <= 1 or T < self.prefill_pad_min else (T + q - 1) // q * q

    def _pack_prefill(self, batch: Batch, pad: bool = False, with_fix: bool = False):
        """Packed step metadata [ids | pos | slots | q_starts | ctx | mask | logits idx | block tables |
        copies (src, dst) | fixups (dst, src)].  with_fix: also returns the number of PLACEHOLDER
        fixups (flat id position, in-flight row) appended at the end (their ids are packed as the
        placeholder and replaced on the device)."""
        S = len(batch.seqs)
        T = self.padded_tokens(batch.num_tokens) if pad else batch.num_tokens
        mb = self.max_blocks
        nc = len(batch.copies)
        fix = []
        if with_fix:
            q0 = 0
            for s, nq in zip(batch.seqs, batch.num_query):
                # a placeholder is always the sequence's last token; the row covers it if it ends there
                if s.ph_row is not None and s.num_computed + nq == s.total_len:
                    fix.append((q0 + nq - 1, s.ph_row))
                q0 += nq
        nf = len(fix)
        buf = np.zeros(3 * T + (S + 1) + 3 * S + S * mb + 2 * nc + 2 * nf, dtype=np.int32)
        if nf:
            fx = np.asarray(fix, dtype=np.int32)
            buf[len(buf) - 2 * nf:len(buf) - nf] = fx[:, 0]
            buf[len(buf) - nf:] = fx[:, 1]
        if nc:   # [src... | dst...] block-copy list (sub-block prefix reuse), before the fixups
            cp = np.asarray(batch.copies, dtype=np.int32)
            e = len(buf) - 2 * nf
            buf[e - 2 * nc:e - nc] = cp[:, 0]
            buf[e - nc:e] = cp[:, 1]
        ids, pos, slots = buf[:T], buf[T:2 * T], buf[2 * T:3 * T]
        slots[batch.num_tokens:] = -1          # padding rows (if any): no cache write
        o = 3 * T
        q_starts = buf[o:o + S + 1]; o += S + 1
        ctx = buf[o:o + S]; o += S
        mask = buf[o:o + S]; o += S
        lidx = buf[o:o + S]; o += S
        bt = buf[o:o + S * mb].reshape(S, mb)
        # one Python pass collects per-sequence scalars, token slices and tables; the per-token
        # arrays are then built with a handful of vectorised numpy ops (was ~10 numpy calls per
        # sequence: ~2.7 ms of GPU-idle host time for a 256-request prefill)
        nqs = np.asarray(batch.num_query, dtype=np.int64)
        tot = np.empty(S, dtype=np.int64)
        toks: list = []
        for i, (s, nq) in enumerate(zip(batch.seqs, batch.num_query)):
            start = s.num_computed               # query = all_ids[start:n] (a chunk may end early)
            n = start + nq
            tot[i] = n
            ng = len(s.output_ids) - s.n_forced
            lp = len(s.prompt_ids)
            if start >= lp:                      # decode row (mixed step): generated tokens only
                toks.extend(s.output_ids[s.n_forced + start - lp:s.n_forced + n - lp])
            else:
                toks.extend(s.prompt_ids[start:min(n, lp)])
                if n > lp:
                    toks.extend(s.output_ids[s.n_forced:s.n_forced + n - lp])
            tbl = s.block_table
            if not tbl:   # a freed (finished) sequence: its slots would alias block 0
                raise RuntimeError(f"prefill row {i} (seq {s.seq_id}) has no KV blocks")
            bt[i, :len(tbl)] = tbl
            mask[i] = mask_index_for(ng, s.params.safe_decode)
        n_real = int(nqs.sum())
        ends = np.cumsum(nqs)
        q_starts[0] = 0
        q_starts[1:] = ends
        ctx[:] = tot
        lidx[:] = ends - 1
        ids[:n_real] = toks
        seq_of = np.repeat(np.arange(S), nqs)
        p = np.arange(n_real, dtype=np.int64) - np.repeat(ends - nqs, nqs) + np.repeat(tot - nqs, nqs)
        pos[:n_real] = p
        bs = self.block_size
        slots[:n_real] = bt[seq_of, p // bs] * bs + p % bs
        return (buf, nf) if with_fix else buf

    def _run_prefill(self, buf: torch.Tensor, T: int, S: int, max_q: int, nc: int = 0, nd: int = 0,
                     t_real: int = 0) -> torch.Tensor:
        mb = self.max_blocks
        if nc:
            n = buf.shape[0]
            ops.kv_block_copy(self.k_cache, self.v_cache, buf[n - 2 * nc:n - nc], buf[n - nc:])
        ids, pos, slots = buf[:T], buf[T:2 * T], buf[2 * T:3 * T]
        o = 3 * T
        q_starts = buf[o:o + S + 1]; o += S + 1
        ctx = buf[o:o + S]; o += S
        mask = buf[o:o + S]; o += S
        lidx = buf[o:o + S].long(); o += S
        bt = buf[o:o + S * mb].view(S, mb)
        meta = AttnMeta(positions=pos, slot_mapping=slots, block_tables=bt, ctx_lens=ctx, logits_indices=lidx,
                        is_decode=False, q_starts=q_starts, max_q_len=max_q, num_decode=nd,
                        num_tokens=t_real or T)
        h = self.model.forward(ids, meta, self.k_cache, self.v_cache)
        return self.model.sample(h, self.mask_bits, mask if self.mask_bits is not None else None)

    # ------------------------------------------------------------------------------------------
    def _bcast_header(self, kind: int, a: int = 0, b: int = 0, c: int = 0, d: int = 0, e: int = 0,
                      f: int = 0, g: int = 0) -> None:
        if self.tp_size == 1:
            return
        self.d_hdr.copy_(torch.tensor([kind, a, b, c, d, e, f, g], dtype=torch.int32))
        self.comm.broadcast(self.d_hdr, src=0)

    def _bcast_header_async(self, kind: int, *vals: int) -> None:
        """The step header from pinned memory (the copy stays asynchronous on the stream); two
        buffers: the one refilled here served the launch before last, which has been read back."""
        if self.tp_size == 1:
            return
        hh = self._h_hdrs[self._hflip]
        self._hflip ^= 1
        h = hh.numpy()
        h[:] = 0
        h[0] = kind
        h[1:1 + len(vals)] = vals
        self.d_hdr.copy_(hh, non_blocking=True)
        self.comm.broadcast(self.d_hdr, src=0)

    @torch.inference_mode()
    def execute(self, batch: Batch) -> List[int]:
        """Run one step for `batch` on every TP rank; returns the sampled token per sequence."""
        B = len(batch.seqs)
        if B == 0:
            return []
        t0 = time.perf_counter()
        if batch.is_decode and B <= self.bmax:
            i = bisect.bisect_left(self.buckets, B)
            # pad to the bucket even when running eagerly: identical shapes -> identical GEMM plans
            # and kernels as the captured graphs (graph replay == eager, token for token)
            Bp = self.buckets[i] if i < len(self.buckets) else B
            self._pack_decode(batch, Bp)
            n_copy = self._off["bt"] + Bp * self.max_blocks
            self._bcast_header(KIND_DECODE, Bp, n_copy)
            self.d_stage[:n_copy].copy_(self.h_stage[:n_copy], non_blocking=True)
            self._launch_decode(Bp, n_copy)
            self.h_out[:B].copy_(self.d_out[:B], non_blocking=True)
            eh = self._copy_err()
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            self._check_err(eh)
            out = self.h_out[:B].tolist()
            self.stats["decode_steps"] += 1
            self.stats["decode_ms"] += (time.perf_counter() - t0) * 1e3
            return out
        host = self._pack_prefill(batch, pad=True)
        T, S, max_q, nc = self.padded_tokens(batch.num_tokens), B, max(batch.num_query), len(batch.copies)
        nd = B - len(batch.prefill_seqs) if self.split_mixed_attention else 0
        self._bcast_header(KIND_PREFILL, T, S, max_q, host.shape[0], nc, nd, batch.num_tokens)
        buf = torch.from_numpy(host).to(self.device, non_blocking=False)
        if self.tp_size > 1:
            self.comm.broadcast(buf, src=0)
        tok = self._run_prefill(buf, T, S, max_q, nc, nd, batch.num_tokens)
        eh = self._copy_err()
        out = tok.cpu().tolist()
        self._check_err(eh)
        self.stats["prefill_steps"] += 1
        self.stats["prefill_tokens"] += T
        self.stats["prefill_ms"] += (time.perf_counter() - t0) * 1e3
        return out

    @torch.inference_mode()
    def worker_loop(self) -> None:
        """Non-driver TP ranks: mirror every step of rank 0 until it broadcasts STOP.  A worker whose
        one-shot collective timed out is out of step with the group: it raises (the process exits,
        its heartbeat stops, rank 0's watchdog marks the engine unhealthy).  The error word of a step
        is read after the next header arrives (that readback synchronises the stream anyway)."""
        pending = None
        while True:
            self.comm.broadcast(self.d_hdr, src=0)
            kind, a, b, c, d, e, f, g = self.d_hdr[:8].tolist()
            self._check_err(pending)
            if kind == KIND_STOP:
                return
            if kind == KIND_DECODE:
                self._launch_decode(a, b)
            elif kind == KIND_PREFILL:
                buf = torch.empty(d, dtype=torch.int32, device=self.device)
                self.comm.broadcast(buf, src=0)
                self._run_prefill(buf, a, b, c, e, f, g)
            pending = self._copy_err()

    def stop_workers(self) -> None:
        self._bcast_header(KIND_STOP)
