"""Assemble an engine (tokenizer, weights, KV pool, runner, scheduler) from `Settings`.

KV sizing for 288 GB HBM3E per MI355X: after the weights (16 GB for Llama-3-8B bf16, 17.6 GB per
GPU for 70B at TP=8) the pool gets `GPU_MEM_FRACTION` of what is left, capped by
`KV_CACHE_TOKENS` (default 1M tokens = 128 GiB for 8B), so batch size is never KV-limited for this
workload.
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch

from ..models.config import get_config
from ..models.weights import ParallelInfo, build_weights
from .engine import LLMEngine
from .runner import ModelRunner
from .safe_decode import build_masks
from .tokenizer import get_tokenizer, tokenizer_path

logger = logging.getLogger("app.engine")


@dataclass
class EngineOptions:
    model: str = "llama3-8b"
    weights: str = "random:0"
    device: str = "cuda"
    tp_rank: int = 0
    tp_size: int = 1
    ep_size: int = 1
    max_batch: int = 256
    max_batched_tokens: int = 0          # 0: the model's default_step_tokens()
    max_model_len: int = 8192      # Llama-3's context; long prompts prefill in chunks
    block_size: int = 16
    kv_cache_tokens: int = 1 << 18  # <= 0: every byte of the GPU_MEM_FRACTION budget
    gpu_mem_fraction: float = 0.90
    graph_buckets: tuple = (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 192, 256)
    use_graphs: bool = True
    safe_decode: bool = True
    ignore_eos: bool = False
    prefix_caching: bool = True

    @classmethod
    def from_settings(cls, s) -> "EngineOptions":
        return cls(model=s.MODEL, weights=s.WEIGHTS, tp_size=s.TP, ep_size=s.EP, max_batch=s.MAX_BATCH,
                   max_batched_tokens=s.MAX_NUM_BATCHED_TOKENS, block_size=s.KV_BLOCK_SIZE,
                   gpu_mem_fraction=s.GPU_MEM_FRACTION,
                   graph_buckets=tuple(b for b in s.graph_buckets() if b <= s.MAX_BATCH) or (1,),
                   safe_decode=s.SAFE_DECODE, ignore_eos=s.IGNORE_EOS, prefix_caching=s.PREFIX_CACHING,
                   kv_cache_tokens=int(os.environ.get("KV_CACHE_TOKENS", 0)),
                   max_model_len=int(os.environ.get("MAX_MODEL_LEN", 8192)),
                   device="cuda" if torch.cuda.is_available() else "cpu")


def build_engine(opts: EngineOptions, comm=None, metrics=None) -> LLMEngine:
    t0 = time.perf_counter()
    cfg = get_config(opts.model)
    tok = get_tokenizer(cfg.vocab_size, cfg.tokenizer, tokenizer_path(opts.weights))
    dev = torch.device(opts.device)
    if dev.type == "cuda":
        from ..ops._hip import require
        require()  # fail loudly: the GPU path never runs without the HIP kernels
        torch.cuda.set_device(dev.index if dev.index is not None else torch.cuda.current_device())
    dtype = torch.bfloat16
    # MoE: experts are sharded over the tensor-parallel group (EP = TP); the all-reduce after the
    # MoE block is the expert combine.  EP is therefore derived, not free (EP=1 with TP>1 would
    # replicate experts and double-count them in that all-reduce).
    ep_size = opts.tp_size if cfg.is_moe else 1
    if cfg.is_moe and opts.ep_size not in (1, opts.tp_size):
        raise ValueError("EP must equal TP (experts are sharded over the tensor-parallel group)")
    par = ParallelInfo(opts.tp_rank, opts.tp_size, opts.tp_rank if ep_size > 1 else 0, ep_size)
    weights = build_weights(opts.weights, cfg, par, device=dev, dtype=dtype)
    # ---- KV pool size ----
    per_block = cfg.num_layers * 2 * (cfg.num_kv_heads // opts.tp_size) * cfg.head_dim * opts.block_size * 2
    # KV_CACHE_TOKENS of pooled KV (not max_batch x max_model_len: with an 8192-token context that
    # would be 2M tokens); at least one full-length sequence fits, the rest is preemption's job.
    # The serving default (KV_CACHE_TOKENS unset / 0) takes the whole GPU_MEM_FRACTION budget left
    # after the weights: ~1.8M tokens of Llama-3-8B KV on a 288 GB MI355X.
    min_blocks = opts.max_model_len // opts.block_size + 1
    if dev.type == "cuda":
        free, _total = torch.cuda.mem_get_info(dev)
        # KA_GPU_MEM_SHARE: this engine's share of the device when several replicas / ranks are
        # placed on one GPU (parallel/dp.py sets it), so they do not all size their pool from the
        # same free-memory reading
        share = float(os.environ.get("KA_GPU_MEM_SHARE", "1"))
        budget = int(free * opts.gpu_mem_fraction * share) - int((4 << 30) * share)   # activations / graphs
        fit = min(max(budget, 0) // per_block, 1 << 20)   # (16M tokens: more than any batch here can hold)
        want_blocks = max(opts.kv_cache_tokens // opts.block_size, min_blocks) if opts.kv_cache_tokens > 0 else fit
        num_blocks = min(want_blocks, fit)
        if num_blocks < min_blocks:
            raise RuntimeError(f"KV pool of {num_blocks} blocks cannot hold one {opts.max_model_len}-token sequence "
                               f"({min_blocks} blocks): {free / 2**30:.1f} GiB free x GPU_MEM_FRACTION "
                               f"{opts.gpu_mem_fraction} x share {share:g}; lower MAX_MODEL_LEN or free the device")
    else:
        want = opts.kv_cache_tokens // opts.block_size if opts.kv_cache_tokens > 0 else 4096
        num_blocks = min(max(want, min_blocks), 4096)
    masks = build_masks(tok, allow_eos=not opts.ignore_eos) if opts.safe_decode else None
    if comm is not None and opts.tp_size > 1:
        from ..parallel.custom_allreduce import maybe_enable
        maybe_enable(comm, dev)   # KA_CUSTOM_AR=1: one-shot all-reduce for the small decode messages
    runner = ModelRunner(cfg, weights, dev, num_blocks=num_blocks, block_size=opts.block_size,
                         max_model_len=opts.max_model_len, graph_buckets=opts.graph_buckets, mask_bits=masks,
                         comm=comm, tp_rank=opts.tp_rank, tp_size=opts.tp_size, ep_rank=par.ep_rank,
                         ep_size=ep_size, use_graphs=opts.use_graphs)
    step_tokens = opts.max_batched_tokens if opts.max_batched_tokens > 0 else cfg.default_step_tokens()
    eng = LLMEngine(runner, tok, max_batch=opts.max_batch, max_batched_tokens=step_tokens,
                    max_model_len=opts.max_model_len, prefix_caching=opts.prefix_caching, metrics=metrics)
    eng.options = opts
    if comm is not None and opts.tp_size > 1:
        _attach_liveness(eng, opts)
    eng.build_seconds = time.perf_counter() - t0
    logger.info("engine built: model=%s tp=%d blocks=%d (%.1f GiB KV) in %.1fs", cfg.name, opts.tp_size,
                num_blocks, num_blocks * per_block / 2**30, eng.build_seconds)
    return eng


def _attach_liveness(eng: LLMEngine, opts: EngineOptions) -> None:
    """TP/EP > 1: workers beat into the rendezvous store, rank 0 watches (parallel/watchdog.py)."""
    from ..parallel.watchdog import Heartbeat, Watchdog, default_store

    store = default_store()
    if store is None:
        return
    interval = float(os.environ.get("WORKER_HEARTBEAT_INTERVAL_S", "1"))
    if opts.tp_rank != 0:
        eng.heartbeat = Heartbeat(store, opts.tp_rank, interval).start()
        return
    eng.watchdog = Watchdog(store, range(1, opts.tp_size), eng.mark_unhealthy,
                            hb_timeout=float(os.environ.get("WORKER_HEARTBEAT_TIMEOUT_S", "30")),
                            step_timeout=float(os.environ.get("ENGINE_STEP_TIMEOUT_S", "120")),
                            interval=interval, step_started=lambda: eng.step_t0)
