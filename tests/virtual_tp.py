"""Virtual tensor parallelism on ONE device (SURVEY.md §4.3 'TP numerics (1 GPU)').

RCCL refuses two ranks on one GPU, so the TP math is validated by running the t shard-models in t
threads on the same device with a `VirtualComm` whose all-reduce sums the shards' partial outputs
(barrier -> sum -> barrier -> copy back) and whose all-gather stacks them.  Because random weights
are generated in parallel-invariant units (models/weights.py), shard r holds exactly the slice of
the TP=1 weights that Megatron sharding assigns it.
"""
from __future__ import annotations

import threading
import traceback

import torch

from ai_agent_kubectl_amd.engine.runner import ModelRunner
from ai_agent_kubectl_amd.engine.scheduler import Batch
from ai_agent_kubectl_amd.engine.sequence import Sequence, SamplingParams
from ai_agent_kubectl_amd.engine.tokenizer import get_tokenizer
from ai_agent_kubectl_amd.models.llama import AttnMeta
from ai_agent_kubectl_amd.models.weights import ParallelInfo, random_weights
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM


class VirtualComm:
    def __init__(self, world: int, timeout: float = 300.0):
        self.world_size = world
        self._bar = threading.Barrier(world, timeout=timeout)   # a failing rank breaks it: no hang
        self._slots = [None] * world
        self._out = None

    def view(self, rank):
        parent = self

        class _R:
            world_size = parent.world_size

            def __init__(self):
                self.rank = rank

            def all_reduce(self, t):
                parent._slots[rank] = t
                parent._bar.wait()
                if rank == 0:
                    parent._out = torch.stack([s.float() for s in parent._slots]).sum(0)
                parent._bar.wait()
                t.copy_(parent._out.to(t.dtype))
                parent._bar.wait()
                return t

            def all_gather(self, t):
                parent._slots[rank] = t
                parent._bar.wait()
                out = torch.stack([s.clone() for s in parent._slots])
                parent._bar.wait()
                return out

            def all_to_all_single(self, t, out_splits=None, in_splits=None):
                w = parent.world_size
                in_splits = list(in_splits) if in_splits is not None else [t.shape[0] // w] * w
                parent._slots[rank] = (t, in_splits)
                parent._bar.wait()
                pieces = []
                for j in range(w):
                    tj, sj = parent._slots[j]
                    off = sum(sj[:rank])
                    pieces.append(tj[off:off + sj[rank]].clone())
                parent._bar.wait()
                return torch.cat(pieces)

            def broadcast(self, t, src=0):
                if rank == src:
                    parent._slots[src] = t
                parent._bar.wait()
                if rank != src:
                    t.copy_(parent._slots[src])
                parent._bar.wait()
                return t

            def barrier(self):
                parent._bar.wait()

            def all_reduce_rmsnorm(self, t, w, eps, residual=None):
                from ai_agent_kubectl_amd import ops
                self.all_reduce(t)
                return ops.rmsnorm(t, w, eps, residual=residual)

        return _R()


class _TinyEngine:
    """Just enough of LLMEngine for EngineLLM.prompt_ids()."""

    def __init__(self, tok):
        self.tokenizer = tok


def _batch(cfg, queries, block_size=16):
    tok = get_tokenizer(cfg.vocab_size, cfg.tokenizer)
    be = EngineLLM(_TinyEngine(tok), max_new_tokens=4)
    seqs = [Sequence(prompt_ids=be.prompt_ids(q), params=SamplingParams()) for q in queries]
    nb = 0
    for s in seqs:
        n = (s.total_len + block_size - 1) // block_size
        s.block_table = list(range(nb, nb + n))
        nb += n
    return Batch(seqs, [s.total_len for s in seqs], is_decode=False, prefill_seqs=seqs), nb


def virtual_tp_logits(cfg, tp: int, device="cuda", queries=("list all pods", "get nodes in prod")):
    batch, nb = _batch(cfg, queries)
    vc = VirtualComm(tp)
    runners = []
    for r in range(tp):
        ep = tp if cfg.is_moe else 1
        W = random_weights(cfg, ParallelInfo(r, tp, r if ep > 1 else 0, ep), seed=0, device=device)
        runners.append(ModelRunner(cfg, W, torch.device(device), num_blocks=nb + 4, max_model_len=512,
                                   graph_buckets=(1,), comm=vc.view(r), tp_rank=r, tp_size=tp,
                                   ep_rank=r if ep > 1 else 0, ep_size=ep, use_graphs=False))
    results = [None] * tp

    def run(r):
        rn = runners[r]
        host = torch.from_numpy(rn._pack_prefill(batch)).to(device)
        T, S = batch.num_tokens, len(batch.seqs)
        mb = rn.max_blocks
        o = 3 * T
        meta = AttnMeta(positions=host[T:2 * T], slot_mapping=host[2 * T:3 * T],
                        block_tables=host[o + 4 * S + 1:o + 4 * S + 1 + S * mb].view(S, mb),
                        ctx_lens=host[o + S + 1:o + 2 * S + 1],
                        logits_indices=host[o + 3 * S + 1:o + 4 * S + 1].long(), is_decode=False,
                        q_starts=host[o:o + S + 1], max_q_len=max(batch.num_query))
        with torch.inference_mode():
            h = rn.model.forward(host[:T], meta, rn.k_cache, rn.v_cache)
            results[r] = rn.model.logits(h)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(tp)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    return torch.cat(results, dim=-1)


def virtual_tp_generate(model: str, tp: int, queries, max_new_tokens: int = 6, device: str = "cuda"):
    """Greedy generation through the real TP engine code on ONE device: `tp` threads, each a full
    TP rank (build_engine with tp_rank / tp_size: sharded weights, KV heads and vocab), rank 0 the
    driver (scheduler + metadata broadcast, LLMEngine.generate_blocking) and the others in
    `ModelRunner.worker_loop()` — the multi-process protocol with VirtualComm as the transport.
    Eager steps (the host-side VirtualComm cannot be captured).  Returns rank 0's output ids."""
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.sequence import SamplingParams
    vc = VirtualComm(tp)
    out, errs = {}, []

    def run(r):
        try:
            eng = build_engine(EngineOptions(model=model, device=device, tp_rank=r, tp_size=tp, ep_size=tp,
                                             max_batch=4, graph_buckets=(1, 2, 4), kv_cache_tokens=4096,
                                             max_model_len=256, use_graphs=False), comm=vc.view(r))
            if r != 0:
                eng.runner.worker_loop()
                return
            be = EngineLLM(eng, max_new_tokens=max_new_tokens, ignore_eos=True)
            params = SamplingParams(max_new_tokens=max_new_tokens, ignore_eos=True)
            seqs = eng.generate_blocking([be.prompt_ids(q) for q in queries], params, forced_prefix=be._forced)
            eng.runner.stop_workers()
            out["ids"] = [s.output_ids for s in seqs]
        except Exception:
            errs.append(traceback.format_exc())
            vc._bar.abort()

    threads = [threading.Thread(target=run, args=(r,)) for r in range(tp)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errs:
        raise RuntimeError(errs[0])
    return out["ids"]


@torch.inference_mode()
def next_token_logits(eng, ids):
    """Logits of the token after `ids` from `eng`'s model (one prefill of the whole sequence)."""
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    r = eng.runner
    seq = Sequence(prompt_ids=list(ids), params=SamplingParams())
    seq.block_table, _, seq.block_hashes = eng.bm.allocate_prompt(seq.all_ids)
    try:
        batch = Batch([seq], [seq.total_len], is_decode=False, prefill_seqs=[seq])
        host = torch.from_numpy(r._pack_prefill(batch)).to(r.device)
        T, S, mb = batch.num_tokens, 1, r.max_blocks
        o = 3 * T
        meta = AttnMeta(positions=host[T:2 * T], slot_mapping=host[2 * T:3 * T],
                        block_tables=host[o + 4 * S + 1:o + 4 * S + 1 + S * mb].view(S, mb),
                        ctx_lens=host[o + S + 1:o + 2 * S + 1], logits_indices=host[o + 3 * S + 1:o + 4 * S + 1].long(),
                        is_decode=False, q_starts=host[o:o + S + 1], max_q_len=T)
        h = r.model.forward(host[:T], meta, r.k_cache, r.v_cache)
        return r.model.logits(h)[0].float()
    finally:
        eng.bm.free_table(seq.block_table)


def assert_same_or_near_tie(eng_ref, prompts, want, got, rel=0.01, abs_tol=0.05):
    """Greedy outputs of two numerically different but equivalent runs (TP = 1 vs TP = t in bf16):
    identical, or the first token where they part is a near-tie of the reference model — its
    logits for the two candidates (teacher-forced on the shared prefix) differ by less than
    rel * |logit| + abs_tol.  Anything else is a real divergence."""
    for p, w, g in zip(prompts, want, got):
        if w == g:
            continue
        k = next(i for i in range(min(len(w), len(g))) if w[i] != g[i])
        lg = next_token_logits(eng_ref, list(p) + list(w[:k]))
        lw, lgot = lg[w[k]].item(), lg[g[k]].item()
        assert lw - lgot <= rel * abs(lw) + abs_tol, (k, w[k], g[k], lw, lgot)
