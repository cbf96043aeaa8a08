"""Model / engine numerics on the GPU (SURVEY.md §4.3 'model (GPU)' and 'TP numerics' rows).

* full forward (real Llama-3-8B layer geometry, 2 layers) through the HIP kernels vs the same
  weights through the fp32 torch references;
* hipGraph decode replay == eager decode, token for token;
* prefix-cache hit == cold prefill (same tokens);
* virtual TP: t shard-forwards summed in place of the all-reduce == TP=1 logits;
* Mixtral (2 layers, 8 experts) HIP path vs reference.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.engine.sequence import SamplingParams  # noqa: E402
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM  # noqa: E402

QUERIES = ["list all pods", "show services in namespace prod", "scale web to 3 replicas",
           "get nodes with labels", "describe deployment api", "logs of pod api-1"]


def _engine(model, graphs, buckets=(1, 2, 4, 8), max_batch=8, kv_cache_tokens=16384, comm=None, **kw):
    opts = EngineOptions(model=model, device="cuda", max_batch=max_batch, graph_buckets=buckets,
                         kv_cache_tokens=kv_cache_tokens, max_model_len=512, use_graphs=graphs, **kw)
    eng = build_engine(opts, comm=comm) if comm is not None else build_engine(opts)
    if graphs:
        eng.runner.capture_graphs()
    return eng


def _prefill_hidden(eng, be, queries):
    """Run one prefill step and return the runner's sampled tokens plus the last hidden states."""
    from ai_agent_kubectl_amd.engine.scheduler import Batch
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    seqs = [Sequence(prompt_ids=be.prompt_ids(q), params=be.params) for q in queries]
    for s in seqs:
        s.block_table, _, s.block_hashes = eng.bm.allocate_prompt(s.all_ids)
    batch = Batch(seqs, [s.total_len for s in seqs], is_decode=False, prefill_seqs=seqs)
    r = eng.runner
    host = torch.from_numpy(r._pack_prefill(batch)).cuda()
    T, S = batch.num_tokens, len(seqs)
    from ai_agent_kubectl_amd.models.llama import AttnMeta
    mb = r.max_blocks
    o = 3 * T
    meta = AttnMeta(positions=host[T:2 * T], slot_mapping=host[2 * T:3 * T],
                    block_tables=host[o + 4 * S + 1:o + 4 * S + 1 + S * mb].view(S, mb),
                    ctx_lens=host[o + S + 1:o + 2 * S + 1], logits_indices=host[o + 3 * S + 1:o + 4 * S + 1].long(),
                    is_decode=False, q_starts=host[o:o + S + 1], max_q_len=max(batch.num_query))
    h = r.model.forward(host[:T], meta, r.k_cache, r.v_cache)
    for s in seqs:
        eng.bm.free_table(s.block_table)
    return h


def test_llama_forward_hip_vs_reference():
    eng = _engine("llama3-8b-2l", graphs=False)
    be = EngineLLM(eng, max_new_tokens=8)
    with torch.inference_mode():
        h_hip = _prefill_hidden(eng, be, QUERIES[:3])
        with ops.force_reference():
            h_ref = _prefill_hidden(eng, be, QUERIES[:3])
        lg_hip = eng.runner.model.logits(h_hip).float()
        lg_ref = eng.runner.model.logits(h_ref).float()
    cos = torch.nn.functional.cosine_similarity(lg_hip, lg_ref, dim=-1)
    assert cos.min().item() > 0.995, cos
    torch.testing.assert_close(h_hip.float(), h_ref.float(), atol=0.1, rtol=0.05)


def test_llama_forward_hip_vs_reference_large_prefill():
    """A prefill step of >= 1024 rows — the shape class of the bench's mixed steps — through the
    prefill kernels the engine dispatches there (csrc/gemm_big.hip: QKV / O / down with the split
    tail, gate_up with the SwiGLU epilogue; the 16-token RoPE + KV window kernel; the varlen
    prefill attention) vs the same weights through the fp32 torch references."""
    eng = _engine("llama3-8b-2l", graphs=False, max_batch=16, kv_cache_tokens=32768)
    be = EngineLLM(eng, max_new_tokens=8)
    queries = [f"{q} in namespace team-{i} sorted by creation time" for i, q in enumerate(QUERIES * 2)]
    n_rows = sum(len(be.prompt_ids(q)) for q in queries)
    assert n_rows >= 1024, n_rows
    x = torch.zeros(n_rows, 4096, device="cuda", dtype=torch.bfloat16)
    assert ops.use_prefill_swiglu(x, eng.runner.model.layers[0]["w13"])
    assert ops.big_gemm_ok(x, eng.runner.model.layers[0]["wqkv"])
    with torch.inference_mode():
        h_hip = _prefill_hidden(eng, be, queries)
        with ops.force_reference():
            h_ref = _prefill_hidden(eng, be, queries)
        lg_hip = eng.runner.model.logits(h_hip).float()
        lg_ref = eng.runner.model.logits(h_ref).float()
    cos = torch.nn.functional.cosine_similarity(lg_hip, lg_ref, dim=-1)
    assert cos.min().item() > 0.995, cos
    torch.testing.assert_close(h_hip.float(), h_ref.float(), atol=0.1, rtol=0.05)
    # the same step with QKV / O / down on gemm_big as well (KA_PREFILL_GEMM=big)
    saved, ops.PREFILL_GEMM = ops.PREFILL_GEMM, "big"
    try:
        assert ops.use_big_gemm(x, eng.runner.model.layers[0]["wqkv"])
        with torch.inference_mode():
            h_big = _prefill_hidden(eng, be, queries)
    finally:
        ops.PREFILL_GEMM = saved
    torch.testing.assert_close(h_big.float(), h_ref.float(), atol=0.1, rtol=0.05)


@pytest.mark.parametrize("B", [1, 4, 8, 16, 256])
def test_decode_chain_vs_fp32_reference(B):
    """The real decode chain — autotuned GEMM plan (gemm_mfma kernels at M = 256 with bf16 split-K
    partials reduced inside the fused RoPE + KV-append + attention kernel and inside the fused
    residual + RMSNorm, GEMV / skinny kernels at M = 1 / 4), the fused decode attention, the LM
    head — over 8 decode steps, each step against the same forward through the fp32 torch
    references (`ops.force_reference`: fp32 GEMMs, reference attention / RoPE / norms) on a copy
    of the same KV cache.  Hidden states and logits to bf16 tolerance; the same step with fp32
    split-K partials (KA_BF16_PARTIALS=0, KA_BF16_QKV_PARTIALS=0) gives the error the bf16
    partials are compared against."""
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    from ai_agent_kubectl_amd.models.llama import AttnMeta
    eng = _engine("llama3-8b-2l", graphs=True, buckets=(1, 4, 8, 16, 256), max_batch=256, kv_cache_tokens=65536)
    be = EngineLLM(eng, max_new_tokens=40, ignore_eos=True)
    params = SamplingParams(max_new_tokens=40, ignore_eos=True)
    sch, r = eng.scheduler, eng.runner
    sch.prefill_max_wait_s = 0.0
    sch.gather_max_s = 0.0
    sch.hold_steps = 0
    if B >= 48:   # the gemm_mfma plans (and their bf16 partials) are what runs at this size
        assert any(v[0] == "gm" for (m, _, _), v in ops.GEMM_PLAN.items() if m == B), ops.GEMM_PLAN
    with torch.inference_mode():
        for i in range(B):
            sch.add(Sequence(prompt_ids=be.prompt_ids(QUERIES[i % len(QUERIES)] + f" #{i}"), params=params,
                             forced_prefix=list(be._forced)))
        while sch.waiting:
            b = sch.schedule()
            eng._apply(b, r.execute(b))
            sch.on_step_done(b)
        assert len(sch.running) == B
        worst = 1.0
        errs = {True: 0.0, False: 0.0}
        m = r.model
        flags = (m.bf16_partials, m.bf16_qkv_partials)
        for step in range(8):
            batch = sch.schedule()
            assert batch.is_decode and len(batch.seqs) == B
            Bp = r.buckets[r.buckets.index(B)]
            r._pack_decode(batch, Bp)
            n = r._off["bt"] + Bp * r.max_blocks
            r.d_stage[:n].copy_(r.h_stage[:n])
            meta = AttnMeta(positions=r._view("pos", Bp), slot_mapping=r._view("slots", Bp),
                            block_tables=r._view("bt", Bp), ctx_lens=r._view("ctx", Bp),
                            logits_indices=r.d_logits_idx[:Bp], is_decode=True)
            ids = r._view("ids", Bp)
            kc, vc = r.k_cache.clone(), r.v_cache.clone()
            k32, v32 = r.k_cache.clone(), r.v_cache.clone()
            h = r.model.forward(ids, meta, r.k_cache, r.v_cache)
            lg = r.model.logits(h).float()
            with ops.force_reference():
                h_ref = r.model.forward(ids, meta, kc, vc)
                lg_ref = r.model.logits(h_ref).float()
            m.bf16_partials = m.bf16_qkv_partials = False
            try:
                lg32 = m.logits(m.forward(ids, meta, k32, v32)).float()
            finally:
                m.bf16_partials, m.bf16_qkv_partials = flags
            errs[True] = max(errs[True], (lg[:B] - lg_ref[:B]).abs().max().item())
            errs[False] = max(errs[False], (lg32[:B] - lg_ref[:B]).abs().max().item())
            del k32, v32
            cos = torch.nn.functional.cosine_similarity(lg[:B], lg_ref[:B], dim=-1)
            worst = min(worst, cos.min().item())
            assert cos.min().item() > 0.995, (step, cos.min().item())
            torch.testing.assert_close(h[:B].float(), h_ref[:B].float(), atol=0.1, rtol=0.05)
            torch.testing.assert_close(lg[:B], lg_ref[:B], atol=0.15, rtol=0.05)
            del kc, vc
            mask = r._view("mask", Bp) if r.mask_bits is not None else None
            tok = r.model.sample(h, r.mask_bits, mask)[:B].tolist()
            eng._apply(batch, tok)
            sch.on_step_done(batch)
    print(f"B={B}: worst logits cosine over 8 steps {worst:.5f}; max |logit - fp32 ref|: bf16 partials "
          f"{errs[True]:.4f}, fp32 partials {errs[False]:.4f}")
    assert errs[True] <= 2 * errs[False] + 0.05, errs


@pytest.mark.parametrize("B", [1, 4, 64])
def test_decode_trajectory_independent_fp32_kv(B):
    """An independent fp32 trajectory: the reference KV cache is written only by the fp32
    reference path, from the prefill on (prefix caching off, so no block is shared), and both paths
    are fed the tokens the HIP path samples (teacher forcing keeps them aligned) for 24 decode steps.
    Unlike test_decode_chain_vs_fp32_reference (which re-bases the reference on the HIP path's cache
    every step) this sees KV drift accumulate: every step's logits stay within bf16 tolerance of
    the fp32 trajectory and the error of the last 8 steps is not a growing multiple of the first 8's."""
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    from ai_agent_kubectl_amd.models.llama import AttnMeta
    eng = _engine("llama3-8b-2l", graphs=False, buckets=(1, 4, 64), max_batch=64, kv_cache_tokens=32768,
                  prefix_caching=False, max_batched_tokens=16384)
    be = EngineLLM(eng, max_new_tokens=40, ignore_eos=True)
    params = SamplingParams(max_new_tokens=40, ignore_eos=True)
    sch, r = eng.scheduler, eng.runner
    sch.prefill_max_wait_s = 0.0
    sch.gather_max_s = 0.0
    sch.hold_steps = 0
    m = r.model
    kc_ref, vc_ref = torch.zeros_like(r.k_cache), torch.zeros_like(r.v_cache)
    errs, coss = [], []
    with torch.inference_mode():
        for i in range(B):
            sch.add(Sequence(prompt_ids=be.prompt_ids(QUERIES[i % len(QUERIES)] + f" #{i}"), params=params))
        b = sch.schedule()
        assert not b.is_decode and len(b.seqs) == B and not b.copies
        host = torch.from_numpy(r._pack_prefill(b)).cuda()
        T, S, mb = b.num_tokens, B, r.max_blocks
        o = 3 * T
        meta = AttnMeta(positions=host[T:2 * T], slot_mapping=host[2 * T:3 * T],
                        block_tables=host[o + 4 * S + 1:o + 4 * S + 1 + S * mb].view(S, mb),
                        ctx_lens=host[o + S + 1:o + 2 * S + 1], logits_indices=host[o + 3 * S + 1:o + 4 * S + 1].long(),
                        is_decode=False, q_starts=host[o:o + S + 1], max_q_len=max(b.num_query))
        mask = host[o + 2 * S + 1:o + 3 * S + 1]
        h = m.forward(host[:T], meta, r.k_cache, r.v_cache)
        with ops.force_reference():
            h_ref = m.forward(host[:T], meta, kc_ref, vc_ref)
        coss.append(torch.nn.functional.cosine_similarity(m.logits(h).float(), m.logits(h_ref).float(), dim=-1).min().item())
        tok = m.sample(h, r.mask_bits, mask if r.mask_bits is not None else None).tolist()
        eng._apply(b, tok)
        sch.on_step_done(b)
        for step in range(24):
            batch = sch.schedule()
            assert batch.is_decode and len(batch.seqs) == B
            r._pack_decode(batch, B)
            n = r._off["bt"] + B * r.max_blocks
            r.d_stage[:n].copy_(r.h_stage[:n])
            meta = AttnMeta(positions=r._view("pos", B), slot_mapping=r._view("slots", B),
                            block_tables=r._view("bt", B), ctx_lens=r._view("ctx", B),
                            logits_indices=r.d_logits_idx[:B], is_decode=True)
            ids = r._view("ids", B)
            h = m.forward(ids, meta, r.k_cache, r.v_cache)
            lg = m.logits(h).float()[:B]
            with ops.force_reference():
                lg_ref = m.logits(m.forward(ids, meta, kc_ref, vc_ref)).float()[:B]
            errs.append((lg - lg_ref).abs().max().item())
            coss.append(torch.nn.functional.cosine_similarity(lg, lg_ref, dim=-1).min().item())
            mask = r._view("mask", B) if r.mask_bits is not None else None
            eng._apply(batch, m.sample(h, r.mask_bits, mask)[:B].tolist())
            sch.on_step_done(batch)
    print(f"B={B}: logits cosine min {min(coss):.5f}; max |logit - fp32 trajectory| first 8 steps "
          f"{max(errs[:8]):.4f}, last 8 {max(errs[-8:]):.4f}")
    assert min(coss) > 0.99, coss
    assert max(errs) < 0.3, errs
    assert max(errs[-8:]) <= 2 * max(errs[:8]) + 0.05, errs


def test_graph_decode_equals_eager():
    params = SamplingParams(max_new_tokens=12, ignore_eos=True)
    outs = []
    # graphs first: capture autotunes the global GEMM plan, which the eager run then reuses, so
    # both runs use identical kernels and the comparison isolates graph replay vs eager launch
    for graphs in (True, False):
        eng = _engine("llama3-8b-2l", graphs=graphs)
        be = EngineLLM(eng, max_new_tokens=12, ignore_eos=True)
        seqs = eng.generate_blocking([be.prompt_ids(q) for q in QUERIES[:5]], params, forced_prefix=be._forced)
        outs.append([s.output_ids for s in seqs])
        if graphs:
            assert eng.runner.stats["graph_replays"] > 0
        del eng
        torch.cuda.empty_cache()
    assert outs[0] == outs[1]


def test_lookahead_matches_sync_gpu():
    """Threaded engine on the GPU (hipGraph decode, chunked prompts, rows of different lengths):
    with lookahead — steps queued ahead of the readback from pinned staging, placeholder inputs
    gathered on the device from the in-flight step's samples, progress events — the tokens equal
    those of the engine without it."""
    import threading
    eng = _engine("llama3-8b-2l", graphs=True)
    be = EngineLLM(eng, max_new_tokens=12, ignore_eos=True)
    prompts = [be.prompt_ids(q) for q in QUERIES]
    lens = [3, 12, 6, 9, 2, 7]
    sch = eng.scheduler
    sch.max_batched_tokens, sch.min_chunk = 64, 8   # prompts prefilled in chunks, mixed steps

    def run(lookahead):
        eng.lookahead = lookahead
        eng.bm.reset_prefix_cache()
        done, ev = {}, threading.Event()

        def cb(seq):
            done[seq.seq_id] = seq
            if len(done) == len(prompts):
                ev.set()

        eng.start()
        try:
            seqs = [eng.submit(p, SamplingParams(max_new_tokens=n, ignore_eos=True), cb, forced_prefix=be._forced)
                    for p, n in zip(prompts, lens)]
            assert ev.wait(120)
        finally:
            eng.shutdown()
        return [list(s.output_ids) for s in seqs]

    off = run(False)
    n0 = eng.lookahead_steps
    on = run(True)
    assert eng.lookahead_steps > n0
    assert on == off
    assert [len(o) - len(be._forced) for o in on] == lens
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_long_context_chunked_prefill_matches_whole():
    """A ~5k-token prompt (MAX_MODEL_LEN 8192) prefilled in 1024-token chunks over several mixed
    steps — each chunk's attention reads the previous chunks from the paged cache — against the
    whole prompt in one step: last-position logits to bf16 tolerance, greedy tokens identical or
    parting only at a near-tie (the two runs sum attention over different query tilings)."""
    from tests.virtual_tp import assert_same_or_near_tie
    eng = build_engine(EngineOptions(model="llama3-8b-2l", device="cuda", max_batch=4, graph_buckets=(1, 2),
                                     kv_cache_tokens=32768, max_model_len=8192, max_batched_tokens=8192))
    be = EngineLLM(eng, max_new_tokens=6, ignore_eos=True)
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    long_q = " ".join(f"pod-{i} in namespace team-{i % 17} restarted" for i in range(320))
    prompt = be.prompt_ids(long_q)
    assert 4000 < len(prompt) < 8000, len(prompt)
    outs = {}
    for budget in (8192, 1024):
        eng.scheduler.max_batched_tokens = budget
        eng.bm.reset_prefix_cache()
        steps0 = eng.runner.stats["prefill_steps"]
        outs[budget] = eng.generate_blocking([prompt], params, forced_prefix=be._forced)[0].output_ids
        n_prefill = eng.runner.stats["prefill_steps"] - steps0
        assert n_prefill == -(-(len(prompt) + len(be._forced)) // budget), n_prefill
    assert_same_or_near_tie(eng, [prompt], [outs[8192]], [outs[1024]])


def test_prefix_cache_hit_matches_cold():
    params = SamplingParams(max_new_tokens=8, ignore_eos=True)
    eng = _engine("llama3-8b-2l", graphs=True)
    be = EngineLLM(eng, max_new_tokens=8, ignore_eos=True)
    cold = eng.generate_blocking([be.prompt_ids(QUERIES[0])], params, forced_prefix=be._forced)[0]
    assert cold.num_cached_prompt == 0
    warm = eng.generate_blocking([be.prompt_ids(QUERIES[0])], params, forced_prefix=be._forced)[0]
    assert warm.num_cached_prompt >= 64
    assert warm.output_ids == cold.output_ids


def test_last_layer_pruning_hidden_matches_full_gpu():
    """Prefill with the last layer continued on the last-token rows only (one-query HIP decode
    attention over the just-appended keys, then O / norm / MLP on S rows) gives the final hidden rows
    of the full forward (prefill attention over every row) to bf16 tolerance; on a ~1.3k-token step
    the gate_up of the other layers takes the gemm_big SwiGLU path."""
    eng = _engine("llama3-8b-2l", graphs=False, max_batch=64, kv_cache_tokens=32768,
                  prefix_caching=False, max_batched_tokens=16384)
    be = EngineLLM(eng, max_new_tokens=4)
    m = eng.runner.model
    queries = [q + f" #{i}" for i in range(12) for q in QUERIES[:1]]
    hs = {}
    with torch.inference_mode():
        for prune in (False, True):
            m.prune_last_layer = prune
            hs[prune] = _prefill_hidden(eng, be, queries).float()
    m.prune_last_layer = True
    assert hs[True].shape == hs[False].shape == (len(queries), m.W["embed"].shape[1])
    torch.testing.assert_close(hs[True], hs[False], atol=0.05, rtol=0.05)


def test_mixed_step_split_attention_hidden_matches_unsplit():
    """One real mixed step (2 decode rows + 1 prompt): the forward with decode rows through the
    decode kernel equals the forward with every row through the varlen prefill kernel (hidden
    states to bf16 tolerance; greedy tokens over many steps would also compare argmax near-ties)."""
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    from ai_agent_kubectl_amd.models.llama import AttnMeta
    eng = _engine("llama3-8b-2l", graphs=False)
    be = EngineLLM(eng, max_new_tokens=8, ignore_eos=True)
    params = SamplingParams(max_new_tokens=8, ignore_eos=True)
    sch, r = eng.scheduler, eng.runner
    sch.prefill_max_wait_s = 0.0
    sch.gather_max_s = 0.0
    sch.hold_steps = 0
    with torch.inference_mode():
        first = [Sequence(prompt_ids=be.prompt_ids(q), params=params, forced_prefix=list(be._forced))
                 for q in QUERIES[:2]]
        for q in first:
            sch.add(q)
        b = sch.schedule()
        eng._apply(b, r.execute(b))
        sch.on_step_done(b)
        sch.add(Sequence(prompt_ids=be.prompt_ids(QUERIES[2]), params=params, forced_prefix=list(be._forced)))
        batch = sch.schedule()
        nd = len(batch.seqs) - len(batch.prefill_seqs)
        assert nd == 2 and len(batch.prefill_seqs) == 1
        host = torch.from_numpy(r._pack_prefill(batch)).cuda()
        T, S, mb = batch.num_tokens, len(batch.seqs), r.max_blocks
        o = 3 * T
        hs = []
        for split_nd in (0, nd):
            meta = AttnMeta(positions=host[T:2 * T], slot_mapping=host[2 * T:3 * T],
                            block_tables=host[o + 4 * S + 1:o + 4 * S + 1 + S * mb].view(S, mb),
                            ctx_lens=host[o + S + 1:o + 2 * S + 1], logits_indices=host[o + 3 * S + 1:o + 4 * S + 1].long(),
                            is_decode=False, q_starts=host[o:o + S + 1], max_q_len=max(batch.num_query),
                            num_decode=split_nd)
            hs.append(r.model.forward(host[:T], meta, r.k_cache, r.v_cache).float())
    torch.testing.assert_close(hs[1], hs[0], atol=0.08, rtol=0.05)
    cos = torch.nn.functional.cosine_similarity(hs[1], hs[0], dim=-1)
    assert cos.min().item() > 0.999, cos


def test_safe_decode_outputs_pass_validator():
    from ai_agent_kubectl_amd.safety import is_safe_kubectl_command
    eng = _engine("llama3-8b-2l", graphs=True)
    be = EngineLLM(eng, max_new_tokens=16)
    seqs = eng.generate_blocking([be.prompt_ids(q) for q in QUERIES], be.params, forced_prefix=be._forced)
    for s in seqs:
        txt = be.tok.decode([t for t in s.output_ids if not be.tok.is_eos(t)])
        assert is_safe_kubectl_command(txt), txt


def test_virtual_tp_matches_tp1():
    """TP=2 shards run sequentially on one GPU with partial sums standing in for the all-reduce."""
    from ai_agent_kubectl_amd.models.config import get_config
    from ai_agent_kubectl_amd.models.llama import LlamaModel
    from ai_agent_kubectl_amd.models.weights import ParallelInfo, random_weights
    from tests.virtual_tp import virtual_tp_logits
    cfg = get_config("llama3-8b-2l")
    full = virtual_tp_logits(cfg, tp=1)
    tp2 = virtual_tp_logits(cfg, tp=2)
    cos = torch.nn.functional.cosine_similarity(full.float(), tp2.float(), dim=-1)
    assert cos.min().item() > 0.999


@pytest.mark.parametrize("model,tp", [("llama3-70b-2l", 4), ("llama3-70b-2l", 8), ("mixtral-2l", 8)])
def test_virtual_tp_spec_geometry_tokens_match_tp1(model, tp):
    """TP = 4 / 8 at Llama-3-70B geometry (64 q / 8 kv heads: 1 KV head and 8 q heads per rank at
    TP = 8, GQA group 8 in the HIP attention kernels) and EP = 8 for Mixtral (one expert per rank,
    all-to-all prefill dispatch): the real driver / worker TP engine code, one rank per thread on
    this GPU, generates the same greedy tokens as TP = 1 (SURVEY.md §4.3 'TP numerics (1 GPU)')."""
    from tests.virtual_tp import assert_same_or_near_tie, virtual_tp_generate
    qs = QUERIES[:3]
    ref = virtual_tp_generate(model, 1, qs)
    got = virtual_tp_generate(model, tp, qs)
    torch.cuda.empty_cache()
    if got != ref:   # bf16 partial sums: only a near-tie of the TP = 1 logits may flip a token
        eng = _engine(model, graphs=False)
        be = EngineLLM(eng, max_new_tokens=6, ignore_eos=True)
        assert_same_or_near_tie(eng, [be.prompt_ids(q) for q in qs], ref, got)


def test_mixtral_forward_hip_vs_reference():
    eng = _engine("mixtral-2l", graphs=False)
    be = EngineLLM(eng, max_new_tokens=8)
    with torch.inference_mode():
        h_hip = _prefill_hidden(eng, be, QUERIES[:2])
        with ops.force_reference():
            h_ref = _prefill_hidden(eng, be, QUERIES[:2])
    torch.testing.assert_close(h_hip.float(), h_ref.float(), atol=0.1, rtol=0.05)
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    seqs = eng.generate_blocking([be.prompt_ids(q) for q in QUERIES[:3]], params, forced_prefix=be._forced)
    assert all(len(s.output_ids) == len(be._forced) + 6 for s in seqs)


@pytest.mark.parametrize("model,B,graphs,long_ctx", [
    ("llama3-8b-2l", 1, False, False), ("llama3-8b-2l", 1, True, False), ("llama3-8b-2l", 1, False, True),
    ("llama3-8b-2l", 2, False, False), ("llama3-8b-2l", 2, True, False), ("llama3-8b-2l", 2, False, True),
    ("llama3-70b-2l/tp8", 1, False, False), ("llama3-70b-2l/tp8", 1, True, False),
    ("llama3-70b-2l/tp8", 1, False, True), ("llama3-70b-2l/tp8", 2, False, True)])
def test_persistent_decode_matches_kernel_chain_and_fp32(model, B, graphs, long_ctx):
    """csrc/decode_persistent.hip (every layer of a decode step of B = 1 / 2 sequences in one launch,
    grid-wide arrival counters, one attention leader per sequence and KV group) against the per-kernel
    decode chain and the fp32 references, over 6 decode steps (the real Llama-3-8B layer geometry, 2
    layers): hidden states within bf16 tolerance, the same KV appended, the tokens equal to the chain's,
    the error word clear — eagerly and as the captured bucket-B hipGraph.  long_ctx: a ~400-token
    context, past the tokens the attention leaders prefetch into their rings (the chunk loop's
    global-load path); at B = 2 the two sequences differ in length.  "/tp8": rank 0 of Llama-3-70B at
    TP = 8 on a virtual communicator (H 8192, 8 q heads over 1 KV head: the GQA-8 attention scratch and
    12-slot rings; its all-reduces are no-ops in the chain and the kernel alike)."""
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    from ai_agent_kubectl_amd.models.llama import AttnMeta
    from ai_agent_kubectl_amd.parallel.comm import VirtualRankComm
    kw = {}
    if model.endswith("/tp8"):
        model = model[:-4]
        kw = dict(comm=VirtualRankComm(8), tp_rank=0, tp_size=8)
    eng = _engine(model, graphs=graphs, buckets=(1, 2), max_batch=2, kv_cache_tokens=8192, **kw)
    be = EngineLLM(eng, max_new_tokens=16, ignore_eos=True)
    sch, r = eng.scheduler, eng.runner
    sch.gather_max_s = 0.0
    sch.prefill_max_wait_s = 0.0
    m = r.model
    with torch.inference_mode():
        for b in range(B):
            ids = be.prompt_ids(["list all pods in kube-system", "show services in namespace prod"][b])
            if long_ctx and b == 0:
                ids = ids + [(7 * i + 11) % 5000 + 100 for i in range(400 - len(ids))]
            sch.add(Sequence(prompt_ids=ids, params=SamplingParams(max_new_tokens=16, ignore_eos=True)))
        while sch.waiting:   # a long prompt may take several (chunked) prefill steps
            b = sch.schedule()
            eng._apply(b, r.execute(b))
            sch.on_step_done(b)
        for step in range(6):
            batch = sch.schedule()
            assert batch.is_decode and len(batch.seqs) == B
            r._pack_decode(batch, B)
            n = r._off["bt"] + B * r.max_blocks
            r.d_stage[:n].copy_(r.h_stage[:n])
            meta = AttnMeta(positions=r._view("pos", B), slot_mapping=r._view("slots", B),
                            block_tables=r._view("bt", B), ctx_lens=r._view("ctx", B),
                            logits_indices=r.d_logits_idx[:B], is_decode=True)
            ids = r._view("ids", B)
            kc, vc = r.k_cache.clone(), r.v_cache.clone()
            kr, vr = r.k_cache.clone(), r.v_cache.clone()
            m.persistent = False
            h_chain = m.forward(ids, meta, kc, vc)
            with ops.force_reference():
                h_ref = m.forward(ids, meta, kr, vr)
            m.persistent = True
            assert m.persistent_ok(B)
            kp, vp = r.k_cache.clone(), r.v_cache.clone()
            h_p = m.forward(ids, meta, kp, vp)
            torch.cuda.synchronize()
            assert m.persistent_err() == 0
            torch.testing.assert_close(h_p.float(), h_ref.float(), atol=0.1, rtol=0.05)
            torch.testing.assert_close(h_p.float(), h_chain.float(), atol=0.1, rtol=0.05)
            for b in range(B):
                slot = int(r._view("slots", B)[b])
                blk, off = slot // 16, slot % 16
                # layer 0's appended K / V come from the same embedding: bf16-exact up to the norm's
                # rounding; later layers see the fp32 residual stream (the chain's is bf16)
                for kk, ref_c, tol in ((kp, kc, 2e-2), (vp, vc, 2e-2)):
                    got = kk[0, blk, :, off] if kk is kp else kk[0, blk, :, :, off]
                    want = ref_c[0, blk, :, off] if kk is kp else ref_c[0, blk, :, :, off]
                    torch.testing.assert_close(got.float(), want.float(), atol=tol, rtol=tol)
                torch.testing.assert_close(kp[:, blk, :, off].float(), kc[:, blk, :, off].float(), atol=0.1, rtol=0.05)
                torch.testing.assert_close(vp[:, blk, :, :, off].float(), vc[:, blk, :, :, off].float(), atol=0.1,
                                           rtol=0.05)
            mask = r._view("mask", B) if r.mask_bits is not None else None
            tok = m.sample(h_p, r.mask_bits, mask)[:B].tolist()
            if graphs:   # the captured bucket-B graph runs the same kernel: the same tokens
                r.graphs.clear()
                r.graph_pool = None
                r.capture_graphs(autotune=False)
                assert r.graph_persistent.get(B)
                r._pack_decode(batch, B)          # capture_graphs reset the staging image
                r.d_stage[:n].copy_(r.h_stage[:n])
                r.graphs[B].replay()
                torch.cuda.synchronize()
                assert r.d_out[:B].tolist() == tok, (step, r.d_out[:B].tolist(), tok)
                assert m.persistent_err() == 0
            else:   # the persistent step's cache writes are the real ones from here on
                r.k_cache.copy_(kp)
                r.v_cache.copy_(vp)
            m.persistent = False
            eng._apply(batch, tok)
            sch.on_step_done(batch)
