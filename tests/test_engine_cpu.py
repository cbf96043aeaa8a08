"""Engine tests that run on CPU (reference ops, tiny models with the real vocab / head layout)."""
import os
import sys

import numpy as np
import pytest
import torch

from ai_agent_kubectl_amd.engine.block_manager import BlockManager, NoFreeBlocks
from ai_agent_kubectl_amd.engine.safe_decode import MASK_BODY, MASK_FIRST, build_masks, forced_prefix
from ai_agent_kubectl_amd.engine.scheduler import Scheduler
from ai_agent_kubectl_amd.engine.sequence import SamplingParams, Sequence, SeqStatus
from ai_agent_kubectl_amd.engine.tokenizer import SyntheticTokenizer, get_tokenizer
from ai_agent_kubectl_amd.prompt import PROMPT_PREFIX, render_prompt
from ai_agent_kubectl_amd.safety import is_safe_kubectl_command

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------- tokenizer ----------------
@pytest.mark.parametrize("vocab,family", [(128256, "llama3"), (32000, "llama2")])
def test_tokenizer_roundtrip_and_density(vocab, family):
    tok = get_tokenizer(vocab, family)
    p = render_prompt("list all pods in namespace prod ünïcode ✓")
    ids = tok.encode(p)
    assert tok.decode(ids) == p
    assert all(0 <= i < vocab for i in ids)
    assert 3.0 < len(p) / len(ids) < 6.0     # ~4 chars/token like a real BPE
    chat = tok.encode_chat("hi")
    assert chat[0] == tok.bos_id


def test_tokenizer_specials():
    tok = get_tokenizer(128256, "llama3")
    assert tok.is_eos(128009) and tok.is_eos(128001) and tok.bos_id == 128000
    assert tok.decode([128000, tok.encode("x")[0]]) == "x"


# ---------------- safe decode ----------------
def test_safe_masks_only_allow_validator_safe_tokens():
    tok = get_tokenizer(128256, "llama3")
    m = build_masks(tok)
    bits = np.unpackbits(m.view(np.uint8), bitorder="little").reshape(2, -1)[:, :tok.vocab_size].astype(bool)
    first = np.nonzero(bits[MASK_FIRST])[0]
    body = np.nonzero(bits[MASK_BODY])[0]
    assert len(first) > 1000 and len(body) > len(first)
    rng = np.random.RandomState(0)
    pre = tok.decode(forced_prefix(tok))
    assert pre == "kubectl"
    for _ in range(300):
        toks = [rng.choice(first)] + list(rng.choice(body, size=rng.randint(0, 12)))
        toks = [t for t in toks if not tok.is_eos(t)]
        assert is_safe_kubectl_command(pre + tok.decode(toks))


# ---------------- block manager ----------------
def test_prefix_cache_sharing_and_eviction():
    bm = BlockManager(num_blocks=12, block_size=4)
    a = list(range(10))                       # 2 full blocks + partial
    t1, c1, h1 = bm.allocate_prompt(a)
    assert c1 == 0 and len(t1) == 3
    bm.register_computed(t1, a, h1)
    t2, c2, h2 = bm.allocate_prompt(a[:8] + [99, 98])
    assert c2 == 8 and t2[:2] == t1[:2] and t2[2] != t1[2]
    assert bm.ref[t1[0]] == 2
    bm.free_table(t1)
    bm.free_table(t2)
    assert bm.num_free == 12
    # cached blocks survive until memory pressure evicts them
    t3, c3, _ = bm.allocate_prompt(a)
    assert c3 == 8
    bm.free_table(t3)
    big, _, _ = bm.allocate_prompt(list(range(100, 148)))   # needs all 12 blocks -> evicts cache
    assert len(big) == 12
    with pytest.raises(NoFreeBlocks):
        bm.allocate_prompt([1, 2, 3])
    bm.free_table(big)
    t4, c4, _ = bm.allocate_prompt(a)
    assert c4 == 0


@pytest.mark.parametrize("native", [False, True])
def test_sub_block_reuse(native):
    if native:
        from ai_agent_kubectl_amd.runtime.native import NativeBlockManager, available
        if not available():
            pytest.skip("native runtime not built")
        bm = NativeBlockManager(num_blocks=12, block_size=4)
    else:
        bm = BlockManager(num_blocks=12, block_size=4)
    a = list(range(1, 13))                    # 3 full blocks once computed
    t1, c1, h1 = bm.allocate_prompt(a)
    bm.register_computed(t1, a, h1)
    b = a[:10] + [77, 78, 79]                 # shares 2 full blocks + 2 tokens of the third
    t2, c2, h2 = bm.allocate_prompt(b)
    assert c2 == 8
    src, r = bm.reuse_partial(t2, b, c2, h2)
    assert (src, r) == (t1[2], 2) and src not in t2
    assert bm.ref_count(src) == 2             # pinned (t1 + the pending copy)
    bm.unpin(src)
    assert bm.ref_count(src) == 1
    # never reaches the last prompt token, nothing shared -> no reuse
    assert bm.reuse_partial(t2, a[:9], 8, h2) is None
    c = a[:8] + [50, 51, 52]
    t3, c3, h3 = bm.allocate_prompt(c)
    assert bm.reuse_partial(t3, c, c3, h3) is None
    # an evicted sibling is never offered
    for t in (t1, t2, t3):
        bm.free_table(t)
    bm.reset_prefix_cache()
    t4, c4, h4 = bm.allocate_prompt(b)
    assert c4 == 0 and bm.reuse_partial(t4, b, c4, h4) is None


def test_last_token_always_recomputed():
    bm = BlockManager(num_blocks=8, block_size=4)
    a = list(range(8))
    t, _, h = bm.allocate_prompt(a)
    bm.register_computed(t, a, h)
    t2, c2, _ = bm.allocate_prompt(a)
    assert c2 == 4        # the block holding the last prompt token is recomputed


# ---------------- scheduler ----------------
def _seq(n, new=4):
    return Sequence(prompt_ids=list(range(1000, 1000 + n)), params=SamplingParams(max_new_tokens=new))


def test_scheduler_budget_and_mixing():
    bm = BlockManager(64, 4, enable_prefix_caching=False)
    sch = Scheduler(bm, max_batch=3, max_batched_tokens=20, prefill_max_wait_s=0.0)
    seqs = [_seq(8), _seq(8), _seq(8), _seq(8)]
    for s in seqs:
        sch.add(s)
    b = sch.schedule()
    assert not b.is_decode and [len(x.all_ids) for x in b.prefill_seqs] == [8, 8]   # budget 20
    for s, n in zip(b.seqs, b.num_query):
        s.num_computed += n
        s.output_ids.append(1)
    sch.on_step_done(b)
    b = sch.schedule()   # third admitted + two decode rows mixed in
    assert len(b.prefill_seqs) == 1 and b.num_query == [1, 1, 8]


def test_scheduler_preempts_when_out_of_blocks():
    bm = BlockManager(5, 4, enable_prefix_caching=False)
    sch = Scheduler(bm, max_batch=4, max_batched_tokens=100, prefill_max_wait_s=0.0)
    s1, s2 = _seq(8, new=8), _seq(8, new=8)
    sch.add(s1)
    sch.add(s2)
    b = sch.schedule()
    assert len(b.prefill_seqs) == 2 and bm.num_free == 1
    for s, n in zip(b.seqs, b.num_query):
        s.num_computed += n
        s.output_ids.append(5)
    sch.on_step_done(b)
    b = sch.schedule()   # both need a 3rd block at length 9 -> one is preempted
    assert b.is_decode and len(b.seqs) == 1
    assert len(sch.waiting) == 1 and sch.waiting[0].status is SeqStatus.WAITING


def _step(sch, b, tok=1):
    """Apply a scheduled batch the way LLMEngine._apply does (chunk rows sample nothing)."""
    for s, n in zip(b.seqs, b.num_query):
        s.num_computed += n
        if id(s) not in b.partial:
            s.output_ids.append(tok)
    sch.on_step_done(b)


def test_scheduler_chunks_long_prompt():
    """A prompt over the step budget is prefilled in budget-sized chunks; the
    running decodes keep their row in every chunk step; an arrival waits for budget."""
    bm = BlockManager(64, 4, enable_prefix_caching=False)
    sch = Scheduler(bm, max_batch=4, max_batched_tokens=20, prefill_max_wait_s=0.0, chunked_prefill=True,
                    min_chunk=8, hold_steps=0)
    short = _seq(6, new=8)
    sch.add(short)
    b = sch.schedule()
    assert b.num_query == [6] and not b.partial
    _step(sch, b)
    long_ = _seq(50)
    sch.add(long_)
    b = sch.schedule()     # 1 decode row + 19-token chunk
    assert b.seqs == [short, long_] and b.num_query == [1, 19] and b.partial == {id(long_)}
    _step(sch, b)
    assert sch.prefilling == [long_] and long_.output_ids == [] and long_.num_computed == 19
    late = _seq(5)
    sch.add(late)
    b = sch.schedule()     # the chunked prompt continues first; the late arrival does not fit
    assert b.seqs == [short, long_] and b.num_query == [1, 19]
    _step(sch, b)
    b = sch.schedule()     # last 12 prompt tokens sample the first token; 7 left for the arrival
    assert b.seqs == [short, long_, late] and b.num_query == [1, 12, 5] and not b.partial
    _step(sch, b)
    assert sch.prefilling == [] and long_.num_computed == 50 and long_.output_ids == [1]
    assert sch.running == [short, long_, late]
    assert sch.schedule().is_decode


def test_scheduler_unchunked_admits_over_budget_prompt_whole():
    bm = BlockManager(64, 4, enable_prefix_caching=False)
    sch = Scheduler(bm, max_batch=4, max_batched_tokens=20, prefill_max_wait_s=0.0, chunked_prefill=False)
    sch.add(_seq(50))
    b = sch.schedule()
    assert b.num_query == [50] and not b.partial


# ---------------- engine end to end (CPU) ----------------
@pytest.fixture(scope="module")
def tiny_engine():
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
    eng = build_engine(EngineOptions(model="tiny-llama", device="cpu", max_batch=8, graph_buckets=(1, 2, 4, 8),
                                     kv_cache_tokens=8192, max_model_len=512))
    return eng, EngineLLM(eng, max_new_tokens=10)


def test_engine_generates_safe_commands_and_hits_prefix_cache(tiny_engine):
    eng, be = tiny_engine
    qs = ["list pods", "show services in prod", "scale web to 3"]
    seqs = eng.generate_blocking([be.prompt_ids(q) for q in qs], be.params, forced_prefix=be._forced)
    for s in seqs:
        txt = be.tok.decode([t for t in s.output_ids if not be.tok.is_eos(t)])
        assert txt.startswith("kubectl ") and is_safe_kubectl_command(txt)
    seqs2 = eng.generate_blocking([be.prompt_ids("get nodes")], be.params, forced_prefix=be._forced)
    assert seqs2[0].num_cached_prompt >= 48
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_prefix_cached_equals_cold(tiny_engine):
    eng, be = tiny_engine
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    ids = be.prompt_ids("describe deployment api")
    eng.bm.reset_prefix_cache()
    cold = eng.generate_blocking([ids], params, forced_prefix=be._forced)[0]
    warm = eng.generate_blocking([ids], params, forced_prefix=be._forced)[0]
    assert cold.num_cached_prompt == 0 and warm.num_cached_prompt > 0
    assert cold.output_ids == warm.output_ids


def test_sub_block_reuse_equals_cold(tiny_engine):
    """KV rows copied from a sibling block give the same tokens as computing them."""
    eng, be = tiny_engine
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    q1, q2 = be.prompt_ids("list pods in prod"), be.prompt_ids("list services in dev")
    eng.bm.reset_prefix_cache()
    cold = eng.generate_blocking([q2], params, forced_prefix=be._forced)[0]
    eng.bm.reset_prefix_cache()
    eng.generate_blocking([q1], params, forced_prefix=be._forced)
    before = eng.bm.partial_tokens
    warm = eng.generate_blocking([q2], params, forced_prefix=be._forced)[0]
    assert eng.bm.partial_tokens > before
    assert warm.num_cached_prompt > cold.num_cached_prompt
    assert cold.output_ids == warm.output_ids
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_mixed_step_split_attention_matches(tiny_engine):
    from tests.engine_helpers import run_staggered
    eng, be = tiny_engine
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    prompts = [be.prompt_ids(q) for q in ("list pods", "get nodes -o wide", "describe svc api", "top pods")]
    alone = [eng.generate_blocking([p], params, forced_prefix=be._forced)[0].output_ids for p in prompts]
    outs = {}
    for split in (False, True):
        eng.runner.split_mixed_attention = split
        eng.bm.reset_prefix_cache()
        try:
            outs[split] = run_staggered(eng, prompts, params, be._forced)
            assert run_staggered.mixed >= 3
        finally:
            eng.runner.split_mixed_attention = True
    assert outs[True] == outs[False] == alone


def _run_thread(eng, prompts, params, forced, abort_idx=None):
    import threading
    done = {}
    ev = threading.Event()

    want = len(prompts) - (abort_idx is not None)   # an abort completes without a callback

    def cb(seq):
        done[seq.seq_id] = seq
        if len(done) == want:
            ev.set()

    eng.start()
    try:
        seqs = [eng.submit(p, params, cb, forced_prefix=forced) for p in prompts]
        if abort_idx is not None:
            eng.abort(seqs[abort_idx])
        assert ev.wait(60)
        if abort_idx is not None:
            import time
            time.sleep(0.2)
    finally:
        eng.shutdown()
    return seqs


def test_padded_prefill_matches_unpadded(tiny_engine):
    """Prefill steps padded to a tile multiple (slot -1 rows, zeroed attention) sample the same tokens."""
    eng, be = tiny_engine
    params = SamplingParams(max_new_tokens=5, ignore_eos=True)
    prompts = [be.prompt_ids(q) for q in ("list pods", "get svc -A", "top nodes")]
    r = eng.runner
    outs = []
    for pad, pmin in ((0, 1 << 30), (64, 1)):
        r.prefill_pad, r.prefill_pad_min = pad, pmin
        eng.bm.reset_prefix_cache()
        outs.append([s.output_ids for s in eng.generate_blocking(prompts, params, forced_prefix=be._forced)])
    r.prefill_pad, r.prefill_pad_min = 256, 1024
    assert r.padded_tokens(1000) == 1000 and r.padded_tokens(1030) == 1280
    assert outs[0] == outs[1]


def test_overlapped_decode_matches_sync(tiny_engine):
    """One decode step in flight while the host applies the previous one (engine._chain) gives the
    same tokens as the synchronous loop, with EOS stops, length stops and an abort mid-flight."""
    eng, be = tiny_engine
    prompts = [be.prompt_ids(q) for q in ("list pods", "get svc -A", "top nodes", "describe pod web-1",
                                          "logs api", "get deploy")]
    outs = {}
    for overlap in (False, True):
        eng.overlap = overlap
        eng.bm.reset_prefix_cache()
        for ignore_eos in (True, False):
            params = SamplingParams(max_new_tokens=7, ignore_eos=ignore_eos)
            seqs = _run_thread(eng, prompts, params, be._forced)
            outs[(overlap, ignore_eos)] = [s.output_ids for s in seqs]
            assert all(s.finish_reason in ("stop", "length") for s in seqs)
        seqs = _run_thread(eng, prompts, SamplingParams(max_new_tokens=7, ignore_eos=True), be._forced, abort_idx=2)
        assert seqs[2].finish_reason == "abort"
    eng.overlap = True
    assert eng.chained_steps > 0
    assert eng.prefill_chains > 0      # first decode queued behind the prefill before its readback
    assert outs[(True, True)] == outs[(False, True)]
    assert outs[(True, False)] == outs[(False, False)]
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_lookahead_steps_match_sync(tiny_engine):
    """Sequences of different lengths (rows leave the batch at different steps, EOS stops allowed)
    and chunked prompts through the threaded engine with lookahead (each composition change
    scheduled from a provisional advance of the in-flight step and queued before its readback, the
    placeholder inputs fixed up on the device) sample the same tokens as without it."""
    import threading
    eng, be = tiny_engine
    prompts = [be.prompt_ids(q) for q in ("list pods", "get svc -A", "top nodes", "describe pod web-1",
                                          "logs api", "get deploy", "get services in namespace kube-system")]
    lens = [3, 9, 5, 7, 2, 8, 6]

    def run(lookahead, ignore_eos):
        eng.lookahead = lookahead
        eng.bm.reset_prefix_cache()
        done, ev = {}, threading.Event()

        def cb(seq):
            done[seq.seq_id] = seq
            if len(done) == len(prompts):
                ev.set()

        eng.start()
        try:
            seqs = [eng.submit(p, SamplingParams(max_new_tokens=n, ignore_eos=ignore_eos), cb,
                               forced_prefix=be._forced) for p, n in zip(prompts, lens)]
            assert ev.wait(60)
        finally:
            eng.shutdown()
        return [list(s.output_ids) for s in seqs]

    sch = eng.scheduler
    saved = sch.max_batched_tokens, sch.min_chunk
    sch.max_batched_tokens, sch.min_chunk = 40, 4
    try:
        n0 = eng.lookahead_steps
        for ignore_eos in (True, False):
            on, off = run(True, ignore_eos), run(False, ignore_eos)
            assert on == off
            assert all(-1 not in o for o in on)
            if ignore_eos:
                assert [len(o) - len(be._forced) for o in on] == lens
        assert eng.lookahead_steps > n0
    finally:
        sch.max_batched_tokens, sch.min_chunk = saved
        eng.lookahead = True
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_lookahead_sync_fallback_drops_finished_rows(tiny_engine):
    """A step scheduled ahead that cannot be queued early (more rows than the largest graph bucket)
    runs after the in-flight step's readback; rows whose sequence that readback finished (EOS) must
    leave it before the runner packs it (their freed block tables would alias KV block 0).  Two
    sequences decode in flight (bmax = 2), five more arrive, EOS stops are frequent (a patched
    is_eos): the engine, stepped by hand, must sample what it samples with KA_LOOKAHEAD=0."""
    from ai_agent_kubectl_amd.engine.engine import LLMEngine
    eng, be = tiny_engine
    prompts = [be.prompt_ids(q) for q in ("list pods", "get svc -A", "top nodes", "describe pod web-1",
                                          "logs api", "get deploy", "get services in namespace kube-system")]
    tok, r, sch = eng.tokenizer, eng.runner, eng.scheduler
    orig_eos, saved = tok.is_eos, (r.bmax, sch.gather_max_s, sch.prefill_max_wait_s)
    calls = {"n": 0}
    orig_filter = LLMEngine._without_finished

    def counting(batch):
        calls["n"] += any(s.finished for s in batch.seqs)
        return orig_filter(batch)

    def run(lookahead, k):
        eng.lookahead = lookahead
        eng.bm.reset_prefix_cache()
        seqs = [eng.submit(p, SamplingParams(max_new_tokens=9), None, forced_prefix=be._forced) for p in prompts[:2]]
        for i in range(400):
            if i == k:
                seqs += [eng.submit(p, SamplingParams(max_new_tokens=9), None, forced_prefix=be._forced)
                         for p in prompts[2:]]
            eng.step()
            if i >= k and all(s.finished for s in seqs) and eng._inflight is None:
                break
        assert all(s.finished for s in seqs) and eng.healthy
        return [(list(s.output_ids), s.finish_reason) for s in seqs]

    tok.is_eos = lambda t: orig_eos(t) or t % 5 == 2
    r.bmax, sch.gather_max_s, sch.prefill_max_wait_s = 2, 0.0, 0.0
    eng._without_finished = counting
    try:
        for k in range(1, 7):
            on, off = run(True, k), run(False, k)
            assert on == off, k
        assert calls["n"] > 0   # the fallback really met rows finished by the readback
    finally:
        tok.is_eos = orig_eos
        r.bmax, sch.gather_max_s, sch.prefill_max_wait_s = saved
        del eng._without_finished
        eng.lookahead = True
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_chunked_prefill_matches_whole_prefill(tiny_engine):
    """Prompts prefilled in 24-token chunks (through the threaded engine: mixed chunk + decode
    steps, overlapped decode) sample the same tokens as one whole-prompt prefill."""
    eng, be = tiny_engine
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    prompts = [be.prompt_ids(q) for q in ("list pods", "get services in namespace kube-system -o wide",
                                          "describe deployment api-gateway")]
    eng.bm.reset_prefix_cache()
    whole = [s.output_ids for s in eng.generate_blocking(prompts, params, forced_prefix=be._forced)]
    sch = eng.scheduler
    saved = sch.max_batched_tokens, sch.min_chunk
    sch.max_batched_tokens, sch.min_chunk = 24, 4
    try:
        eng.bm.reset_prefix_cache()
        chunked = [s.output_ids for s in eng.generate_blocking(prompts, params, forced_prefix=be._forced)]
        eng.bm.reset_prefix_cache()
        threaded = [s.output_ids for s in _run_thread(eng, prompts, params, be._forced)]
    finally:
        sch.max_batched_tokens, sch.min_chunk = saved
    assert min(len(p) for p in prompts) + len(be._forced) > 24   # every prompt really was chunked
    assert chunked == whole and threaded == whole
    assert eng.lookahead_steps > 0
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_api_with_engine_backend(tiny_engine):
    from fastapi.testclient import TestClient
    from ai_agent_kubectl_amd.api import create_app
    from ai_agent_kubectl_amd.config import Settings
    eng, be = tiny_engine
    app = create_app(Settings(RATE_LIMIT="1000/minute"), backend=be)
    with TestClient(app) as c:      # lifespan starts / stops the engine thread
        r = c.post("/kubectl-command", json={"query": "list all pods"})
        assert r.status_code == 200, r.text
        assert is_safe_kubectl_command(r.json()["kubectl_command"])
        assert c.post("/kubectl-command", json={"query": "list all pods"}).json()["from_cache"] is True
        m = c.get("/metrics").text
        assert "llm_ttft_seconds_count 1.0" in m
        assert "llm_queue_wait_seconds_count 1.0" in m
        assert 'llm_step_seconds_count{phase="prefill"}' in m and 'llm_step_seconds_count{phase="decode"}' in m


# ---------------- tensor parallel numerics ----------------
@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_virtual_tp2_matches_tp1_cpu(model):
    sys.path.insert(0, ROOT)
    from tests.virtual_tp import virtual_tp_logits
    from ai_agent_kubectl_amd.models.config import get_config
    cfg = get_config(model)
    a = virtual_tp_logits(cfg, 1, device="cpu").float()
    b = virtual_tp_logits(cfg, 2, device="cpu").float()
    assert torch.nn.functional.cosine_similarity(a, b, dim=-1).min() > 0.9999
    assert torch.equal(a.argmax(-1), b.argmax(-1))


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_virtual_tp2_generate_matches_tp1_cpu(model):
    """Driver / worker TP protocol (header + metadata broadcasts, worker_loop, vocab-parallel
    argmax, EP all-to-all prefill for Mixtral) with one rank per thread: same greedy tokens."""
    sys.path.insert(0, ROOT)
    from tests.virtual_tp import virtual_tp_generate
    qs = ["list all pods", "show services in prod", "scale web to 3"]
    assert virtual_tp_generate(model, 2, qs, device="cpu") == virtual_tp_generate(model, 1, qs, device="cpu")


def test_openai_compatible_chat(tiny_engine):
    from fastapi.testclient import TestClient
    from ai_agent_kubectl_amd.api import create_app
    from ai_agent_kubectl_amd.config import Settings
    eng, be = tiny_engine
    app = create_app(Settings(RATE_LIMIT="1000/minute", API_AUTH_KEY="k", MODEL="tiny-llama"), backend=be)
    with TestClient(app) as c:
        body = {"model": "tiny-llama", "messages": [{"role": "user", "content": "list pods"}], "max_tokens": 5}
        assert c.post("/v1/chat/completions", json=body).status_code == 401
        r = c.post("/v1/chat/completions", json=body, headers={"Authorization": "Bearer k"})
        assert r.status_code == 200, r.text
        j = r.json()
        assert j["object"] == "chat.completion" and j["usage"]["completion_tokens"] <= 5
        assert isinstance(j["choices"][0]["message"]["content"], str)
        assert c.get("/v1/models", headers={"X-API-Key": "k"}).json()["data"][0]["id"] == "tiny-llama"


def test_native_block_manager_matches_python():
    import random
    from ai_agent_kubectl_amd.runtime.native import NativeBlockManager, available
    if not available():
        pytest.skip("native runtime not built")
    rng = random.Random(0)
    py_bm, nv_bm = BlockManager(40, 4), NativeBlockManager(40, 4)
    prefixes = [[rng.randrange(50) for _ in range(rng.randrange(4, 17))] for _ in range(4)]
    live = []
    for step in range(400):
        op = rng.random()
        if op < 0.5 and len(live) < 8:
            toks = rng.choice(prefixes) + [rng.randrange(50) for _ in range(rng.randrange(1, 9))]
            res = []
            register = rng.random() < 0.8
            for bm in (py_bm, nv_bm):
                try:
                    t, c, h = bm.allocate_prompt(toks)
                    part = bm.reuse_partial(t, toks, c, h)
                    if part:
                        bm.unpin(part[0])
                    res.append((t, c, part))
                    if register:
                        bm.register_computed(t, toks, h)
                except NoFreeBlocks:
                    res.append(None)
            assert res[0] == res[1], step
            if res[0] is not None:
                live.append([res[0][0], list(res[0][0]), toks])
        elif op < 0.75 and live:
            ent = rng.choice(live)
            n = len(ent[2]) + rng.randrange(1, 6)
            outs = []
            for bm, tbl in ((py_bm, ent[0]), (nv_bm, ent[1])):
                try:
                    bm.ensure_capacity(tbl, n)
                    outs.append(list(tbl))
                except NoFreeBlocks:
                    outs.append(None)
            assert outs[0] == outs[1], step
        elif live:
            ent = live.pop(rng.randrange(len(live)))
            py_bm.free_table(ent[0])
            nv_bm.free_table(ent[1])
        assert py_bm.num_free == nv_bm.num_free
    assert py_bm.hits == nv_bm.hits and py_bm.queries == nv_bm.queries
    assert py_bm.partial_tokens == nv_bm.partial_tokens > 0


def test_native_tokenizer_matches_python():
    from ai_agent_kubectl_amd.runtime.native import available
    if not available():
        pytest.skip("native runtime not built")
    tok = get_tokenizer(128256, "llama3")
    assert tok._native is not None
    text = render_prompt("list all pods in namespace prod ünïcode ✓ --sort-by=.metadata.name")
    native = tok.encode(text)
    saved, tok._native = tok._native, None
    try:
        assert tok.encode(text) == native
    finally:
        tok._native = saved


def test_scheduler_gathers_a_streaming_burst_when_idle():
    import time
    bm = BlockManager(64, 16)
    sch = Scheduler(bm, max_batch=8, max_batched_tokens=4096, gather_max_s=0.05, gather_quiet_s=0.01)
    a = _seq(20)
    sch.add(a)
    assert sch.gathering() and sch.schedule().seqs == []        # newest arrival is fresh: hold
    time.sleep(0.015)                                            # quiet gap passed
    assert not sch.gathering()
    b = sch.schedule()
    assert b.prefill_seqs == [a]
    # with sequences running, gathering never applies (the mixed-step policy decides)
    sch.on_step_done(b)
    sch.add(_seq(20))
    assert not sch.gathering()
    # a burst that keeps arriving is cut off at gather_max_s
    sch2 = Scheduler(BlockManager(64, 16), max_batch=8, max_batched_tokens=4096, gather_max_s=0.02,
                     gather_quiet_s=0.01)
    first = _seq(10)
    sch2.add(first)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.03:
        if sch2.gathering():
            sch2.add(_seq(10))
        time.sleep(0.002)
    assert not sch2.gathering() and len(sch2.schedule().prefill_seqs) >= 2


def test_scheduler_gather_is_short_for_steady_arrivals():
    """Without a drained burst (open-loop arrivals into an idle engine) the gather window closes
    after two quiet gaps even while requests keep arriving; after a large batch drains it may run
    to gather_max_s."""
    import time
    sch = Scheduler(BlockManager(256, 16), max_batch=64, max_batched_tokens=4096, gather_max_s=0.1,
                    gather_quiet_s=0.005)
    sch.add(_seq(10))
    t0 = time.perf_counter()
    while sch.gathering() and time.perf_counter() - t0 < 0.2:
        sch.add(_seq(10))              # an arrival every ~2 ms keeps the quiet gap from closing
        time.sleep(0.002)
    assert time.perf_counter() - t0 < 0.08   # well short of gather_max_s (slack for a loaded host)
    sch2 = Scheduler(BlockManager(256, 16), max_batch=64, max_batched_tokens=4096, gather_max_s=0.1,
                     gather_quiet_s=0.005)
    sch2._idle_since, sch2._drained = time.perf_counter(), 64     # a 64-request wave just drained
    sch2.burst_quiet_s = 0.05   # a loaded host (pytest -n) may oversleep the 2-ms gaps past the default
    sch2.add(_seq(10))
    t0 = time.perf_counter()
    while sch2.gathering() and time.perf_counter() - t0 < 0.2:
        sch2.add(_seq(10))
        time.sleep(0.002)
    assert time.perf_counter() - t0 > 0.03
    # ... but it closes as soon as as many requests are back as just finished
    sch3 = Scheduler(BlockManager(256, 16), max_batch=64, max_batched_tokens=4096, gather_max_s=10.0,
                     gather_quiet_s=5.0)
    sch3._idle_since, sch3._drained = time.perf_counter(), 40
    for _ in range(39):
        sch3.add(_seq(10))
    assert sch3.gathering()
    sch3.add(_seq(10))
    assert not sch3.gathering()


def test_scheduler_batches_prefills_while_decoding():
    bm = BlockManager(64, 4, enable_prefix_caching=False)
    sch = Scheduler(bm, max_batch=16, max_batched_tokens=1000, prefill_max_wait_s=10.0, hold_steps=0)
    first = _seq(8)
    sch.add(first)
    b = sch.schedule()
    assert b.prefill_seqs == [first]          # nothing running -> admit immediately
    first.num_computed, first.output_ids = 8, [1]
    sch.on_step_done(b)
    for _ in range(3):
        sch.add(_seq(8))
    assert sch.schedule().is_decode           # 3 waiting < 4 and young -> keep decoding
    sch.add(_seq(8))
    b = sch.schedule()
    assert len(b.prefill_seqs) == 4           # batch of 4 admitted together (+1 decode row mixed)


def test_scheduler_holds_arrivals_until_the_running_wave_drains():
    """Wave merging: arrivals that find every running sequence within hold_steps of its token
    limit wait; once the wave drains, the gather window opens at the idle moment and keeps the
    held requests until the drained wave's clients come back (or gather_max_s)."""
    from ai_agent_kubectl_amd.engine.block_manager import BlockManager
    from ai_agent_kubectl_amd.engine.scheduler import Scheduler
    import time as _t
    sch = Scheduler(BlockManager(256, 16), max_batch=8, max_batched_tokens=4096, gather_max_s=0.0,
                    gather_quiet_s=0.01, hold_steps=4, hold_max_s=10.0, prefill_min_frac=0.0,
                    prefill_max_wait_s=0.0)
    p = SamplingParams(max_new_tokens=6, ignore_eos=True)
    first = [Sequence(prompt_ids=list(range(i, i + 20)), params=p) for i in range(3)]
    for s in first:
        sch.add(s)
    b = sch.schedule()
    assert b.prefill_seqs == first
    for s in first:
        s.output_ids.append(1)
    sch.on_step_done(b)
    # far from the limit (5 tokens left > hold 4): an arrival is admitted as a mixed step
    late = Sequence(prompt_ids=list(range(100, 120)), params=p)
    sch.add(late)
    assert sch.schedule().prefill_seqs == [late]
    sch.running.append(late)
    late.status = first[0].status
    for s in first + [late]:
        s.output_ids.extend([1] * 4)
    # every running sequence within 4 tokens of its limit -> hold the next arrival
    held = Sequence(prompt_ids=list(range(200, 220)), params=p)
    sch.add(held)
    b = sch.schedule()
    assert b.is_decode and held in sch.waiting
    # the wave drains: idle from now on; the held request alone does not end the gather window
    sch.gather_max_s = 0.05
    for s in first + [late]:
        s.status = SeqStatus.FINISHED
    sch.on_step_done(b)
    assert not sch.running and sch.gathering()
    comeback = Sequence(prompt_ids=list(range(300, 320)), params=p)
    sch.add(comeback)
    assert sch.gathering()                          # newest arrival is fresh
    _t.sleep(0.02)
    assert not sch.gathering()                      # quiet gap passed: admit both together
    assert sch.schedule().prefill_seqs == [held, comeback]


def test_pack_prefill_matches_per_sequence_reference():
    """runner._pack_prefill (vectorised) against a per-sequence construction from first principles,
    on a mixed batch: fresh prompts, a prefix-cached prompt and decode rows, with padding."""
    import numpy as np

    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.safe_decode import forced_prefix, mask_index_for
    from ai_agent_kubectl_amd.engine.scheduler import Batch
    from ai_agent_kubectl_amd.engine.sequence import SamplingParams, Sequence

    eng = build_engine(EngineOptions(model="tiny-llama", device="cpu", max_batch=16, kv_cache_tokens=4096,
                                     max_model_len=512, use_graphs=False))
    tok = eng.tokenizer
    forced = forced_prefix(tok)
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    prompts = [tok.encode(f"query number {i} " * (i + 3)) for i in range(5)]
    seqs = [Sequence(prompt_ids=p, params=params, forced_prefix=list(forced)) for p in prompts]
    eng.generate_blocking([prompts[0]], params, forced_prefix=forced)     # warm the prefix cache
    for s in seqs[:2]:                                                   # two sequences already decoding
        eng.scheduler.add(s)
    eng.scheduler.gather_max_s = 0.0    # admit now (no burst gathering)
    b0 = eng.scheduler.schedule()
    assert len(b0.prefill_seqs) == 2
    eng._apply(b0, eng.runner.execute(b0))
    eng.scheduler.on_step_done(b0)
    for s in seqs[:2]:
        eng.bm.ensure_capacity(s.block_table, s.total_len)
    for s in seqs[2:]:
        eng.scheduler.add(s)
        t, cached, hashes = eng.bm.allocate_prompt(s.all_ids)
        s.block_table, s.block_hashes, s.num_computed = t, hashes, cached
    rows = [(s, 1) for s in seqs[:2]] + [(s, s.total_len - s.num_computed) for s in seqs[2:]]
    batch = Batch([r[0] for r in rows], [r[1] for r in rows], is_decode=False)
    batch.prefill_seqs = list(seqs[2:])
    buf = eng.runner._pack_prefill(batch, pad=True)

    T = eng.runner.padded_tokens(batch.num_tokens)
    S, mb, bs = len(rows), eng.runner.max_blocks, eng.runner.block_size
    ids, pos, slots = buf[:T], buf[T:2 * T], buf[2 * T:3 * T]
    o = 3 * T
    q_starts = buf[o:o + S + 1]; o += S + 1
    ctx = buf[o:o + S]; o += S
    mask = buf[o:o + S]; o += S
    lidx = buf[o:o + S]; o += S
    bt = buf[o:o + S * mb].reshape(S, mb)
    t = 0
    for i, (s, nq) in enumerate(rows):
        start = s.total_len - nq
        assert q_starts[i] == t and ctx[i] == s.total_len and lidx[i] == t + nq - 1
        assert list(ids[t:t + nq]) == s.all_ids[start:s.total_len]
        assert list(pos[t:t + nq]) == list(range(start, s.total_len))
        want = [s.block_table[p // bs] * bs + p % bs for p in range(start, s.total_len)]
        assert list(slots[t:t + nq]) == want
        assert list(bt[i, :len(s.block_table)]) == s.block_table
        assert mask[i] == mask_index_for(s.num_generated, s.params.safe_decode)
        t += nq
    assert q_starts[S] == t and np.all(slots[t:] == -1)


def test_moe_sorted_matches_grouped_and_batched():
    """Prefill MoE path (one host sync per layer) == per-expert bucketing == dense formulation,
    for the full expert set and for an EP shard."""
    import torch

    from ai_agent_kubectl_amd.models.config import get_config
    from ai_agent_kubectl_amd.models.moe import moe_batched, moe_grouped, moe_sorted
    cfg = get_config("tiny-mixtral")
    torch.manual_seed(0)
    T, H, I, E = 37, cfg.hidden, cfg.intermediate, cfg.num_experts
    x = torch.randn(T, H)
    for ep_rank, ep_size in ((0, 1), (1, 2)):
        el = E // ep_size
        L = {"router": torch.randn(E, H) * 0.1, "w13": torch.randn(el, 2 * I, H) * 0.05,
             "w2": torch.randn(el, H, I) * 0.05}
        a = moe_sorted(x, L, cfg, ep_rank, ep_size)
        b = moe_grouped(x, L, cfg, ep_rank, ep_size)
        c = moe_batched(x, L, cfg, ep_rank, ep_size)
        torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(a, c, atol=1e-4, rtol=1e-4)


def test_gemm_plan_file_roundtrip(tmp_path):
    """Persisted decode GEMM plans (ops/autotune.py): save merges entries keyed by M,N,K,consumer;
    load fills GEMM_PLAN for what it holds and reports what is missing; the committed MI355X file
    covers every Llama-3-8B decode bucket up to 512."""
    from ai_agent_kubectl_amd import ops
    from ai_agent_kubectl_amd.ops.autotune import DEFAULT_PLAN_FILE, load_plan, save_plan
    path = str(tmp_path / "plan.json")
    rep = {(64, 4096, 4096): {"choice": "gm", "split": 8, "cfg": 5, "us": 13.0, "blas_us": 20.0},
           (256, 28672, 4096): {"choice": "blas", "split": 0, "cfg": 0, "us": 66.0, "blas_us": 66.0}}
    save_plan(path, rep, {(4096, 4096): "norm-bf16", (28672, 4096): "plain"})
    saved = dict(ops.GEMM_PLAN)
    try:
        missing = load_plan(path, {(64, 4096, 4096): "norm-bf16", (256, 28672, 4096): "plain",
                                   (128, 28672, 4096): "plain", (64, 4096, 4096 * 2): "plain"})
        assert missing == {(128, 28672, 4096), (64, 4096, 8192)}
        assert ops.GEMM_PLAN[(64, 4096, 4096)] == ("gm", 8, 5) and ops.GEMM_PLAN[(256, 28672, 4096)] == ("blas", 0, 0)
        # a different consumer context is a different entry
        assert load_plan(path, {(64, 4096, 4096): "plain"}) == {(64, 4096, 4096)}
        ctx = {(6144, 4096): "attn-bf16", (4096, 4096): "norm-bf16", (28672, 4096): "plain",
               (4096, 14336): "norm-bf16", (128256, 4096): "plain"}
        wanted = {(M, N, K): c for (N, K), c in ctx.items()
                  for M in (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 160, 192, 256, 320, 384, 448, 512)}
        assert load_plan(DEFAULT_PLAN_FILE, wanted) == set()
    finally:
        ops.GEMM_PLAN.clear()
        ops.GEMM_PLAN.update(saved)


def test_last_layer_pruning_matches_full(tiny_engine):
    """Prefill / mixed steps continue the last layer on each sequence's last row only (after the
    QKV + RoPE + KV append every row needs): the same tokens as computing every row, in whole
    prefills, staggered mixed steps and padded steps."""
    from tests.engine_helpers import run_staggered
    eng, be = tiny_engine
    model = eng.runner.model
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    prompts = [be.prompt_ids(q) for q in ("list pods", "get nodes -o wide", "describe svc api", "top pods")]
    outs = {}
    for prune in (False, True):
        model.prune_last_layer = prune
        eng.bm.reset_prefix_cache()
        try:
            whole = [s.output_ids for s in eng.generate_blocking(prompts, params, forced_prefix=be._forced)]
            eng.bm.reset_prefix_cache()
            mixed = run_staggered(eng, prompts, params, be._forced)
        finally:
            model.prune_last_layer = True
        outs[prune] = (whole, mixed)
    assert outs[True] == outs[False]


def test_last_layer_pruning_hidden_matches():
    """Model level: the final hidden rows of a prefill step with and without pruning agree to fp32
    rounding (the pruned path's attention runs as one-query decode rows)."""
    import numpy as np
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.scheduler import Batch
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
    from ai_agent_kubectl_amd.models.llama import AttnMeta
    eng = build_engine(EngineOptions(model="tiny-llama", device="cpu", max_batch=8, use_graphs=False,
                                     kv_cache_tokens=4096, max_model_len=512))
    be = EngineLLM(eng, max_new_tokens=4)
    r = eng.runner
    seqs = [Sequence(prompt_ids=be.prompt_ids(q), params=be.params) for q in ("list pods", "scale web to 3")]
    for s in seqs:
        s.block_table, _, s.block_hashes = eng.bm.allocate_prompt(s.all_ids)
    batch = Batch(seqs, [s.total_len for s in seqs], is_decode=False, prefill_seqs=seqs)
    host = torch.from_numpy(r._pack_prefill(batch).astype(np.int32))
    T, S, mb = batch.num_tokens, len(seqs), r.max_blocks
    o = 3 * T
    meta = AttnMeta(positions=host[T:2 * T], slot_mapping=host[2 * T:3 * T],
                    block_tables=host[o + 4 * S + 1:o + 4 * S + 1 + S * mb].view(S, mb),
                    ctx_lens=host[o + S + 1:o + 2 * S + 1], logits_indices=host[o + 3 * S + 1:o + 4 * S + 1].long(),
                    is_decode=False, q_starts=host[o:o + S + 1], max_q_len=max(batch.num_query))
    hs = {}
    for prune in (False, True):
        r.model.prune_last_layer = prune
        hs[prune] = r.model.forward(host[:T], meta, r.k_cache, r.v_cache).float()
    r.model.prune_last_layer = True
    assert hs[True].shape == hs[False].shape == (S, r.model.W["embed"].shape[1])
    torch.testing.assert_close(hs[True], hs[False], atol=2e-2, rtol=2e-2)
