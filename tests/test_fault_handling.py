"""Engine fault handling: a failing step answers 503 for its in-flight requests, a
recoverable fault leaves the engine serving again, a fatal one (a one-shot TP collective that timed
out waiting for a peer, csrc/allreduce.hip's error word) never returns the step's stale tokens and
stops the engine (exit for the supervisor).  The reference's only recovery is the container
restart policy (`/root/reference/docker-compose.yml:14`)."""
import asyncio

import httpx
import pytest
import torch

from ai_agent_kubectl_amd.engine.engine import EXIT_FATAL
from ai_agent_kubectl_amd.engine.runner import CollectiveTimeout


@pytest.fixture(scope="module")
def tiny():
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
    eng = build_engine(EngineOptions(model="tiny-llama", device="cpu", max_batch=8, graph_buckets=(1, 2, 4, 8),
                                     kv_cache_tokens=8192, max_model_len=512))
    return eng, EngineLLM(eng, max_new_tokens=6)


def _app(be):
    from ai_agent_kubectl_amd.api import create_app
    from ai_agent_kubectl_amd.config import Settings
    return create_app(Settings(RATE_LIMIT="100000/minute", CACHE_TTL=0), backend=be)


async def _post_all(app, be, queries):
    await be.start()
    try:
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            return await asyncio.gather(*[c.post("/kubectl-command", json={"query": q}) for q in queries])
    finally:
        await be.close()


class _FakeOneShot:
    """Stands in for parallel/custom_allreduce.OneShotAllReduce: only its state word matters here."""

    def __init__(self, err: int):
        self.state = torch.tensor([0, 0, err, 0], dtype=torch.int32)


def test_recoverable_step_fault_fails_inflight_then_serves_again(tiny):
    eng, be = tiny
    app = _app(be)
    eng.fault_step, eng.fault_kind = eng.steps, "error"
    r0 = eng.recoveries
    try:
        rs = asyncio.run(_post_all(app, be, ["list pods", "get nodes", "top pods"]))
        codes = [r.status_code for r in rs]
        # the requests in the faulting step get 503; any admitted after the recovery are served
        assert codes[0] == 503 and set(codes) <= {200, 503}, codes
        assert "injected engine step fault" in rs[0].json()["detail"]
        assert eng.healthy and eng.recoveries == r0 + 1
        rs = asyncio.run(_post_all(app, be, ["list pods", "describe svc api"]))
        assert [r.status_code for r in rs] == [200, 200]
        assert all(r.json()["kubectl_command"].startswith("kubectl ") for r in rs)
    finally:
        eng.fault_step = -1
        eng.healthy = True
    assert all(eng.bm.ref_count(b) == 0 for b in range(eng.bm.num_blocks))


def test_collective_timeout_is_503_never_200_and_fatal(tiny):
    """The one-shot collectives' error word set (a peer never arrived) turns the step into a
    CollectiveTimeout at readback: the requests get 503 (not the stale tokens with 200), the engine
    stays unhealthy (/ready 503) and, with exit_on_fatal, exits with EXIT_FATAL."""
    from fastapi.testclient import TestClient
    eng, be = tiny
    app = _app(be)
    comm = eng.runner.comm
    exits = []
    saved_exit, saved_flag = eng._exit, eng.exit_on_fatal
    comm.custom_ar = _FakeOneShot(err=1)
    eng._exit, eng.exit_on_fatal = exits.append, True
    try:
        rs = asyncio.run(_post_all(app, be, ["list pods", "get svc"]))
        assert [r.status_code for r in rs] == [503, 503]
        assert "peer never arrived" in rs[0].json()["detail"]
        assert not eng.healthy and isinstance(eng.last_error, CollectiveTimeout)
        assert exits == [EXIT_FATAL]
        with TestClient(app) as c:
            assert c.get("/ready").status_code == 503
            assert c.post("/kubectl-command", json={"query": "list all pods now"}).status_code == 503
    finally:
        del comm.custom_ar
        eng._exit, eng.exit_on_fatal = saved_exit, saved_flag
        eng.healthy, eng.last_error = True, None


def test_persistent_stall_is_503_then_chain_serves(tiny):
    """The persistent batch-1 kernel's error word set (a grid wait ran out) turns the step into a
    recoverable PersistentStall at readback: the request gets 503 (never the stale tokens), the
    engine recovers with the persistent path switched off, and the next request is served."""
    from ai_agent_kubectl_amd.engine.runner import PersistentStall
    eng, be = tiny
    app = _app(be)
    r, m = eng.runner, eng.runner.model
    word = torch.tensor([1], dtype=torch.int32)
    saved = (r._persistent_step, m.persistent_err_word, m.persistent)
    r._persistent_step = lambda Bp: Bp == 1
    m.persistent_err_word = lambda: word
    m.persistent = True
    r0 = eng.recoveries
    try:
        rs = asyncio.run(_post_all(app, be, ["list pods in kube-system"]))
        assert rs[0].status_code == 503, rs[0].text
        assert "grid wait timeout" in rs[0].json()["detail"]
        assert isinstance(eng.last_error, PersistentStall) and not eng.is_fatal(eng.last_error)
        assert eng.healthy and eng.recoveries == r0 + 1 and m.persistent is False
        word.zero_()
        rs = asyncio.run(_post_all(app, be, ["get nodes please"]))
        assert rs[0].status_code == 200
    finally:
        r._persistent_step, m.persistent_err_word, m.persistent = saved
        eng.healthy, eng.last_error = True, None


class _FakeGraph:
    """Stands in for a captured bucket-1 decode graph: replay runs the step eagerly."""
    def __init__(self, runner, B):
        self.runner, self.B, self.replays = runner, B, 0

    def replay(self):
        self.replays += 1
        self.runner._decode_forward(self.B)


def test_persistent_stall_drops_the_persistent_graph(tiny):
    """with decode graphs on, the bucket-1 graph captured with the persistent kernel
    keeps launching it after model.persistent is switched off.  The runner must keep reading that
    graph's error word while it exists, and a stall must drop the graph (batch 1 then runs the kernel
    chain eagerly) instead of replaying stale results without an error."""
    from ai_agent_kubectl_amd.engine.runner import PersistentStall
    eng, be = tiny
    app = _app(be)
    r, m = eng.runner, eng.runner.model
    word = torch.tensor([0], dtype=torch.int32)
    saved = (m.persistent_err_word, m.persistent, dict(r.graphs), dict(r.graph_persistent))
    g = _FakeGraph(r, 1)
    r.graphs[1] = g
    r.graph_persistent[1] = True
    m.persistent_err_word = lambda: word
    m.persistent = False          # the model's flag alone no longer decides: the graph holds the kernel
    stalls0 = r.stats["persistent_stalls"]
    try:
        assert r._persistent_step(1)
        rs = asyncio.run(_post_all(app, be, ["list pods in default"]))
        assert rs[0].status_code == 200 and g.replays > 0
        word.fill_(1)
        rs = asyncio.run(_post_all(app, be, ["list pods in kube-public"]))
        assert rs[0].status_code == 503, rs[0].text
        assert isinstance(eng.last_error, PersistentStall)
        assert 1 not in r.graphs and 1 not in r.graph_persistent
        assert r.stats["persistent_stalls"] == stalls0 + 1
        assert not r._persistent_step(1)
        n = g.replays
        rs = asyncio.run(_post_all(app, be, ["get deployments now"]))   # word still set: not read any more
        assert rs[0].status_code == 200 and g.replays == n
    finally:
        m.persistent_err_word, m.persistent = saved[0], saved[1]
        r.graphs.clear()
        r.graphs.update(saved[2])
        r.graph_persistent.clear()
        r.graph_persistent.update(saved[3])
        eng.healthy, eng.last_error = True, None


def test_persistent_stall_retires_graph_until_synchronized(tiny):
    """a stall must not destroy the persistent graph while the engine may still have
    a chained replay of it queued.  The graph leaves service at once (no new replay can pick it) but is
    only released by health_check(), after its device synchronize."""
    from ai_agent_kubectl_amd.engine.runner import PersistentStall
    eng, be = tiny
    r, m = eng.runner, eng.runner.model
    saved = (m.persistent, dict(r.graphs), dict(r.graph_persistent))
    g = _FakeGraph(r, 2)
    r.graphs[2] = g
    r.graph_persistent[2] = True
    try:
        with pytest.raises(PersistentStall):
            r._check_err(torch.tensor([0, 1], dtype=torch.int32))
        assert 2 not in r.graphs and 2 not in r.graph_persistent
        assert any(x is g for x in r._retired_graphs), "graph released before a synchronize"
        r.health_check()
        assert not r._retired_graphs
    finally:
        m.persistent = saved[0]
        r.graphs.clear()
        r.graphs.update(saved[1])
        r.graph_persistent.clear()
        r.graph_persistent.update(saved[2])
        r._retired_graphs.clear()


def test_error_word_clear_is_transparent(tiny):
    """A zero error word changes nothing (the readback rides behind every step's tokens)."""
    eng, be = tiny
    from ai_agent_kubectl_amd.engine.sequence import SamplingParams
    params = SamplingParams(max_new_tokens=5, ignore_eos=True)
    ids = be.prompt_ids("list pods in prod")
    eng.bm.reset_prefix_cache()
    plain = eng.generate_blocking([ids], params, forced_prefix=be._forced)[0].output_ids
    eng.runner.comm.custom_ar = _FakeOneShot(err=0)
    try:
        eng.bm.reset_prefix_cache()
        with_word = eng.generate_blocking([ids], params, forced_prefix=be._forced)[0].output_ids
    finally:
        del eng.runner.comm.custom_ar
    assert plain == with_word


def test_repeated_faults_become_fatal(tiny):
    eng, be = tiny
    saved = eng.max_recoveries, list(eng._recovery_times)
    eng.max_recoveries = 1
    eng._recovery_times = []
    try:
        assert eng._recover(RuntimeError("transient")) and eng.healthy
        assert not eng._recover(RuntimeError("transient again"))
        assert eng.is_fatal(RuntimeError("HIP error: an illegal memory access was encountered"))
        assert eng.is_fatal(CollectiveTimeout("x"))
        assert not eng.is_fatal(RuntimeError("some host-side bug"))
    finally:
        eng.max_recoveries, eng._recovery_times = saved
        eng.healthy = True


def test_watchdog_verdict_with_exit_on_fatal_fails_inflight_and_exits():
    """engine.mark_unhealthy (the TP watchdog's callback) with exit_on_fatal: in-flight requests are
    failed with the verdict and the process exits with EXIT_FATAL (no minutes-long collective wait)."""
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.sequence import SamplingParams
    eng = build_engine(EngineOptions(model="tiny-llama", device="cpu", max_batch=4, graph_buckets=(1, 2, 4),
                                     kv_cache_tokens=4096, max_model_len=256))
    exits, done, flushed = [], [], []
    eng._exit = exits.append
    eng.exit_on_fatal = True
    eng.step_end_hooks.append(lambda: flushed.append(1))
    seq = eng.submit([5, 6, 7], SamplingParams(max_new_tokens=4), done.append)
    eng._drain_inbox()                       # admitted, not yet stepped (the engine thread is "blocked")
    eng.mark_unhealthy("TP/EP worker rank 1 heartbeat lost")
    assert exits == [EXIT_FATAL] and not eng.healthy
    assert done == [seq] and seq.finish_reason == "error" and "heartbeat lost" in str(seq.error)
    assert flushed
    eng2_exits = []
    eng.exit_on_fatal, eng._exit = False, eng2_exits.append
    eng.mark_unhealthy("again")              # without exit_on_fatal: only unhealthy
    assert eng2_exits == []


def test_persistent_default_off_on_a_shared_gpu(monkeypatch):
    """the persistent kernel's grid barriers need the whole GPU, so the default
    (auto) turns it off when several replicas share one device (KA_GPU_MEM_SHARE < 1, set by
    parallel/dp.py); an explicit KA_PERSISTENT_DECODE=0/1 wins either way."""
    from ai_agent_kubectl_amd.models.llama import persistent_default
    monkeypatch.delenv("KA_PERSISTENT_DECODE", raising=False)
    monkeypatch.delenv("KA_GPU_MEM_SHARE", raising=False)
    assert persistent_default()
    monkeypatch.setenv("KA_GPU_MEM_SHARE", "0.5")
    assert not persistent_default()
    monkeypatch.setenv("KA_PERSISTENT_DECODE", "1")
    assert persistent_default()
    monkeypatch.setenv("KA_GPU_MEM_SHARE", "1.0")
    monkeypatch.setenv("KA_PERSISTENT_DECODE", "0")
    assert not persistent_default()
