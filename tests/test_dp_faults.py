"""DP replica faults (parallel/dp.py): one replica's engine exits mid-step (fault
injection KA_FAULT_REPLICA=0 KA_FAULT_STEP=<n>:exit, the path a fatal engine fault takes): only the
requests in flight on that replica fail with LLMUnavailableError (HTTP 503), the other replica keeps
serving, the supervisor respawns the dead one in a fresh process and the router reconnects to it.
CPU, tiny model."""
import asyncio
import os
import time

import pytest

from ai_agent_kubectl_amd.config import Settings
from ai_agent_kubectl_amd.llm.base import LLMUnavailableError
from ai_agent_kubectl_amd.safety import is_safe_kubectl_command


@pytest.mark.slow
def test_replica_crash_fails_only_its_requests_and_comes_back(monkeypatch):
    from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM
    monkeypatch.setenv("KA_FAULT_REPLICA", "0")
    monkeypatch.setenv("KA_FAULT_STEP", "2:exit")
    s = Settings(LLM_BACKEND="engine", MODEL="tiny-llama", MAX_BATCH=8, MAX_NEW_TOKENS=8, HIPGRAPH_BUCKETS="1,2,4,8")
    r = DPRouterLLM(s, 2, devices=["cpu", "cpu"], start_timeout=300)

    async def one(q):
        try:
            return await r.generate(q)
        except LLMUnavailableError as e:
            return e

    async def run():
        await r.start()
        assert all(x.up for x in r.replicas)
        pids0 = {h["pid"] for h in await r.control("health")}
        first = await asyncio.gather(*[one(f"list pods in ns{i}") for i in range(12)])
        failed = [x for x in first if isinstance(x, LLMUnavailableError)]
        ok = [x for x in first if isinstance(x, str)]
        # replica 0 died with its requests in flight: those (and only those) are 503s
        assert failed and ok, first
        assert all("replica 0 died" in str(e) for e in failed)
        assert all(is_safe_kubectl_command(x) for x in ok)
        # new requests meanwhile go to the live replica
        mid = await asyncio.gather(*[one(f"get svc {i}") for i in range(4)])
        assert all(isinstance(x, str) for x in mid), mid
        # the supervisor respawns replica 0; the router reconnects
        deadline = time.time() + 120
        while time.time() < deadline and not (r.replicas[0].up and r.reconnects >= 1):
            await asyncio.sleep(0.2)
        assert r.replicas[0].up and r.supervisor.respawned >= 1
        health = await r.control("health")
        assert len(health) == 2 and all(h["healthy"] for h in health)
        assert {h["pid"] for h in health} != pids0
        after = await asyncio.gather(*[one(f"describe deploy {i}") for i in range(12)])
        assert all(isinstance(x, str) and is_safe_kubectl_command(x) for x in after), after
        await r.close()

    asyncio.run(run())
    assert not any(p.is_alive() for p in r.supervisor.procs if p is not None)


@pytest.mark.slow
def test_lost_tp_worker_makes_replica_exit_and_respawn(monkeypatch):
    """DP=1 x TP=2 replica on the CPU (gloo): the TP worker rank is killed while the engine is idle.
    Rank 0's watchdog sees its heartbeat stop, fails what is in flight and exits with EXIT_FATAL
    (engine.mark_unhealthy with exit_on_fatal), so the supervisor respawns the whole TP group: requests
    meanwhile answer 503 (LLMUnavailableError), and afterwards the respawned group serves again."""
    import psutil

    from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM
    monkeypatch.setenv("WORKER_HEARTBEAT_INTERVAL_S", "0.2")
    monkeypatch.setenv("WORKER_HEARTBEAT_TIMEOUT_S", "3")
    monkeypatch.delenv("KA_FAULT_STEP", raising=False)
    s = Settings(LLM_BACKEND="engine", MODEL="tiny-llama", MAX_BATCH=4, MAX_NEW_TOKENS=6, HIPGRAPH_BUCKETS="1,2,4")
    r = DPRouterLLM(s, 1, devices=[["cpu", "cpu"]], start_timeout=300)

    async def one(q):
        try:
            return await r.generate(q)
        except LLMUnavailableError as e:
            return e

    async def run():
        await r.start()
        assert r.replicas[0].up
        ok = await asyncio.gather(*[one(f"list pods in ns{i}") for i in range(3)])
        assert all(isinstance(x, str) and is_safe_kubectl_command(x) for x in ok), ok
        rep = psutil.Process(r.supervisor.procs[0].pid)
        workers = []
        deadline = time.time() + 30
        while not workers and time.time() < deadline:   # ka-tp-0.1: parallel/dp.py set_proc_name
            workers = [c for c in rep.children(recursive=True) if c.name().startswith("ka-tp")]
            await asyncio.sleep(0.1)
        assert workers, [c.name() for c in rep.children(recursive=True)]
        for w in workers:
            w.kill()
        # the replica exits on the watchdog verdict; until it is back, misses answer 503
        deadline = time.time() + 60
        while time.time() < deadline and r.supervisor.procs[0].is_alive() and r.supervisor.procs[0].pid == rep.pid:
            await asyncio.sleep(0.1)
        assert r.supervisor.procs[0].pid != rep.pid or r.supervisor.procs[0].exitcode == 75
        down = await one("get nodes")
        assert isinstance(down, (str, LLMUnavailableError))
        deadline = time.time() + 180
        while time.time() < deadline and not (r.replicas[0].up and r.supervisor.respawned >= 1):
            await asyncio.sleep(0.2)
        assert r.replicas[0].up and r.supervisor.respawned >= 1
        after = await asyncio.gather(*[one(f"describe deploy {i}") for i in range(3)])
        assert all(isinstance(x, str) and is_safe_kubectl_command(x) for x in after), after
        await r.close()

    asyncio.run(run())
    assert not any(p.is_alive() for p in r.supervisor.procs if p is not None)


@pytest.mark.slow
def test_unhealthy_replica_is_routed_around():
    """A replica whose engine reports unhealthy (without exiting) is pushed to the router as
    ('health', idx, False): new requests go to the other replica, and the replica itself rejects
    any 'gen' with an error instead of queueing it."""
    from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM, _Replica
    s = Settings(LLM_BACKEND="engine", MODEL="tiny-llama", MAX_BATCH=4, MAX_NEW_TOKENS=6, HIPGRAPH_BUCKETS="1,2,4")
    r = DPRouterLLM(s, 2, devices=["cpu", "cpu"], start_timeout=300)

    async def run():
        await r.start()
        r._dispatch(r.replicas[0], "health", 0, False)
        assert not r.replicas[0].healthy and r.healthy()
        outs = await asyncio.gather(*[r.generate(f"get pods {i}") for i in range(6)])
        assert all(is_safe_kubectl_command(x) for x in outs)
        assert r.replicas[0].inflight == 0
        r._dispatch(r.replicas[1], "health", 1, False)
        assert not r.healthy()
        with pytest.raises(LLMUnavailableError):
            await r.generate("get svc")
        r._dispatch(r.replicas[0], "health", 0, True)
        assert isinstance(await r.generate("get svc"), str)
        await r.close()

    asyncio.run(run())
