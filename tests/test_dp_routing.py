"""Least-loaded DP routing across API workers: with W workers in front of N
replicas, each worker publishes its in-flight count per replica into the shared state's load table
(runtime/shared_state.h, one row per worker) and picks the replica with the least total, so the
workers balance the replicas as one router would.  CPU only: two routers in one process stand for
two API workers (no replica is running; the table and the pick are what is tested)."""
import asyncio
import os
import uuid

import pytest

from ai_agent_kubectl_amd.config import Settings
from ai_agent_kubectl_amd.shared_state import SharedStore


def _native_ok():
    from ai_agent_kubectl_amd.runtime import native
    return native._native is not None


pytestmark = pytest.mark.skipif(not _native_ok(), reason="native runtime not built")


def test_load_table_rows_and_pick():
    name = "/ka_load_%s" % uuid.uuid4().hex[:8]
    a, b = SharedStore(name, 16), SharedStore(name, 16)
    try:
        a.load_set(0, 0, 5)
        b.load_set(1, 1, 2)
        b.load_set(1, 0, 1)
        assert a.load_total(0) == 6 and a.load_total(1) == 2
        assert a.load_pick(2, 0b11) == 1          # least total
        assert a.load_pick(2, 0b01) == 0          # only replica 0 live
        assert a.load_pick(2, 0) == -1
        a.load_clear_worker(1)                    # a respawned worker's row starts at zero
        assert a.load_total(0) == 5 and a.load_total(1) == 0
        assert a.load_pick(3, 0b111) == 1         # ties: lowest index (1 and 2 both empty)
    finally:
        SharedStore.unlink(name)


def test_routers_balance_over_each_others_load(tmp_path):
    from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM, ReplicaDirectory
    name = "ka_route_%s" % uuid.uuid4().hex[:8]
    s = Settings(LLM_BACKEND="engine", MODEL="tiny-llama", SHARED_STATE=name, CACHE_MAXSIZE=64)
    eps = ReplicaDirectory([str(tmp_path / "r0.sock"), str(tmp_path / "r1.sock")], b"key")
    r0 = DPRouterLLM(s, 2, endpoints=eps, client_id=0)
    r1 = DPRouterLLM(s, 2, endpoints=eps, client_id=1)
    try:
        for r in (r0, r1):
            for rep in r.replicas:
                rep.up = True
        # worker 0 has 3 requests on replica 0; worker 1 (idle itself) must route to replica 1
        r0.replicas[0].inflight = 3
        r0._publish_load(r0.replicas[0])
        assert r1._pick(r1.replicas).idx == 1
        # without the shared table each worker would only see its own (empty) counts
        assert min(r1.replicas, key=lambda x: x.inflight).idx == 0
        # replica 1 goes down: everything routes to replica 0
        assert r1._pick([r1.replicas[0]]).idx == 0
        # the load drains: worker 0 publishes 0 and the tie goes to the lower index
        r0.replicas[0].inflight = 0
        r0._publish_load(r0.replicas[0])
        assert r1._pick(r1.replicas).idx == 0
    finally:
        asyncio.run(r0.close())
        asyncio.run(r1.close())
        SharedStore.unlink(name)
