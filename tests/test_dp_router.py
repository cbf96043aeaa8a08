"""DP router: two engine replica processes (CPU, tiny model) behind one API process."""
import asyncio

import pytest

from ai_agent_kubectl_amd.config import Settings
from ai_agent_kubectl_amd.safety import is_safe_kubectl_command


@pytest.mark.slow
def test_dp_router_two_replicas_balanced():
    from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM
    s = Settings(LLM_BACKEND="engine", MODEL="tiny-llama", MAX_BATCH=8, MAX_NEW_TOKENS=6,
                 HIPGRAPH_BUCKETS="1,2,4,8")
    r = DPRouterLLM(s, 2, devices=["cpu", "cpu"], start_timeout=300)

    async def run():
        await r.start()
        assert all(x.up for x in r.replicas)
        outs = await asyncio.gather(*[r.generate(f"list pods in ns{i}") for i in range(12)])
        await r.close()
        return outs

    outs = asyncio.run(run())
    assert len(outs) == 12 and all(is_safe_kubectl_command(o) for o in outs)
    assert all(x.inflight == 0 for x in r.replicas)


@pytest.mark.slow
def test_api_over_dp_router():
    from fastapi.testclient import TestClient
    from ai_agent_kubectl_amd.api import create_app
    from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM
    s = Settings(LLM_BACKEND="engine", MODEL="tiny-llama", MAX_BATCH=4, MAX_NEW_TOKENS=4, RATE_LIMIT="100/minute",
                 HIPGRAPH_BUCKETS="1,2,4")
    app = create_app(s, backend=DPRouterLLM(s, 2, devices=["cpu", "cpu"], start_timeout=300))
    with TestClient(app) as c:
        r1 = c.post("/kubectl-command", json={"query": "get nodes"})
        r2 = c.post("/kubectl-command", json={"query": "get nodes"})
        assert r1.status_code == 200 and r1.json()["from_cache"] is False
        assert r2.json()["from_cache"] is True   # one global cache in the API process
        # engine metrics recorded in the replica processes reach the API's /metrics
        import time
        deadline = time.time() + 10
        while time.time() < deadline:
            m = c.get("/metrics").text
            if "llm_ttft_seconds_count 1.0" in m:
                break
            time.sleep(0.2)
        assert "llm_ttft_seconds_count 1.0" in m and "llm_tpot_seconds_count 1.0" in m
        assert "llm_kv_blocks_used" in m
