"""API golden tests: SURVEY.md Appendix A transcripts (reference app.py run unmodified).

Timestamps are masked; everything else is compared byte-for-byte.  The one deliberate deviation is
quirk Q1 (/execute error paths), covered both in fixed mode (default) and COMPAT_STRICT_500 mode.
"""
import asyncio
import json
import re

import pytest
from fastapi.testclient import TestClient

from ai_agent_kubectl_amd.api import create_app
from ai_agent_kubectl_amd.config import Settings
from ai_agent_kubectl_amd.llm.stub import StubRuleLLM

TS = re.compile(r'"(start_time|end_time)":"[0-9T:.\-]+"')
DUR = re.compile(r'"duration_ms":[0-9.e\-]+')


def mask(text):
    return DUR.sub('"duration_ms":D', TS.sub(r'"\1":"T"', text))


def make(backend=None, **kw):
    kw.setdefault("API_AUTH_KEY", "k")
    kw.setdefault("RATE_LIMIT", "1000/minute")
    s = Settings(**kw)
    app = create_app(s, backend=StubRuleLLM() if backend is None else backend)
    return TestClient(app, raise_server_exceptions=False), app


H = {"X-API-Key": "k"}


def test_generate_and_cache_hit():
    c, _ = make()
    r = c.post("/kubectl-command", json={"query": "list   all\npods"}, headers=H)
    assert r.status_code == 200
    assert r.headers["content-type"] == "application/json"
    assert mask(r.text) == ('{"kubectl_command":"kubectl get pods","execution_result":null,"execution_error":null,'
                            '"from_cache":false,"metadata":{"start_time":"T","end_time":"T","duration_ms":D,'
                            '"success":true,"error_type":null,"error_code":null}}')
    assert '"duration_ms":0.0' in r.text
    r = c.post("/kubectl-command", json={"query": "list all pods"}, headers=H)
    assert r.json()["from_cache"] is True and r.json()["kubectl_command"] == "kubectl get pods"


def test_timestamps_are_naive_isoformat():
    c, _ = make()
    md = c.post("/kubectl-command", json={"query": "get nodes"}, headers=H).json()["metadata"]
    assert re.fullmatch(r"\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d(\.\d{6})?", md["start_time"])


def test_min_length_422():
    c, _ = make()
    r = c.post("/kubectl-command", json={"query": "ab"}, headers=H)
    assert r.status_code == 422
    assert r.text == ('{"detail":[{"type":"string_too_short","loc":["body","query"],"msg":"String should have '
                      'at least 3 characters","input":"ab","ctx":{"min_length":3}}]}')


def test_wrong_type_422():
    c, _ = make(API_AUTH_KEY=None)
    r = c.post("/kubectl-command", json={"query": 123})
    assert r.status_code == 422
    assert r.text == ('{"detail":[{"type":"string_type","loc":["body","query"],"msg":"Input should be a valid '
                      'string","input":123}]}')


def test_auth_missing_and_invalid_before_validation():
    c, _ = make()
    r = c.post("/kubectl-command", json={"query": "list pods"})
    assert (r.status_code, r.text) == (401, '{"detail":"Missing X-API-Key header"}')
    r = c.post("/kubectl-command", json={"q": "abc"}, headers={"X-API-Key": "z"})
    assert (r.status_code, r.text) == (401, '{"detail":"Invalid API Key"}')


def test_auth_disabled_whitespace_query_and_extra_field():
    c, app = make(API_AUTH_KEY=None)
    r = c.post("/kubectl-command", json={"query": "    "})
    assert r.status_code == 200
    assert "" in app.state.service.cache  # quirk Q5: cache key ""
    r = c.post("/kubectl-command", json={"query": "get nodes", "execute": True})
    assert r.status_code == 200 and r.json()["kubectl_command"] == "kubectl get nodes"


def test_unsafe_generation_422():
    c, _ = make(StubRuleLLM(raw="rm -rf /"))
    r = c.post("/kubectl-command", json={"query": "delete everything"}, headers=H)
    assert (r.status_code, r.text) == (
        422, '{"detail":"LLM generated unsafe command: Generated command failed safety checks: rm -rf /"}')


def test_fence_strip_and_bash_fence_422():
    c, _ = make(StubRuleLLM(raw="```kubectl get svc```"))
    r = c.post("/kubectl-command", json={"query": "services"}, headers=H)
    assert r.status_code == 200 and r.json()["kubectl_command"] == "kubectl get svc"
    c, _ = make(StubRuleLLM(raw="```bash\nkubectl get svc\n```"))
    r = c.post("/kubectl-command", json={"query": "services"}, headers=H)
    assert r.status_code == 422
    assert r.text == ('{"detail":"LLM generated unsafe command: Generated command failed safety checks: '
                      'bash\\nkubectl get svc"}')


def test_llm_timeout_504():
    c, _ = make(StubRuleLLM(delay_s=2.0), LLM_TIMEOUT=1)
    r = c.post("/kubectl-command", json={"query": "list pods"}, headers=H)
    assert (r.status_code, r.text) == (504, '{"detail":"LLM request timed out"}')


def test_llm_error_500_and_no_cache_store():
    c, app = make(StubRuleLLM(error=RuntimeError("boom")))
    r = c.post("/kubectl-command", json={"query": "list pods"}, headers=H)
    assert (r.status_code, r.text) == (500, '{"detail":"Error processing query with LLM: boom"}')
    assert len(app.state.service.cache) == 0


def test_chain_none_503_but_cache_hits_still_work():
    s = Settings(API_AUTH_KEY="k", RATE_LIMIT="1000/minute")
    app = create_app(s, backend=None)
    app.state.service.cache["list pods"] = "kubectl get pods"
    c = TestClient(app)
    r = c.post("/kubectl-command", json={"query": "get nodes"}, headers=H)
    assert (r.status_code, r.text) == (503, '{"detail":"LLM Chain not initialized"}')
    r = c.post("/kubectl-command", json={"query": "list pods"}, headers=H)
    assert r.status_code == 200 and r.json()["from_cache"] is True


def test_execute_table_raw_error(fake_kubectl):
    c, _ = make()
    r = c.post("/execute", json={"execute": "kubectl get pods"}, headers=H)
    assert r.status_code == 200
    assert mask(r.text) == (
        '{"kubectl_command":"kubectl get pods","execution_result":{"type":"table","data":[{"name":"nginx-1",'
        '"ready":"1/1","status":"Running","restarts":"0","age":"5m"},{"name":"redis-0","ready":"1/1",'
        '"status":"Running","restarts":"2","age":"1h"}]},"execution_error":null,"from_cache":false,'
        '"metadata":{"start_time":"T","end_time":"T","duration_ms":D,"success":true,"error_type":null,'
        '"error_code":null}}')
    r = c.post("/execute", json={"execute": "kubectl get ns"}, headers=H)
    assert r.json()["execution_result"] == {"type": "raw", "data": "default"}
    r = c.post("/execute", json={"execute": "kubectl get foo"}, headers=H)
    assert mask(r.text) == (
        '{"kubectl_command":"kubectl get foo","execution_result":null,"execution_error":{"type":"kubectl_error",'
        '"code":"1","message":"error: the server doesn\'t have a resource type \\"foo\\""},"from_cache":false,'
        '"metadata":{"start_time":"T","end_time":"T","duration_ms":D,"success":false,"error_type":"kubectl_error",'
        '"error_code":"1"}}')


@pytest.mark.parametrize("cmd", ["kubectl get pods; rm", "kubectl get 'pods", "ls -la", "kubectl get $(x)"])
def test_execute_safety_400(cmd):
    c, _ = make()
    r = c.post("/execute", json={"execute": cmd}, headers=H)
    assert (r.status_code, r.text) == (400, '{"detail":"Command failed safety checks"}')


def test_execute_timeout_fixed_and_strict(fake_kubectl):
    c, _ = make(EXECUTION_TIMEOUT=1)
    r = c.post("/execute", json={"execute": "kubectl sleep"}, headers=H)
    body = r.json()
    assert r.status_code == 200
    assert body["execution_error"] == {"type": "timeout", "message": "Command execution timed out after 1s"}
    assert body["metadata"]["success"] is False and body["metadata"]["error_type"] == "timeout"
    c, _ = make(EXECUTION_TIMEOUT=1, COMPAT_STRICT_500=True)
    r = c.post("/execute", json={"execute": "kubectl sleep"}, headers=H)
    assert r.status_code == 500 and r.headers["content-type"].startswith("text/plain")
    assert r.text == "Internal Server Error"


@pytest.mark.parametrize("cmd", ["kubectl get pods", "kubectl get pods | grep x", "kubectl get pods\nrm -rf /",
                                 "  kubectl get pods"])
def test_execute_not_found_passes_validator(no_kubectl, cmd):
    c, _ = make(API_AUTH_KEY=None)
    r = c.post("/execute", json={"execute": cmd})
    assert r.status_code == 200
    assert r.json()["execution_error"]["type"] == "not_found"
    c, _ = make(API_AUTH_KEY=None, COMPAT_STRICT_500=True)
    r = c.post("/execute", json={"execute": cmd})
    assert r.status_code == 500


def test_health_405_404():
    c, _ = make()
    assert c.get("/health").text == '{"status":"healthy"}'
    r = c.get("/kubectl-command")
    assert (r.status_code, r.text) == (405, '{"detail":"Method Not Allowed"}')
    r = c.get("/nope")
    assert (r.status_code, r.text) == (404, '{"detail":"Not Found"}')


def test_rate_limit_decorated_route_after_auth_and_validation():
    c, _ = make(RATE_LIMIT="2/minute")
    # 401 and 422 do not consume the route bucket
    assert c.post("/kubectl-command", json={"query": "list pods"}).status_code == 401
    assert c.post("/kubectl-command", json={"query": "x"}, headers=H).status_code == 422
    assert c.post("/kubectl-command", json={"query": "list pods"}, headers=H).status_code == 200
    assert c.post("/kubectl-command", json={"query": "list pods"}, headers=H).status_code == 200
    r = c.post("/kubectl-command", json={"query": "list pods"}, headers=H)
    assert (r.status_code, r.text) == (429, '{"error":"Rate limit exceeded: 2 per 1 minute"}')
    assert "x-ratelimit-limit" not in {k.lower() for k in r.headers}
    # separate bucket per route
    assert c.post("/execute", json={"execute": "kubectl get pods; x"}, headers=H).status_code == 400


def test_rate_limit_middleware_default_routes():
    c, _ = make(RATE_LIMIT="3 per minute")
    for _ in range(3):
        assert c.get("/health").status_code == 200
    r = c.get("/health")
    assert (r.status_code, r.text) == (429, '{"error":"Rate limit exceeded: 3 per 1 minute"}')
    # /metrics has its own bucket; unmatched paths are never limited
    assert c.get("/metrics").status_code == 200
    for _ in range(5):
        assert c.get("/nope").status_code == 404


def test_metrics_names_and_labels():
    c, _ = make()
    c.post("/kubectl-command", json={"query": "list pods"}, headers=H)
    c.post("/kubectl-command", json={"query": "list pods"})
    c.get("/nope")
    text = c.get("/metrics").text
    for name in ["http_requests_total", "http_request_size_bytes", "http_response_size_bytes",
                 "http_request_duration_seconds_bucket", "http_request_duration_highr_seconds_bucket",
                 "process_cpu_seconds_total", "python_info", "kubectl_agent_cache_misses_total"]:
        assert name in text, name
    assert re.search(r'http_requests_total\{[^}]*handler="/kubectl-command"[^}]*status="2xx"[^}]*\} 1\.0', text)
    assert re.search(r'http_requests_total\{[^}]*handler="/kubectl-command"[^}]*status="4xx"[^}]*\} 1\.0', text)
    assert re.search(r'http_requests_total\{[^}]*handler="none"', text)
    assert 'le="60.0"' in text and 'http_request_duration_seconds_bucket{handler="/kubectl-command",le="0.5"' in \
        text.replace('method="POST",', '')
    text2 = c.get("/metrics").text
    assert re.search(r'http_requests_total\{[^}]*handler="/metrics"', text2)


def test_openapi_and_docs():
    c, _ = make()
    spec = c.get("/openapi.json").json()
    assert spec["info"] == {"title": "Kubectl NLP Service", "version": "1.0.0"}
    assert set(spec["paths"]) >= {"/kubectl-command", "/execute", "/health", "/metrics"}
    assert c.get("/docs").status_code == 200
    assert c.get("/redoc").status_code == 200


def test_fault_injection_and_ready():
    c, _ = make(FAULT_LLM_ERROR="unavailable")
    r = c.post("/kubectl-command", json={"query": "list pods"}, headers=H)
    assert r.status_code == 503
    c, _ = make(FAULT_LLM_DELAY_MS=1500, LLM_TIMEOUT=1)
    r = c.post("/kubectl-command", json={"query": "list pods"}, headers=H)
    assert (r.status_code, r.text) == (504, '{"detail":"LLM request timed out"}')
    c, _ = make(FAULT_LLM_ERROR="kaboom")
    assert c.post("/kubectl-command", json={"query": "x y z"}, headers=H).json() == {
        "detail": "Error processing query with LLM: kaboom"}
    assert c.get("/ready").status_code == 200
    s = Settings(RATE_LIMIT="100/minute")
    assert TestClient(create_app(s, backend=None)).get("/ready").status_code == 503


def test_metrics_batched_updates_match_per_request_observe():
    """HTTP metrics are applied in bulk (every 256 requests and before every /metrics render): the
    scraped counts, sums and histogram buckets equal what per-request observe() calls give."""
    from prometheus_client import CollectorRegistry, Histogram

    from ai_agent_kubectl_amd.metrics import HIGHR_BUCKETS, LOWR_BUCKETS
    c, _ = make()
    n = 300   # crosses the 256-request flush boundary
    for i in range(n):
        assert c.post("/kubectl-command", json={"query": f"list pods {i % 7}"}, headers=H).status_code == 200
    app = c.app
    mw = app.middleware_stack
    while mw is not None and not hasattr(mw, "flush"):
        mw = getattr(mw, "app", None)
    assert mw is not None
    durs = [d for (_, _, _, d) in mw._pending]
    assert 0 < len(durs) < 256          # the last requests are still pending before the scrape
    text = c.get("/metrics").text
    assert re.search(r'http_requests_total\{handler="/kubectl-command",method="POST",status="2xx"\} 300\.0', text)
    assert re.search(r'http_request_size_bytes_count\{handler="/kubectl-command"\} 300\.0', text)
    assert re.search(r'http_request_duration_seconds_count\{handler="/kubectl-command",method="POST"\} 300\.0', text)
    assert re.search(r'http_request_duration_highr_seconds_count (\d+)\.0', text)
    # bucket placement: first upper bound >= value, exactly as Histogram.observe
    reg = CollectorRegistry()
    h = Histogram("x", "x", buckets=HIGHR_BUCKETS, registry=reg)
    lo = Histogram("y", "y", buckets=LOWR_BUCKETS, registry=reg)
    for v in (0.0, 0.01, 0.0100001, 0.5, 59.9, 60.0, 61.0):
        h.observe(v)
        lo.observe(v)
    import bisect
    got = [0] * len(h._upper_bounds)
    for v in (0.0, 0.01, 0.0100001, 0.5, 59.9, 60.0, 61.0):
        got[bisect.bisect_left(h._upper_bounds, v)] += 1
    assert got == [b.get() for b in h._buckets]


def test_generated_reply_template_is_byte_identical():
    """The /kubectl-command success reply template == the generic json.dumps path, byte for byte."""
    from ai_agent_kubectl_amd.api.app import _command_body, _generated_json, _json
    for cmd in ["kubectl get pods", 'kubectl get pods -l "app=x"', "kubectl get pods -o jsonpath='{.items}'",
                "kubectl get ns \\\\ x", "kubectl describe pod ünïcødé-π", "kubectl get pods\\n--all", "kubectl   x"]:
        for hit in (False, True):
            md = {"metadata": {"start_time": "2026-10-16T12:00:00.123456", "end_time": "2026-10-16T12:00:00.123999",
                               "duration_ms": 0.0, "success": True}}
            assert _generated_json(cmd, hit, md["metadata"]["start_time"], md["metadata"]["end_time"]) == \
                _json(_command_body(cmd, hit, md)).body
