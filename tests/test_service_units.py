"""Unit tests for the CPU service pieces (SURVEY.md §4.3 'unit' row)."""
import asyncio
import shlex

import pytest
from hypothesis import given, settings as hsettings, strategies as st

from ai_agent_kubectl_amd.cache import TTLCache
from ai_agent_kubectl_amd.config import Settings, load_dotenv, parse_dotenv
from ai_agent_kubectl_amd.executor import execute_command_async, parse_kubectl_output
from ai_agent_kubectl_amd.llm.stub import rule_translate
from ai_agent_kubectl_amd.ratelimit import FixedWindowLimiter, RateLimitExceeded, parse_many
from ai_agent_kubectl_amd.safety import (UnsafeCommandError, is_safe_kubectl_command, parse_llm_output,
                                         sanitize_query)


class Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


# ---------------- safety ----------------
def test_sanitize():
    assert sanitize_query("  list \t all\r\npods  ") == "list all pods"
    assert sanitize_query("    ") == ""


@pytest.mark.parametrize("bad", [";", "&&", "||", "`", "$", "(", ")", "<", ">"])
def test_blacklist(bad):
    assert not is_safe_kubectl_command(f"kubectl get pods {bad} x")


@pytest.mark.parametrize("ok", ["kubectl get pods | grep x", "kubectl get pods & x", "kubectl get {a}",
                                "kubectl get pods *", "kubectl get pods\nrm -rf /", "  kubectl get pods  ",
                                "kubectl get pods -l 'app=web'"])
def test_validator_quirk_q3_passes(ok):
    assert is_safe_kubectl_command(ok)


@pytest.mark.parametrize("bad", ["kubectl", "kubectlget pods", "kubectl get 'pods", 'kubectl get "x',
                                 "oc get pods", ""])
def test_validator_rejects(bad):
    assert not is_safe_kubectl_command(bad)


def test_parser_fences():
    assert parse_llm_output("  ```kubectl get svc```  ") == "kubectl get svc"
    with pytest.raises(UnsafeCommandError):
        parse_llm_output("```bash\nkubectl get svc\n```")
    with pytest.raises(ValueError):
        parse_llm_output("rm -rf /")


@hsettings(max_examples=200, deadline=None)
@given(st.text(alphabet="kubectl getpods-n;&|`$()<>'\"\n ", max_size=40))
def test_validator_property(s):
    ok = is_safe_kubectl_command(s)
    if ok:
        c = s.strip()
        assert c.startswith("kubectl ")
        assert not any(b in c for b in (";", "&&", "||", "`", "$", "(", ")", "<", ">"))
        shlex.split(c)


# ---------------- cache ----------------
def test_ttl_cache_expiry_and_lru():
    clk = Clock()
    c = TTLCache(maxsize=2, ttl=10, timer=clk)
    c["a"] = 1
    clk.t = 1
    c["b"] = 2
    assert c.get("a") == 1          # touches a -> b is LRU
    c["c"] = 3                      # evicts b
    assert c.get("b") is None and c.get("a") == 1 and c.get("c") == 3
    clk.t = 10.5                    # a expired at 10, c expires at 11
    assert c.get("a") is None and "a" not in c
    assert c.get("c") == 3
    clk.t = 11
    assert len(c) == 0


def test_ttl_refresh_on_set_and_zero_maxsize():
    clk = Clock()
    c = TTLCache(maxsize=5, ttl=10, timer=clk)
    c["a"] = 1
    clk.t = 9
    c["a"] = 2
    clk.t = 15
    assert c.get("a") == 2
    z = TTLCache(maxsize=0, ttl=10)
    with pytest.raises(ValueError):
        z["x"] = 1


# ---------------- rate limiter ----------------
def test_parse_many():
    assert [str(x) for x in parse_many("10/minute")] == ["10 per 1 minute"]
    assert [str(x) for x in parse_many("5 per second; 100/2 hours|7 per day")] == [
        "5 per 1 second", "100 per 2 hour", "7 per 1 day"]
    with pytest.raises(ValueError):
        parse_many("lots")


def test_fixed_window_starts_at_first_hit():
    clk = Clock()
    lim = FixedWindowLimiter(parse_many("2/minute"), timer=clk)
    clk.t = 30
    lim.check("1.2.3.4", "r")
    clk.t = 80
    lim.check("1.2.3.4", "r")
    with pytest.raises(RateLimitExceeded) as ei:
        lim.check("1.2.3.4", "r")
    assert ei.value.detail == "2 per 1 minute"
    lim.check("5.6.7.8", "r")       # other client
    lim.check("1.2.3.4", "other")   # other scope
    clk.t = 90                      # window [30, 90) over
    lim.check("1.2.3.4", "r")


def test_multi_limits_stop_at_first_violation():
    clk = Clock()
    lim = FixedWindowLimiter(parse_many("1/second;3/minute"), timer=clk)
    lim.check("c", "r")
    with pytest.raises(RateLimitExceeded) as ei:
        lim.check("c", "r")
    assert ei.value.detail == "1 per 1 second"


# ---------------- dotenv / settings ----------------
def test_dotenv_semantics(tmp_path):
    text = open("/root/reference/.env-sample").read() if __import__("os").path.exists(
        "/root/reference/.env-sample") else "CACHE_TTL=300      # seconds\n"
    vals = parse_dotenv(text)
    assert vals["CACHE_TTL"] == "300"
    p = tmp_path / ".env"
    p.write_text("export A=1 # c\nB='x # y'\nC=\"q\\nz\"\n# skip\nD=keep\n")
    env = {"D": "orig"}
    assert load_dotenv(str(p), environ=env)
    assert env == {"A": "1", "B": "x # y", "C": "q\nz", "D": "orig"}


def test_settings_defaults_and_int_parse():
    s = Settings.from_env(environ={})
    assert (s.CACHE_MAXSIZE, s.CACHE_TTL, s.LLM_TIMEOUT, s.EXECUTION_TIMEOUT, s.RATE_LIMIT, s.LOG_LEVEL,
            s.OPENAI_MODEL, s.PORT, s.HOST) == (100, 300, 60, 30, "10/minute", "INFO", "gpt-3.5-turbo", 8000, "0.0.0.0")
    assert s.API_AUTH_KEY is None
    s = Settings.from_env(environ={"CACHE_TTL": "5", "LOG_LEVEL": "debug", "SAFE_DECODE": "0", "API_AUTH_KEY": ""})
    assert s.CACHE_TTL == 5 and s.LOG_LEVEL == "DEBUG" and s.SAFE_DECODE is False and s.API_AUTH_KEY is None
    with pytest.raises(ValueError):
        Settings.from_env(environ={"CACHE_TTL": "abc"})


# ---------------- executor ----------------
def test_table_parser_quirk_q6():
    out = parse_kubectl_output("NAME   AGE\nmy pod   5m")
    assert out == {"type": "table", "data": [{"name": "my", "age": "pod"}]}
    assert parse_kubectl_output("x") == {"type": "raw", "data": "x"}


def test_executor_direct(fake_kubectl):
    res = asyncio.run(execute_command_async("kubectl get ns", timeout=5))
    assert res["execution_result"] == {"type": "raw", "data": "default"}
    assert res["metadata"]["success"] is True
    res = asyncio.run(execute_command_async("kubectl get 'x", timeout=5, strict_compat=True))
    assert res == {"execution_error": "Invalid command format: No closing quotation"}


# ---------------- stub LLM ----------------
@pytest.mark.parametrize("q,cmd", [
    ("list all pods", "kubectl get pods"),
    ("show services in namespace prod", "kubectl get services -n prod"),
    ("get deployments across all namespaces", "kubectl get deployments -A"),
    ("scale web to 3 replicas", "kubectl scale deployment web --replicas=3"),
    ("logs of pod api-1", "kubectl logs api-1"),
    ("restart deployment web", "kubectl rollout restart deployment web"),
])
def test_stub_rules(q, cmd):
    assert rule_translate(q) == cmd
    assert is_safe_kubectl_command(cmd)


# ---------------- remote OpenAI-compatible backend ----------------
def test_openai_backend_request_shape_and_retries():
    import httpx
    from ai_agent_kubectl_amd.llm.remote import OpenAIChatLLM
    calls = []

    def handler(request: httpx.Request):
        calls.append(request)
        if len(calls) == 1:
            return httpx.Response(503, json={"error": "busy"})
        body = __import__("json").loads(request.content)
        assert body["temperature"] == 0 and body["model"] == "gpt-x"
        assert body["messages"][0]["role"] == "user" and "User Request: list pods" in body["messages"][0]["content"]
        return httpx.Response(200, json={"choices": [{"message": {"content": "kubectl get pods"}}]})

    s = Settings(OPENAI_API_KEY="sk-test", OPENAI_MODEL="gpt-x", OPENAI_BASE_URL="http://llm.local/v1")
    be = OpenAIChatLLM(s, transport=httpx.MockTransport(handler))
    be_sleep = asyncio.sleep

    async def run():
        return await be.generate("list pods")

    assert asyncio.run(run()) == "kubectl get pods"
    assert len(calls) == 2 and calls[1].headers["authorization"] == "Bearer sk-test"
    assert str(calls[1].url) == "http://llm.local/v1/chat/completions"


def test_openai_backend_without_key_is_degraded_mode():
    from fastapi.testclient import TestClient
    from ai_agent_kubectl_amd.api import create_app
    app = create_app(Settings(LLM_BACKEND="openai", RATE_LIMIT="100/minute"))
    r = TestClient(app).post("/kubectl-command", json={"query": "list pods"})
    assert (r.status_code, r.text) == (503, '{"detail":"LLM Chain not initialized"}')


def test_cpulist_parse_and_pin_noop():
    import os

    from ai_agent_kubectl_amd.utils.runtime import _parse_cpulist, pin_process
    assert _parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert _parse_cpulist("") == []
    before = os.sched_getaffinity(0)
    pin_process(sorted(before))          # pinning to the current mask is a no-op for every thread
    assert os.sched_getaffinity(0) == before
    pin_process([])
    assert os.sched_getaffinity(0) == before
