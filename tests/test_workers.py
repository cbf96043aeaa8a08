"""Multi-worker HTTP tier (serve.py WORKERS > 1, parallel/workers.py) on the CPU: 3 API worker
processes on one port in front of 2 tiny-llama engine replicas.

* a cache miss answered by one worker is `from_cache: true` when another worker answers the same
  query (the reference's single-process cache semantics, `app.py:312-322`, kept global);
* the rate limit is one budget across workers (`app.py:298`: 5/minute -> the 6th request from
  the client is 429 whichever worker it reaches);
* /metrics aggregates the workers.
The responses carry `x-ka-worker: <pid>` (KA_WORKER_HEADER=1) so the test can see which worker
answered; every request uses a fresh TCP connection so SO_REUSEPORT spreads them."""
import http.client
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from ai_agent_kubectl_amd.runtime import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not native.available(), reason="native runtime not built")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _post(port, path, body, timeout=120):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request("POST", path, body=json.dumps(body), headers={"Content-Type": "application/json"})
        r = c.getresponse()
        return r.status, r.getheader("x-ka-worker"), r.read()
    finally:
        c.close()


def _get(port, path, timeout=30, source=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout,
                                   source_address=(source, 0) if source else None)
    try:
        c.request("GET", path)
        r = c.getresponse()
        return r.status, r.getheader("x-ka-worker"), r.read()
    finally:
        c.close()


@pytest.fixture
def service(tmp_path):
    port = _free_port()
    env = dict(os.environ, LLM_BACKEND="engine", MODEL="tiny-llama", DP="2", ENGINE_DEVICES="cpu,cpu", WORKERS="3",
               HOST="127.0.0.1", PORT=str(port), RATE_LIMIT="5/minute", MAX_NEW_TOKENS="6", HIPGRAPH_BUCKETS="1,2,4",
               MAX_BATCH="4", KV_CACHE_TOKENS="4096", MAX_MODEL_LEN="256", KA_WORKER_HEADER="1", LOG_LEVEL="WARNING",
               PYTHONPATH=ROOT)
    env.pop("API_AUTH_KEY", None)
    log = open(tmp_path / "serve.log", "w")
    p = subprocess.Popen([sys.executable, "-m", "ai_agent_kubectl_amd.serve"], cwd=str(tmp_path), env=env,
                         stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        deadline = time.time() + 240
        while time.time() < deadline:
            if p.poll() is not None:
                raise AssertionError("serve exited early:\n" + (tmp_path / "serve.log").read_text())
            try:
                if _get(port, "/health", timeout=2)[0] == 200:
                    break
            except OSError:
                time.sleep(0.5)
        else:
            raise AssertionError("service did not come up:\n" + (tmp_path / "serve.log").read_text())
        # the first /health answer only proves ONE worker is listening: probe from other loopback
        # source addresses (each its own rate-limit key, and a different SO_REUSEPORT hash) until
        # every worker has answered
        seen, i = set(), 10
        while len(seen) < 3 and time.time() < deadline + 60:
            try:
                st, w, _ = _get(port, "/health", timeout=5, source="127.0.0.%d" % i)
                if st == 200:
                    seen.add(w)
            except OSError:
                time.sleep(0.2)
            i = 10 + (i - 9) % 200
        yield port, p, tmp_path
    finally:
        if p.poll() is None:
            os.killpg(p.pid, 15)
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, 9)
                p.wait(10)
        log.close()


def test_three_workers_share_cache_limiter_and_metrics(service):
    port, proc, tmp = service
    # /health is default-limited too (quirk Q9) and would eat the 5/minute budget: the readiness
    # probe above used one hit of /health's own scope, the POST route has its own window.
    st, w_first, body = _post(port, "/kubectl-command", {"query": "list all pods in prod"})
    assert st == 200, body
    first = json.loads(body)
    assert first["from_cache"] is False and first["kubectl_command"].startswith("kubectl ")
    seen = {w_first}
    served = 1
    # 4 more requests are within the budget: all cache hits, answered by other workers too
    for _ in range(4):
        st, w, body = _post(port, "/kubectl-command", {"query": "list   all pods\nin prod"})
        assert st == 200, body
        r = json.loads(body)
        assert r["from_cache"] is True and r["kubectl_command"] == first["kubectl_command"]
        seen.add(w)
        served += 1
    # the 6th request of this client in the window is refused, whichever worker gets it
    st, w, body = _post(port, "/kubectl-command", {"query": "list all pods in prod"})
    assert st == 429, body
    assert json.loads(body) == {"error": "Rate limit exceeded: 5 per 1 minute"}
    seen.add(w)
    assert len(seen) >= 2, "all requests landed on one worker: %s" % seen
    # /metrics (also default-limited, its own scope) aggregates the workers' counters (each
    # worker publishes its batched HTTP observations every 50 ms)
    time.sleep(0.3)
    st, _, text = _get(port, "/metrics")
    assert st == 200
    lines = [ln for ln in text.decode().splitlines()
             if ln.startswith("http_requests_total{") and 'handler="/kubectl-command"' in ln]
    total = sum(float(ln.rsplit(" ", 1)[1]) for ln in lines)
    assert total >= served, text.decode()[:2000]
