"""The production server on the GPU (serve.py, WORKERS=2: two uvicorn API workers on one port
sharing the shared-memory cache / limiter, one engine replica on cuda:0), with the serving defaults
for the KV pool (the whole GPU_MEM_FRACTION budget) and the 8192-token context: health, generation,
a cache hit answered from the other worker's entry, and the engine histograms on /metrics."""
import http.client
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _req(port, method, path, body=None, timeout=120):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request(method, path, body=json.dumps(body) if body is not None else None,
                  headers={"Content-Type": "application/json"})
        r = c.getresponse()
        return r.status, r.read()
    finally:
        c.close()


def test_serve_two_workers_engine_on_gpu(tmp_path):
    port = _port()
    env = dict(os.environ, LLM_BACKEND="engine", MODEL="llama3-8b-2l", DP="1", ENGINE_DEVICES="cuda:0",
               WORKERS="2", HOST="127.0.0.1", PORT=str(port), RATE_LIMIT="1000/minute", MAX_NEW_TOKENS="8",
               MAX_BATCH="8", HIPGRAPH_BUCKETS="1,2,4,8", GPU_MEM_FRACTION="0.3", LOG_LEVEL="WARNING",
               PYTHONPATH=ROOT)
    for k in ("API_AUTH_KEY", "KV_CACHE_TOKENS", "MAX_MODEL_LEN"):
        env.pop(k, None)
    log = open(tmp_path / "serve.log", "w")
    p = subprocess.Popen([sys.executable, "-m", "ai_agent_kubectl_amd.serve"], cwd=str(tmp_path), env=env,
                         stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        deadline = time.time() + 240
        while True:
            assert p.poll() is None, (tmp_path / "serve.log").read_text()[-3000:]
            try:
                if _req(port, "GET", "/health", timeout=2)[0] == 200:
                    break
            except OSError:
                pass
            assert time.time() < deadline, "server did not come up"
            time.sleep(1.0)
        st, body = _req(port, "POST", "/kubectl-command", {"query": "list all pods in kube-system"})
        assert st == 200, body
        first = json.loads(body)
        assert first["kubectl_command"].startswith("kubectl ") and first["from_cache"] is False
        hits = 0
        for _ in range(6):   # fresh connections: SO_REUSEPORT spreads them over both workers
            st, body = _req(port, "POST", "/kubectl-command", {"query": "list all pods in  kube-system"})
            assert st == 200
            r = json.loads(body)
            assert r["kubectl_command"] == first["kubectl_command"]
            hits += r["from_cache"]
        assert hits == 6
        time.sleep(0.3)
        st, text = _req(port, "GET", "/metrics")
        text = text.decode()
        assert st == 200
        assert 'llm_step_seconds_count{phase="decode"}' in text and 'llm_step_seconds_count{phase="prefill"}' in text
        assert "llm_ttft_seconds_count" in text and "llm_queue_wait_seconds_count" in text
    finally:
        if p.poll() is None:
            os.killpg(p.pid, 15)
            try:
                p.wait(60)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, 9)
                p.wait(10)
        log.close()


def test_serve_dp2_x_tp2_on_one_gpu(tmp_path):
    """DP=2 x TP=2 (two replicas, each a TP group of two processes: parallel/dp.py) behind two API
    workers on one port, all four ranks on cuda:0 (KA_TP_BACKEND=gloo stands in for RCCL, which
    refuses two ranks on one device; the decode all-reduces / all-gathers are the one-shot IPC
    kernels, csrc/allreduce.hip).  Two-layer model with the real Llama-3-8B layer geometry."""
    port = _port()
    env = dict(os.environ, LLM_BACKEND="engine", MODEL="llama3-8b-2l", DP="2", TP="2", WORKERS="2",
               ENGINE_DEVICES="cuda:0,cuda:0,cuda:0,cuda:0", KA_TP_BACKEND="gloo", HOST="127.0.0.1",
               PORT=str(port), RATE_LIMIT="1000/minute", MAX_NEW_TOKENS="8", HIPGRAPH_BUCKETS="1,2,4",
               MAX_BATCH="4", KV_CACHE_TOKENS="16384", MAX_MODEL_LEN="512", LOG_LEVEL="WARNING", PYTHONPATH=ROOT)
    for k in ("API_AUTH_KEY", "RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    log = open(tmp_path / "serve.log", "w")
    p = subprocess.Popen([sys.executable, "-m", "ai_agent_kubectl_amd.serve"], cwd=str(tmp_path), env=env,
                         stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        deadline = time.time() + 300
        while time.time() < deadline:
            assert p.poll() is None, (tmp_path / "serve.log").read_text()[-4000:]
            try:
                if _req(port, "GET", "/ready", timeout=2)[0] == 200:
                    break
            except OSError:
                pass
            time.sleep(1.0)
        else:
            raise AssertionError("service did not come up:\n" + (tmp_path / "serve.log").read_text()[-4000:])
        from ai_agent_kubectl_amd.safety import is_safe_kubectl_command
        seen = []
        for q in ("list all pods in prod", "get nodes -o wide", "describe deployment api", "top pods"):
            st, body = _req(port, "POST", "/kubectl-command", {"query": q})
            assert st == 200, (body, (tmp_path / "serve.log").read_text()[-6000:])
            cmd = json.loads(body)["kubectl_command"]
            assert is_safe_kubectl_command(cmd), cmd
            seen.append(cmd)
        st, body = _req(port, "POST", "/kubectl-command", {"query": "list all pods   in prod"})
        assert st == 200 and json.loads(body)["from_cache"] is True
    finally:
        if p.poll() is None:
            os.killpg(p.pid, 15)
            try:
                p.wait(60)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, 9)
                p.wait(10)
        log.close()
