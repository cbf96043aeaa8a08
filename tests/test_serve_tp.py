"""The service entry point with tensor parallelism, end to end over HTTP on the CPU (gloo, tiny model):

* `torchrun --nproc-per-node 2 -m ai_agent_kubectl_amd.serve` with TP=2: rank 0 serves HTTP and
  schedules, rank 1 mirrors every step in ModelRunner.worker_loop (serve.py);
* `serve.py` with DP=2 x TP=2 and 2 API workers: two replicas, each a TP group whose rank 0 spawned
  its TP worker (parallel/dp.py), behind one port with a shared cache (parallel/workers.py).
Replies must pass the reference's safety validator; the second ask of a query is a cache hit."""
import http.client
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from ai_agent_kubectl_amd.safety import is_safe_kubectl_command

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _req(port, method, path, body=None, timeout=120):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request(method, path, body=json.dumps(body) if body is not None else None,
                  headers={"Content-Type": "application/json"})
        r = c.getresponse()
        return r.status, r.read()
    finally:
        c.close()


def _serve(cmd, env, tmp_path, port, deadline_s=300):
    log = open(tmp_path / "serve.log", "w")
    p = subprocess.Popen(cmd, cwd=str(tmp_path), env=env, stdout=log, stderr=subprocess.STDOUT,
                         start_new_session=True)
    deadline = time.time() + deadline_s
    while time.time() < deadline:
        if p.poll() is not None:
            raise AssertionError("serve exited early:\n" + (tmp_path / "serve.log").read_text()[-4000:])
        try:
            if _req(port, "GET", "/ready", timeout=2)[0] == 200:
                return p, log
        except OSError:
            pass
        time.sleep(0.5)
    raise AssertionError("service did not come up:\n" + (tmp_path / "serve.log").read_text()[-4000:])


def _stop(p, log):
    if p.poll() is None:
        os.killpg(p.pid, 15)
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, 9)
            p.wait(10)
    log.close()


def _env(port, **kw):
    env = dict(os.environ, LLM_BACKEND="engine", MODEL="tiny-llama", HOST="127.0.0.1", PORT=str(port),
               RATE_LIMIT="1000/minute", MAX_NEW_TOKENS="6", HIPGRAPH_BUCKETS="1,2,4", MAX_BATCH="4",
               KV_CACHE_TOKENS="4096", MAX_MODEL_LEN="256", LOG_LEVEL="WARNING", PYTHONPATH=ROOT, **kw)
    for k in ("API_AUTH_KEY", "RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _check_service(port):
    st, body = _req(port, "POST", "/kubectl-command", {"query": "list all pods in kube-system"})
    assert st == 200, body
    first = json.loads(body)
    assert first["from_cache"] is False and is_safe_kubectl_command(first["kubectl_command"])
    st, body = _req(port, "POST", "/kubectl-command", {"query": "list   all pods in kube-system"})
    assert st == 200 and json.loads(body)["from_cache"] is True
    for q in ("get nodes -o wide", "describe deployment api", "scale web to 3 replicas"):
        st, body = _req(port, "POST", "/kubectl-command", {"query": q})
        assert st == 200, body
        assert is_safe_kubectl_command(json.loads(body)["kubectl_command"])


@pytest.mark.slow
def test_torchrun_serve_tp2(tmp_path):
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", "-m", "ai_agent_kubectl_amd.serve"]
    p, log = _serve(cmd, _env(port, TP="2"), tmp_path, port)
    try:
        _check_service(port)
    finally:
        _stop(p, log)


@pytest.mark.slow
def test_serve_dp2_x_tp2_two_workers(tmp_path):
    port = _free_port()
    cmd = [sys.executable, "-m", "ai_agent_kubectl_amd.serve"]
    p, log = _serve(cmd, _env(port, TP="2", DP="2", WORKERS="2", ENGINE_DEVICES="cpu"), tmp_path, port)
    try:
        _check_service(port)
    finally:
        _stop(p, log)


@pytest.mark.slow
def test_serve_tp8_70b_head_geometry(tmp_path):
    """serve.py with TP = 8 on the CPU (gloo): one replica whose rank 0 spawns 7 TP worker ranks, at
    the Llama-3-70B head layout (64 q / 8 kv heads, one KV head per rank) with small layers."""
    port = _free_port()
    cmd = [sys.executable, "-m", "ai_agent_kubectl_amd.serve"]
    env = _env(port, TP="8", DP="1", ENGINE_DEVICES="cpu")
    env["MODEL"] = "llama3-70b-tiny"
    p, log = _serve(cmd, env, tmp_path, port, deadline_s=600)
    try:
        _check_service(port)
    finally:
        _stop(p, log)
