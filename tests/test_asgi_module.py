"""`ai_agent_kubectl_amd.asgi:app` is a ready ASGI app (the `uvicorn app:app` entry point of the
reference, Dockerfile:33), built from the environment at import."""
import importlib
import sys

from fastapi.testclient import TestClient


def test_module_level_app(monkeypatch, tmp_path):
    monkeypatch.chdir(tmp_path)          # no stray ./.env
    monkeypatch.setenv("LLM_BACKEND", "stub")
    monkeypatch.setenv("RATE_LIMIT", "100/minute")
    monkeypatch.delenv("API_AUTH_KEY", raising=False)
    sys.modules.pop("ai_agent_kubectl_amd.asgi", None)
    mod = importlib.import_module("ai_agent_kubectl_amd.asgi")
    with TestClient(mod.app) as c:
        r = c.get("/health")
        assert r.status_code == 200 and r.json() == {"status": "healthy"}
        r = c.post("/kubectl-command", json={"query": "list all pods"})
        assert r.status_code == 200 and r.json()["kubectl_command"].startswith("kubectl ")
