"""Deterministic rule-based LLM (BASELINE config #1: plumbing, no GPU, no API key).

Maps common natural-language requests to kubectl commands with a small rule table.  It lets the
whole HTTP surface run and be benchmarked on CPU and is what the tests
use as the default backend.  Fault-injection hooks (`delay_s`, `error`, `raw`) make the 504 / 500 /
422 paths of `app.py:188-197` testable without a real model.
"""
from __future__ import annotations

import asyncio
import re
from typing import Optional

from .base import LLMBackend

_RESOURCES = [
    (r"\bpods?\b", "pods"), (r"\bservices?\b|\bsvc\b", "services"), (r"\bdeployments?\b|\bdeploy\b", "deployments"),
    (r"\bnodes?\b", "nodes"), (r"\bnamespaces?\b|\bns\b", "namespaces"), (r"\bconfig ?maps?\b", "configmaps"),
    (r"\bsecrets?\b", "secrets"), (r"\bingress(es)?\b", "ingress"), (r"\bpvcs?\b|persistent volume claims?", "pvc"),
    (r"\bpvs?\b|persistent volumes?", "pv"), (r"\bcron ?jobs?\b", "cronjobs"), (r"\bjobs?\b", "jobs"),
    (r"\bstateful ?sets?\b", "statefulsets"), (r"\bdaemon ?sets?\b", "daemonsets"), (r"\breplica ?sets?\b", "replicasets"),
    (r"\bevents?\b", "events"), (r"\bendpoints?\b", "endpoints"), (r"\bservice ?accounts?\b", "serviceaccounts"),
]


def _resource(q: str) -> Optional[str]:
    # service accounts / config maps before their sub-words
    for pat, name in sorted(_RESOURCES, key=lambda x: -len(x[0])):
        if re.search(pat, q):
            return name
    return None


def _namespace_flags(q: str) -> str:
    if re.search(r"\ball namespaces\b|\bevery namespace\b|\bacross namespaces\b", q):
        return " -A"
    m = re.search(r"\b(?:in|from) (?:the )?(?:namespace )?([a-z0-9][a-z0-9\-]*)(?: namespace)?\b", q)
    if m and m.group(1) not in ("the", "all", "my", "a", "cluster", "namespace"):
        return f" -n {m.group(1)}"
    return ""


def rule_translate(query: str) -> str:
    q = query.lower().strip()
    ns = _namespace_flags(q)
    m = re.search(r"\bscale (?:the )?(?:deployment )?([a-z0-9][a-z0-9\-]*) to (\d+)", q)
    if m:
        return f"kubectl scale deployment {m.group(1)} --replicas={m.group(2)}{ns}"
    m = re.search(r"\brestart (?:the )?(?:deployment )?([a-z0-9][a-z0-9\-]*)", q)
    if m:
        return f"kubectl rollout restart deployment {m.group(1)}{ns}"
    m = re.search(r"\blogs? (?:of|for|from) (?:the )?(?:pod )?([a-z0-9][a-z0-9\-]*)", q)
    if m:
        return f"kubectl logs {m.group(1)}{ns}"
    q_res = re.sub(r"\b(?:in|from|across) (?:the |all )?(?:namespace )?[a-z0-9\-]*(?: namespaces?)?\b", " ", q)
    res = _resource(q_res) or _resource(q) or "all"
    m = re.search(r"\b(?:describe|details of|details for) (?:the )?(?:\w+ )?([a-z0-9][a-z0-9\-]*)$", q)
    if re.search(r"\bdescribe\b|\bdetails\b", q):
        name = m.group(1) if m else ""
        if name and name not in (res, res.rstrip("s")):
            return f"kubectl describe {res} {name}{ns}"
        return f"kubectl describe {res}{ns}"
    if re.search(r"\b(count|how many)\b", q):
        return f"kubectl get {res} --no-headers{ns}"
    wide = " -o wide" if re.search(r"\bwide\b|\bdetailed\b|\bip\b", q) else ""
    return f"kubectl get {res}{ns}{wide}"


class StubRuleLLM(LLMBackend):
    name = "stub"

    def __init__(self, delay_s: float = 0.0, error: Optional[BaseException] = None, raw: Optional[str] = None):
        self.delay_s = delay_s
        self.error = error
        self.raw = raw
        self.calls = 0

    async def generate(self, query: str) -> str:
        self.calls += 1
        if self.delay_s:
            await asyncio.sleep(self.delay_s)
        if self.error is not None:
            raise self.error
        if self.raw is not None:
            return self.raw
        return rule_translate(query)
