"""LLM backend interface.

Replaces the LangChain `RunnableSequence` (`PromptTemplate | ChatOpenAI | KubectlOutputParser`,
`/root/reference/app.py:106-118`).  A backend turns the sanitised query into the model's raw text;
`run_llm` in `api/service.py` applies the timeout and the output parser exactly where
`chain.ainvoke` + `asyncio.wait_for` did (`app.py:177-197`).
"""
from __future__ import annotations

import abc
from typing import Dict, Optional


class LLMUnavailableError(RuntimeError):
    """Backend cannot serve (engine not ready, worker died, OOM) -> HTTP 503."""


class LLMBackend(abc.ABC):
    name = "base"

    @abc.abstractmethod
    async def generate(self, query: str) -> str:
        """Return the raw completion for the (already sanitised) query."""

    async def start(self) -> None:  # pragma: no cover - trivial
        return None

    async def close(self) -> None:  # pragma: no cover - trivial
        return None

    def attach_metrics(self, metrics) -> None:
        """Give the backend the app's metrics registry (engine TTFT/TPOT/queue gauges)."""
        return None

    def healthy(self) -> bool:
        return True

    def stats(self) -> Dict[str, float]:
        return {}


def build_backend(settings, metrics=None) -> Optional[LLMBackend]:
    """Backend factory keyed by `LLM_BACKEND` (stub | engine | openai).

    Mirrors app.py:119-122: a failure while building leaves the service in degraded mode
    (backend None -> every cache miss answers 503 "LLM Chain not initialized").
    """
    kind = settings.LLM_BACKEND.lower()
    if kind == "stub":
        from .stub import StubRuleLLM
        return StubRuleLLM()
    if kind == "openai":
        from .remote import OpenAIChatLLM
        return OpenAIChatLLM(settings)
    if kind == "engine":
        import os
        under_torchrun = int(os.environ.get("WORLD_SIZE", "1")) > 1
        if settings.DP > 1 or (settings.ENGINE_PROCESS and not under_torchrun):
            # engine replica process(es) — each a TP group of TP devices — behind this API process:
            # HTTP handling and the GPU loop never contend for one GIL (SURVEY.md §7.3 hard part 6).
            # Under torchrun with TP > 1 this process is TP rank 0 itself (serve.py).
            from ..parallel.dp import DPRouterLLM
            return DPRouterLLM(settings, max(1, settings.DP))
        from .engine_backend import EngineLLM
        return EngineLLM.from_settings(settings, metrics=metrics)
    raise ValueError(f"unknown LLM_BACKEND {settings.LLM_BACKEND!r}")
