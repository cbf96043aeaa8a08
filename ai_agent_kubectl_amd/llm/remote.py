"""Optional remote OpenAI-compatible chat backend (`LLM_BACKEND=openai`).

Keeps the reference's remote path available (`ChatOpenAI(temperature=0, api_key, model,
request_timeout=LLM_TIMEOUT[, base_url])`, `/root/reference/app.py:106-118`) without LangChain or
the OpenAI SDK: one user message, temperature 0, `OPENAI_MODEL`, `OPENAI_BASE_URL`, and the SDK's
default of 2 retries on connection errors / 408 / 409 / 429 / 5xx.
It also works against this framework's own `/v1/chat/completions` endpoint (api/openai_compat.py).
"""
from __future__ import annotations

import asyncio

import httpx

from ..prompt import render_prompt
from .base import LLMBackend, LLMUnavailableError

_RETRY_STATUS = {408, 409, 429, 500, 502, 503, 504}


class OpenAIChatLLM(LLMBackend):
    name = "openai"

    def __init__(self, settings, max_retries: int = 2, transport=None):
        if not settings.OPENAI_API_KEY:
            # ChatOpenAI raises at construction without a key -> app.py:119-122 degraded mode.
            raise LLMUnavailableError("OPENAI_API_KEY not set")
        self.base_url = (settings.OPENAI_BASE_URL or "https://api.openai.com/v1").rstrip("/")
        self.model = settings.OPENAI_MODEL
        self.api_key = settings.OPENAI_API_KEY
        self.timeout = settings.LLM_TIMEOUT
        self.max_retries = max_retries
        self._client = httpx.AsyncClient(timeout=self.timeout, transport=transport)

    async def generate(self, query: str) -> str:
        body = {"model": self.model, "temperature": 0,
                "messages": [{"role": "user", "content": render_prompt(query)}]}
        headers = {"Authorization": f"Bearer {self.api_key}"}
        last_exc = None
        for attempt in range(self.max_retries + 1):
            try:
                r = await self._client.post(self.base_url + "/chat/completions", json=body, headers=headers)
                if r.status_code in _RETRY_STATUS and attempt < self.max_retries:
                    await asyncio.sleep(min(0.5 * 2 ** attempt, 8.0))
                    continue
                r.raise_for_status()
                return r.json()["choices"][0]["message"]["content"]
            except (httpx.ConnectError, httpx.ReadError, httpx.RemoteProtocolError) as e:
                last_exc = e
                if attempt < self.max_retries:
                    await asyncio.sleep(min(0.5 * 2 ** attempt, 8.0))
                    continue
                raise
        raise last_exc  # pragma: no cover

    async def close(self) -> None:
        await self._client.aclose()
