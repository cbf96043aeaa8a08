"""`LLM_BACKEND=engine`: the on-node MI355X inference engine behind the reference's chain call.

`generate(query)` does what `chain.ainvoke({"query": q})` did (`/root/reference/app.py:184`):
PromptTemplate.format (prompt.py) -> single user turn in the model's chat template -> greedy decode
(temperature 0) -> text for `KubectlOutputParser` semantics (safety.parse_llm_output).

Tokenisation keeps the instruction prefix as a separately encoded, cached token run so that every
request's prompt starts with identical token ids and the engine's prefix cache shares its KV blocks.
Cancellation (the service's `LLM_TIMEOUT` -> 504) aborts the sequence and frees its blocks.
"""
from __future__ import annotations

import asyncio
import logging
from typing import List, Optional

from ..engine.safe_decode import forced_prefix
from ..engine.sequence import SamplingParams
from ..prompt import PROMPT_PREFIX, PROMPT_SUFFIX
from .base import LLMBackend, LLMUnavailableError

logger = logging.getLogger("app.engine")


class EngineLLM(LLMBackend):
    name = "engine"

    def __init__(self, engine, max_new_tokens: int = 24, ignore_eos: bool = False, safe_decode: bool = True):
        self.engine = engine
        self.tok = engine.tokenizer
        self.params = SamplingParams(max_new_tokens=max_new_tokens, ignore_eos=ignore_eos, safe_decode=safe_decode)
        before, after = self.tok.chat_prefix_suffix()
        self._prefix_ids: List[int] = before + self.tok.encode(PROMPT_PREFIX)
        self._after_ids: List[int] = after
        self._forced = forced_prefix(self.tok) if safe_decode else []
        self._started = False

    @classmethod
    def from_settings(cls, settings, metrics=None) -> "EngineLLM":
        from ..engine.builder import EngineOptions, build_engine

        opts = EngineOptions.from_settings(settings)
        comm = None
        if settings.TP > 1:
            from ..parallel.launch import init_tp

            comm, rank = init_tp(settings.TP)
            opts.tp_rank = rank
            opts.device = f"cuda:{rank}" if opts.device == "cuda" else opts.device
        eng = build_engine(opts, comm=comm, metrics=metrics)
        if opts.use_graphs and opts.device.startswith("cuda"):
            eng.runner.capture_graphs()
        return cls(eng, max_new_tokens=settings.MAX_NEW_TOKENS, ignore_eos=settings.IGNORE_EOS,
                   safe_decode=settings.SAFE_DECODE)

    def prompt_ids(self, query: str) -> List[int]:
        return self._prefix_ids + self.tok.encode(query + PROMPT_SUFFIX) + self._after_ids

    async def start(self) -> None:
        if not self._started:
            from ..utils.runtime import tune_gc
            tune_gc()
            self.engine.start()
            self._started = True

    async def close(self) -> None:
        if self._started:
            self.engine.shutdown()
            self._started = False

    def healthy(self) -> bool:
        return self.engine.healthy

    def attach_metrics(self, metrics) -> None:
        if metrics is not None and getattr(self.engine, "metrics", None) is None:
            self.engine.metrics = metrics

    async def generate(self, query: str) -> str:
        if not self._started:
            await self.start()
        if not self.engine.healthy:
            raise LLMUnavailableError(f"engine unhealthy: {self.engine.last_error}")
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()

        def done(seq):
            loop.call_soon_threadsafe(_resolve, fut, seq)

        seq = self.engine.submit(self.prompt_ids(query), self.params, done, forced_prefix=self._forced)
        try:
            seq = await fut
        except asyncio.CancelledError:
            self.engine.abort(seq)
            raise
        if seq.error is not None:
            if seq.finish_reason == "error":
                raise LLMUnavailableError(str(seq.error))
            raise RuntimeError(str(seq.error))
        ids = [t for t in seq.output_ids if not self.tok.is_eos(t)]
        return self.tok.decode(ids)

    def stats(self):
        return dict(self.engine.runner.stats)

    # ---- OpenAI-compatible chat (api/openai_compat.py) ----------------------------------------
    def chat_ids(self, messages) -> List[int]:
        """Multi-turn chat template of the model family (Llama-3 header tokens / Llama-2 [INST])."""
        tok = self.tok
        if tok.family == "llama3":
            s = tok.specials
            ids = [s["<|begin_of_text|>"]]
            for m in messages:
                ids += [s["<|start_header_id|>"]] + tok.encode(m["role"]) + [s["<|end_header_id|>"]]
                ids += tok.encode("\n\n" + m["content"]) + [s["<|eot_id|>"]]
            ids += [s["<|start_header_id|>"]] + tok.encode("assistant") + [s["<|end_header_id|>"]] + tok.encode("\n\n")
            return ids
        text = "".join(f"[INST] {m['content']} [/INST]" if m["role"] != "assistant" else f" {m['content']} "
                       for m in messages)
        return [tok.bos_id] + tok.encode(text)

    async def generate_chat(self, messages, max_tokens: int = 64, safe: bool = False):
        """Returns (text, finish_reason, prompt_tokens, completion_tokens)."""
        if not self._started:
            await self.start()
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()
        params = SamplingParams(max_new_tokens=max_tokens, ignore_eos=False, safe_decode=safe)
        ids = self.chat_ids(messages)
        seq = self.engine.submit(ids, params, lambda sq: loop.call_soon_threadsafe(_resolve, fut, sq),
                                 forced_prefix=self._forced if safe else None)
        try:
            seq = await fut
        except asyncio.CancelledError:
            self.engine.abort(seq)
            raise
        if seq.error is not None:
            raise LLMUnavailableError(str(seq.error))
        out = [t for t in seq.output_ids if not self.tok.is_eos(t)]
        return self.tok.decode(out), ("stop" if seq.finish_reason == "stop" else "length"), len(ids), len(seq.output_ids)


def _resolve(fut: asyncio.Future, seq) -> None:
    if not fut.done():
        fut.set_result(seq)
