"""OpenAI-compatible `/v1/chat/completions` and `/v1/models` served by the on-node engine.

The reference is an OpenAI *client* (`ChatOpenAI`, `/root/reference/app.py:117`).  Exposing the same
wire format from this service lets existing OpenAI-speaking clients (including another copy of the
reference pointed at `OPENAI_BASE_URL=http://<this host>/v1`, or this framework's own
`LLM_BACKEND=openai`) use the MI355X engine directly.  Greedy decoding (temperature is accepted and
ignored: the reference always used 0, app.py:109); `max_tokens` caps the completion.
Auth: when API_AUTH_KEY is set, `Authorization: Bearer <key>` or `X-API-Key: <key>`.
"""
from __future__ import annotations

import time
import uuid
from typing import List, Optional

from fastapi import Header, HTTPException, Request
from pydantic import BaseModel, Field


class ChatMessage(BaseModel):
    role: str
    content: str


class ChatRequest(BaseModel):
    model: Optional[str] = None
    messages: List[ChatMessage] = Field(..., min_length=1)
    max_tokens: Optional[int] = Field(None, ge=1, le=4096)
    temperature: Optional[float] = 0.0
    stream: Optional[bool] = False


def install(app, svc, settings) -> None:
    backend = svc.backend
    if backend is None or not hasattr(backend, "generate_chat"):
        return

    def _auth(authorization: Optional[str], x_api_key: Optional[str]) -> None:
        key = settings.API_AUTH_KEY
        if not key:
            return
        bearer = authorization[7:] if authorization and authorization.lower().startswith("bearer ") else None
        if bearer != key and x_api_key != key:
            raise HTTPException(status_code=401, detail="Invalid API Key")

    @app.get("/v1/models")
    async def list_models(authorization: Optional[str] = Header(None), x_api_key: Optional[str] = Header(None)):
        _auth(authorization, x_api_key)
        return {"object": "list", "data": [{"id": settings.MODEL, "object": "model", "owned_by": "local"}]}

    @app.post("/v1/chat/completions")
    async def chat_completions(req: ChatRequest, request: Request, authorization: Optional[str] = Header(None),
                               x_api_key: Optional[str] = Header(None)):
        _auth(authorization, x_api_key)
        if req.stream:
            raise HTTPException(status_code=400, detail="stream=true is not supported")
        msgs = [m.model_dump() for m in req.messages]
        text, finish, n_in, n_out = await backend.generate_chat(msgs, max_tokens=req.max_tokens or 64)
        return {
            "id": "chatcmpl-" + uuid.uuid4().hex[:24], "object": "chat.completion", "created": int(time.time()),
            "model": req.model or settings.MODEL,
            "choices": [{"index": 0, "message": {"role": "assistant", "content": text}, "finish_reason": finish}],
            "usage": {"prompt_tokens": n_in, "completion_tokens": n_out, "total_tokens": n_in + n_out},
        }
