"""FastAPI application: the reference's HTTP surface, byte-compatible.

Routes, status codes and bodies follow `/root/reference/app.py:131-389` (SURVEY.md §3.2-3.5,
Appendix A goldens):

* `POST /kubectl-command` (`app.py:284-346`): auth dep -> body validation -> per-route rate limit ->
  sanitise -> cache -> LLM (503/504/422/500 mapping of `app.py:177-197`) -> cache store ->
  `CommandResponse` with synthetic metadata (quirk Q2).  Never executes.
* `POST /execute` (`app.py:356-389`): auth -> body -> limit -> validator (400) -> subprocess.
* `GET /health` (`app.py:348-354`): constant `{"status":"healthy"}`.
* `GET /metrics` (`app.py:138`): Prometheus exposition.
* `/docs`, `/redoc`, `/openapi.json` from FastAPI, title "Kubectl NLP Service" v1.0.0.

Middleware order matches the reference: the rate-limit middleware is inner, the Prometheus
middleware outermost (added last), so 401/429/500 responses are counted.

Hot path note: successful responses are JSON-encoded here with the exact separators/ordering
FastAPI's `JSONResponse` uses, skipping a redundant pydantic round trip per request.
"""
from __future__ import annotations

import asyncio
import os
import contextlib
import json
import logging
from typing import Any, Dict, Optional

from fastapi import Depends, FastAPI, Header, HTTPException, Request, status
from fastapi.responses import JSONResponse, Response

from .. import safety
from ..cache import TTLCache
from ..shared_state import SharedFixedWindowLimiter, SharedTTLCache, open_from_settings
from ..config import Settings
from ..executor import execute_command_async, utcnow_iso
from ..llm.base import LLMBackend, LLMUnavailableError, build_backend
from ..metrics import CONTENT_TYPE, PrometheusMiddleware, ServiceMetrics
from ..ratelimit import (FixedWindowLimiter, RateLimitExceeded, RateLimitMiddleware, client_address,
                         parse_many, rate_limit_body)
from ..schemas import CommandResponse, ExecuteRequest, Query

logger = logging.getLogger("app")

_UNSET = object()


def _json(content: Dict[str, Any], status_code: int = 200) -> Response:
    body = json.dumps(content, ensure_ascii=False, allow_nan=False, indent=None,
                      separators=(",", ":")).encode("utf-8")
    return Response(content=body, status_code=status_code, media_type="application/json")


def _command_body(command: str, from_cache: bool, execution_data: Dict[str, Any]) -> Dict[str, Any]:
    md = execution_data["metadata"]
    return {
        "kubectl_command": command,
        "execution_result": execution_data.get("execution_result"),
        "execution_error": execution_data.get("execution_error"),
        "from_cache": from_cache,
        "metadata": {
            "start_time": md["start_time"],
            "end_time": md["end_time"],
            "duration_ms": float(md["duration_ms"]),
            "success": md["success"],
            "error_type": md.get("error_type"),
            "error_code": md.get("error_code"),
        },
    }


_STR = json.JSONEncoder(ensure_ascii=False).encode   # the str encoding json.dumps(ensure_ascii=False) uses


def _generated_json(command: str, from_cache: bool, start: str, end: str) -> bytes:
    """Byte-for-byte `_json(_command_body(command, from_cache, <synthetic metadata>))` for the
    /kubectl-command success reply (app.py:333-346: duration 0.0, success true, no execution
    fields), assembled from a fixed template: the reply of every generated or cached command
    skips the generic dict walk of json.dumps (tests/test_api_golden.py checks the equality)."""
    return (b'{"kubectl_command":' + _STR(command).encode("utf-8")
            + (b',"execution_result":null,"execution_error":null,"from_cache":true,"metadata":{"start_time":'
               if from_cache else
               b',"execution_result":null,"execution_error":null,"from_cache":false,"metadata":{"start_time":')
            + _STR(start).encode("utf-8") + b',"end_time":' + _STR(end).encode("utf-8")
            + b',"duration_ms":0.0,"success":true,"error_type":null,"error_code":null}}')


async def _lag_probe(metrics, period: float = 0.05) -> None:
    """Observe how late the event loop wakes a 50 ms sleeper (GIL / blocking-call diagnostics)."""
    loop = asyncio.get_running_loop()
    # several API workers: /metrics is rendered by whichever worker gets the scrape, from every
    # worker's shared samples, so each worker publishes its batched HTTP observations promptly
    shared = bool(os.environ.get("PROMETHEUS_MULTIPROC_DIR"))
    while True:
        t0 = loop.time()
        await asyncio.sleep(period)
        metrics.loop_lag.observe(max(0.0, loop.time() - t0 - period))
        if shared:
            for flush in metrics.flush_hooks:
                flush()


class FastPathMiddleware:
    """Pure-ASGI fast path for the two POST routes' common case.

    FastAPI's per-request dependency solving, body-field validation and response plumbing cost
    ~0.3 ms of Python per request — more than the rest of the handler — and every request of a
    burst pays it serially on the event loop.  For a request that FastAPI would certainly accept
    (JSON content type, a JSON object whose field is a str of the minimum length, valid or disabled
    auth) this middleware calls the same handler function directly and renders errors exactly like
    FastAPI's HTTPException / rate-limit handlers.  Anything else — missing/invalid key (401 before
    422, Q-ordering), bad JSON, wrong types, other content types — is replayed untouched into the
    FastAPI stack, so every error body stays byte-identical (tests/test_api_golden.py)."""

    def __init__(self, app, settings: Settings, routes):
        self.app = app
        self.key = settings.API_AUTH_KEY
        self.routes = routes
        self.hits = 0

    async def __call__(self, scope, receive, send):
        ent = self.routes.get(scope.get("path")) if scope["type"] == "http" and scope["method"] == "POST" else None
        if ent is None:
            await self.app(scope, receive, send)
            return
        ctype = key = None
        for k, v in scope["headers"]:
            if k == b"content-type":
                if ctype is None:
                    ctype = v
            elif k == b"x-api-key":
                if key is None:
                    key = v
        if (ctype is None or ctype.split(b";")[0].strip().lower() != b"application/json"
                or (self.key and (key is None or key.decode("latin-1") != self.key))):
            await self.app(scope, receive, send)
            return
        chunks, tail = [], None
        while True:
            msg = await receive()
            if msg["type"] != "http.request":
                tail = msg
                break
            chunks.append(msg.get("body", b""))
            if not msg.get("more_body", False):
                break
        body = b"".join(chunks)
        field, min_len, handler = ent
        value = None
        if tail is None and body:
            try:
                obj = json.loads(body)
                value = obj.get(field) if isinstance(obj, dict) else None
            except ValueError:
                value = None
        if not isinstance(value, str) or len(value) < min_len:
            await self.app(scope, _replay(body, tail, receive), send)
            return
        self.hits += 1
        logger.debug("API key verified." if self.key else "API key auth disabled.")
        try:
            resp = await handler(value, scope)
        except HTTPException as e:           # fastapi.exception_handlers.http_exception_handler
            resp = _json({"detail": e.detail}, status_code=e.status_code)
            if e.headers:
                resp.headers.update(e.headers)
        except RateLimitExceeded as e:       # the app's RateLimitExceeded handler
            resp = Response(content=rate_limit_body(e), status_code=429, media_type="application/json")
        await resp(scope, receive, send)


def _replay(body: bytes, tail, receive):
    sent = [False]

    async def replay():
        if not sent[0]:
            sent[0] = True
            return {"type": "http.request", "body": body, "more_body": False}
        if tail is not None:
            return tail
        return await receive()
    return replay


class KubectlService:
    """State shared by the routes: settings, cache, limiter, metrics and the LLM backend."""

    def __init__(self, settings: Settings, backend: Optional[LLMBackend], metrics: ServiceMetrics):
        self.settings = settings
        self.backend = backend
        self.metrics = metrics
        self.route_limits = parse_many(settings.RATE_LIMIT)
        # several API workers (serve.py WORKERS > 1): one cache and one set of limit windows in
        # shared memory, so from_cache and 429 are global as with the reference's single process
        self.shared = open_from_settings(settings)
        if self.shared is not None:
            self.cache = SharedTTLCache(self.shared, maxsize=settings.CACHE_MAXSIZE, ttl=settings.CACHE_TTL)
            self.limiter = SharedFixedWindowLimiter(self.shared, default_limits=self.route_limits)
        else:
            self.cache = TTLCache(maxsize=settings.CACHE_MAXSIZE, ttl=settings.CACHE_TTL)
            self.limiter = FixedWindowLimiter(default_limits=self.route_limits)

    async def run_llm(self, query: str) -> str:
        """`run_llm_chain_async` (app.py:177-197): timeout + parser + HTTP error mapping."""
        if self.backend is None:
            raise HTTPException(status_code=status.HTTP_503_SERVICE_UNAVAILABLE, detail="LLM Chain not initialized")
        timeout = self.settings.LLM_TIMEOUT

        s = self.settings

        async def _chain() -> str:
            if s.FAULT_LLM_DELAY_MS:          # fault injection: exercise 504 paths
                await asyncio.sleep(s.FAULT_LLM_DELAY_MS / 1000.0)
            if s.FAULT_LLM_ERROR:
                if s.FAULT_LLM_ERROR == "unavailable":
                    raise LLMUnavailableError("injected fault")
                raise RuntimeError(s.FAULT_LLM_ERROR)
            return safety.parse_llm_output(await self.backend.generate(query))

        loop = asyncio.get_running_loop()
        t0 = loop.time()
        task = asyncio.current_task()
        fired = []

        def _expire():
            fired.append(True)
            task.cancel()

        # asyncio.wait_for semantics without its per-call task: cancel this task at the deadline
        # and turn that cancellation into the timeout (what asyncio.timeout does on 3.11+)
        timer = loop.call_later(timeout, _expire) if timeout is not None else None
        try:
            try:
                command = await _chain()
            except asyncio.CancelledError:
                if fired:
                    raise asyncio.TimeoutError() from None
                raise
            finally:
                if timer is not None:
                    timer.cancel()
            self.metrics.llm_latency.observe(loop.time() - t0)
            logger.info("LLM generated command for query '%s': %s", query, command)
            return command
        except asyncio.TimeoutError:
            self.metrics.llm_errors.labels("timeout").inc()
            logger.error(f"LLM chain timed out after {timeout}s for query: {query}")
            raise HTTPException(status_code=status.HTTP_504_GATEWAY_TIMEOUT, detail="LLM request timed out")
        except LLMUnavailableError as e:
            self.metrics.llm_errors.labels("unavailable").inc()
            logger.error(f"LLM backend unavailable: {e}")
            raise HTTPException(status_code=status.HTTP_503_SERVICE_UNAVAILABLE, detail=f"LLM backend unavailable: {e}")
        except ValueError as ve:
            self.metrics.llm_errors.labels("unsafe").inc()
            logger.error(f"LLM generated unsafe command: {ve}")
            raise HTTPException(status_code=422,
                                detail=f"LLM generated unsafe command: {ve}")
        except Exception as e:
            self.metrics.llm_errors.labels("error").inc()
            logger.exception(f"Error running LLM chain for query '{query}': {e}")
            raise HTTPException(status_code=status.HTTP_500_INTERNAL_SERVER_ERROR,
                                detail=f"Error processing query with LLM: {e}")


def create_app(settings: Optional[Settings] = None, backend: Any = _UNSET,
               metrics: Optional[ServiceMetrics] = None) -> FastAPI:
    settings = settings or Settings.from_env()
    metrics = metrics or ServiceMetrics()
    if backend is _UNSET:
        try:
            backend = build_backend(settings, metrics=metrics)
        except Exception:
            logger.exception("Failed to initialize LLM backend.")  # app.py:119-122
            backend = None
    if backend is not None and hasattr(backend, "attach_metrics"):
        backend.attach_metrics(metrics)
    svc = KubectlService(settings, backend, metrics)

    if not settings.API_AUTH_KEY:
        logger.warning("API_AUTH_KEY environment variable not set. API authentication is disabled.")

    @contextlib.asynccontextmanager
    async def lifespan(app):
        from ..utils.runtime import tune_gc
        tune_gc()
        if svc.backend is not None:
            await svc.backend.start()
        probe = asyncio.get_running_loop().create_task(_lag_probe(metrics))
        try:
            yield
        finally:
            probe.cancel()
            if svc.backend is not None:
                await svc.backend.close()

    app = FastAPI(title="Kubectl NLP Service", version="1.0.0", lifespan=lifespan)
    app.state.service = svc
    app.state.limiter = svc.limiter

    async def _rate_limited(request: Request, exc: RateLimitExceeded):
        return Response(content=rate_limit_body(exc), status_code=429, media_type="application/json")

    app.add_exception_handler(RateLimitExceeded, _rate_limited)

    async def verify_api_key(x_api_key: Optional[str] = Header(None)):
        """app.py:141-151 — X-API-Key header; disabled when API_AUTH_KEY is unset."""
        if not settings.API_AUTH_KEY:
            logger.debug("API key auth disabled.")
            return
        if not x_api_key:
            logger.warning("Missing X-API-Key header.")
            raise HTTPException(status_code=status.HTTP_401_UNAUTHORIZED, detail="Missing X-API-Key header")
        if x_api_key != settings.API_AUTH_KEY:
            logger.warning("Invalid API Key received.")
            raise HTTPException(status_code=status.HTTP_401_UNAUTHORIZED, detail="Invalid API Key")
        logger.debug("API key verified.")

    decorated = set()

    def limited(fn):
        decorated.add("%s.%s" % (fn.__module__, fn.__name__))
        return fn

    async def kubectl_command(query: str, scope) -> Response:
        """POST /kubectl-command after auth + body validation (app.py:299-346); shared by the
        FastAPI route and the fast path."""
        svc.limiter.check(client_address(scope), "%s.get_kubectl_command" % __name__, svc.route_limits)
        logger.info("Received query: '%s'", query)
        sanitized_query = safety.sanitize_query(query)
        from_cache = False
        try:
            cached = svc.cache.get(sanitized_query)
            if cached is not None:
                logger.info("Cache hit for query: %s", sanitized_query)
                svc.metrics.cache_hits.inc()
                command = cached
                from_cache = True
            else:
                logger.info("Cache miss for query: %s", sanitized_query)
                svc.metrics.cache_misses.inc()
                logger.debug("Calling LLM for query: %s", sanitized_query)
                command = await svc.run_llm(sanitized_query)
                svc.cache[sanitized_query] = command
                logger.debug("Stored result in cache for query: %s", sanitized_query)
        except HTTPException:
            raise
        except Exception as e:
            logger.exception(f"Unexpected error processing query '{sanitized_query}': {e}")
            raise HTTPException(status_code=status.HTTP_500_INTERNAL_SERVER_ERROR,
                                detail="Internal server error processing request")
        now = utcnow_iso()
        return Response(content=_generated_json(command, from_cache, now, utcnow_iso()), status_code=200,
                        media_type="application/json")

    async def execute(command: str, scope) -> Response:
        """POST /execute after auth + body validation (app.py:369-389)."""
        svc.limiter.check(client_address(scope), "%s.execute_kubectl_command" % __name__, svc.route_limits)
        logger.info("Received execute request for command: '%s'", command)
        if not safety.is_safe_kubectl_command(command):
            raise HTTPException(status_code=status.HTTP_400_BAD_REQUEST, detail="Command failed safety checks")
        execution_data = await execute_command_async(
            command, timeout=settings.EXECUTION_TIMEOUT, kubectl_bin=settings.KUBECTL_BIN,
            strict_compat=settings.COMPAT_STRICT_500)
        if "metadata" in execution_data:
            svc.metrics.execute_duration.observe(execution_data["metadata"]["duration_ms"] / 1000.0)
        # COMPAT_STRICT_500: a result without metadata raises KeyError -> plain-text 500 (quirk Q1).
        return _json(_command_body(command, False, execution_data))

    @app.post("/kubectl-command",
              response_model=CommandResponse,
              dependencies=[Depends(verify_api_key)],
              summary="Generate and optionally execute a kubectl command from natural language",
              responses={
                  200: {"description": "Command generated (and optionally executed)"},
                  400: {"description": "Invalid input query"},
                  401: {"description": "Unauthorized (Missing or invalid API Key)"},
                  422: {"description": "Unsafe command generated by LLM"},
                  429: {"description": "Rate limit exceeded"},
                  500: {"description": "Internal server error"},
                  503: {"description": "Service unavailable (LLM or execution issue)"},
                  504: {"description": "Gateway timeout (LLM or execution)"},
              })
    @limited
    async def get_kubectl_command(q: Query, request: Request):
        """Takes a natural language query, generates a kubectl command using the on-node LLM,
        validates it, and returns it (never executes; app.py:299-346)."""
        return await kubectl_command(q.query, request.scope)

    @app.get("/health",
             summary="Health check endpoint",
             status_code=status.HTTP_200_OK,
             responses={200: {"description": "Service is healthy"}})
    async def health_check():
        return {"status": "healthy"}

    @app.post("/execute",
              response_model=CommandResponse,
              dependencies=[Depends(verify_api_key)],
              summary="Execute a kubectl command",
              responses={
                  200: {"description": "Command executed successfully"},
                  400: {"description": "Invalid command"},
                  401: {"description": "Unauthorized (Missing or invalid API Key)"},
                  429: {"description": "Rate limit exceeded"},
                  500: {"description": "Internal server error"},
                  504: {"description": "Gateway timeout (execution)"},
              })
    @limited
    async def execute_kubectl_command(req: ExecuteRequest, request: Request):
        """Executes a provided kubectl command (app.py:369-389)."""
        return await execute(req.execute, request.scope)

    @app.get("/ready", summary="Readiness: 200 once the LLM backend can serve, else 503")
    async def readiness():
        ok = svc.backend is not None and svc.backend.healthy()
        body = {"status": "ready" if ok else "not ready", "backend": getattr(svc.backend, "name", None)}
        return _json(body, status_code=200 if ok else 503)

    from .openai_compat import install as _install_openai
    _install_openai(app, svc, settings)

    @app.get("/metrics", include_in_schema=True)
    async def metrics_endpoint():
        return Response(content=svc.metrics.render(), headers={"Content-Type": CONTENT_TYPE})

    # Middleware: fast path innermost, rate-limit, Prometheus outermost (app.py:134 then :138).
    if settings.API_FAST_PATH:
        app.add_middleware(FastPathMiddleware, settings=settings,
                           routes={"/kubectl-command": ("query", 3, kubectl_command),
                                   "/execute": ("execute", 0, execute)})
    app.add_middleware(RateLimitMiddleware, limiter=svc.limiter, exempt_endpoints=lambda: decorated,
                       routes=lambda: app.routes)
    app.add_middleware(PrometheusMiddleware, metrics=metrics, routes=lambda: app.routes)
    return app
