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
import contextlib
import json
import logging
from typing import Any, Dict, Optional

from fastapi import Depends, FastAPI, Header, HTTPException, Request, status
from fastapi.responses import JSONResponse, Response

from .. import safety
from ..cache import TTLCache
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


async def _lag_probe(metrics, period: float = 0.05) -> None:
    """Observe how late the event loop wakes a 50 ms sleeper (GIL / blocking-call diagnostics)."""
    loop = asyncio.get_running_loop()
    while True:
        t0 = loop.time()
        await asyncio.sleep(period)
        metrics.loop_lag.observe(max(0.0, loop.time() - t0 - period))


class KubectlService:
    """State shared by the routes: settings, cache, limiter, metrics and the LLM backend."""

    def __init__(self, settings: Settings, backend: Optional[LLMBackend], metrics: ServiceMetrics):
        self.settings = settings
        self.backend = backend
        self.metrics = metrics
        self.cache = TTLCache(maxsize=settings.CACHE_MAXSIZE, ttl=settings.CACHE_TTL)
        self.route_limits = parse_many(settings.RATE_LIMIT)
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
        try:
            command = await asyncio.wait_for(_chain(), timeout=timeout)
            self.metrics.llm_latency.observe(loop.time() - t0)
            logger.info(f"LLM generated command for query '{query}': {command}")
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
            raise HTTPException(status_code=status.HTTP_422_UNPROCESSABLE_ENTITY,
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
        svc.limiter.check(client_address(request.scope), "%s.get_kubectl_command" % __name__, svc.route_limits)
        logger.info(f"Received query: '{q.query}'")
        sanitized_query = safety.sanitize_query(q.query)
        from_cache = False
        try:
            cached = svc.cache.get(sanitized_query)
            if cached is not None:
                logger.info(f"Cache hit for query: {sanitized_query}")
                svc.metrics.cache_hits.inc()
                command = cached
                from_cache = True
            else:
                logger.info(f"Cache miss for query: {sanitized_query}")
                svc.metrics.cache_misses.inc()
                logger.debug(f"Calling LLM for query: {sanitized_query}")
                command = await svc.run_llm(sanitized_query)
                svc.cache[sanitized_query] = command
                logger.debug(f"Stored result in cache for query: {sanitized_query}")
        except HTTPException:
            raise
        except Exception as e:
            logger.exception(f"Unexpected error processing query '{sanitized_query}': {e}")
            raise HTTPException(status_code=status.HTTP_500_INTERNAL_SERVER_ERROR,
                                detail="Internal server error processing request")
        now = utcnow_iso()
        execution_data = {"metadata": {"start_time": now, "end_time": utcnow_iso(), "duration_ms": 0.0,
                                       "success": True}}
        return _json(_command_body(command, from_cache, execution_data))

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
        svc.limiter.check(client_address(request.scope), "%s.execute_kubectl_command" % __name__,
                          svc.route_limits)
        logger.info(f"Received execute request for command: '{req.execute}'")
        if not safety.is_safe_kubectl_command(req.execute):
            raise HTTPException(status_code=status.HTTP_400_BAD_REQUEST, detail="Command failed safety checks")
        execution_data = await execute_command_async(
            req.execute, timeout=settings.EXECUTION_TIMEOUT, kubectl_bin=settings.KUBECTL_BIN,
            strict_compat=settings.COMPAT_STRICT_500)
        if "metadata" in execution_data:
            svc.metrics.execute_duration.observe(execution_data["metadata"]["duration_ms"] / 1000.0)
        # COMPAT_STRICT_500: a result without metadata raises KeyError -> plain-text 500 (quirk Q1).
        return _json(_command_body(req.execute, False, execution_data))

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

    # Middleware: rate-limit inner, Prometheus outermost (app.py:134 then :138).
    app.add_middleware(RateLimitMiddleware, limiter=svc.limiter, exempt_endpoints=lambda: decorated,
                       routes=lambda: app.routes)
    app.add_middleware(PrometheusMiddleware, metrics=metrics, routes=lambda: app.routes)
    return app
