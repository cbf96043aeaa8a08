"""Prometheus instrumentation.

HTTP metrics reproduce what `Instrumentator().instrument(app).expose(app)` gives the reference
(`/root/reference/app.py:136-138`; prometheus-fastapi-instrumentator 7.0.0 defaults, SURVEY.md
Appendix B.3):

* `http_requests_total{method,status,handler}` — status grouped to `2xx`/`4xx`/...;
* `http_request_size_bytes{handler}` / `http_response_size_bytes{handler}` — Summaries of the
  Content-Length headers (0 when absent);
* `http_request_duration_seconds{method,handler}` — buckets 0.1, 0.5, 1, +Inf;
* `http_request_duration_highr_seconds` — unlabelled, 21 buckets 0.01 … 60;
* default `process_*` / `python_*` collectors;
* handler = route template (`none` for unmatched paths); `/metrics` itself is instrumented;
  the middleware is outermost so 401/429/500 are counted.

Engine/business metrics are added on top (SURVEY.md §5.5 target): cache hit/miss counters, LLM
TTFT/TPOT/latency histograms, batch size, queue depth and KV-block usage gauges.

Each app gets its own `CollectorRegistry` so that several apps can live in one process (tests,
DP replicas) without duplicate-registration errors.
"""
from __future__ import annotations

import bisect
import os
import time
from typing import Callable, List, Optional

from prometheus_client import (CollectorRegistry, Counter, GCCollector, Gauge, Histogram,
                               PlatformCollector, ProcessCollector, Summary, generate_latest)

CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"
HIGHR_BUCKETS = (0.01, 0.025, 0.05, 0.075, 0.1, 0.25, 0.5, 0.75, 1, 1.5, 2, 2.5, 3, 3.5, 4, 4.5,
                 5, 7.5, 10, 30, 60)
LOWR_BUCKETS = (0.1, 0.5, 1)


class ServiceMetrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None, default_collectors: bool = True):
        r = self.registry = registry or CollectorRegistry(auto_describe=True)
        if default_collectors:
            ProcessCollector(registry=r)
            PlatformCollector(registry=r)
            GCCollector(registry=r)
        self.requests_total = Counter(
            "http_requests_total", "Total number of requests by method, status and handler.",
            ("method", "status", "handler"), registry=r)
        self.request_size = Summary(
            "http_request_size_bytes",
            "Content length of incoming requests by handler. Only value of header is respected. "
            "Otherwise ignored. No percentile calculated. ", ("handler",), registry=r)
        self.response_size = Summary(
            "http_response_size_bytes",
            "Content length of outgoing responses by handler. Only value of header is respected. "
            "Otherwise ignored. No percentile calculated. ", ("handler",), registry=r)
        self.latency_highr = Histogram(
            "http_request_duration_highr_seconds",
            "Latency with many buckets but no API specific labels. Made for more accurate "
            "percentile calculations. ", buckets=HIGHR_BUCKETS, registry=r)
        self.latency_lowr = Histogram(
            "http_request_duration_seconds",
            "Latency with only few buckets by handler. Made to be only used if aggregation by "
            "handler is important. ", ("method", "handler"), buckets=LOWR_BUCKETS, registry=r)
        # --- engine / business metrics (not in the reference) ---
        self.cache_hits = Counter("kubectl_agent_cache_hits_total", "Response cache hits.", registry=r)
        self.cache_misses = Counter("kubectl_agent_cache_misses_total", "Response cache misses.", registry=r)
        self.llm_latency = Histogram("llm_request_seconds", "End-to-end LLM generation latency.",
                                     buckets=HIGHR_BUCKETS, registry=r)
        self.llm_ttft = Histogram("llm_ttft_seconds", "Time to first token.", buckets=HIGHR_BUCKETS, registry=r)
        self.llm_tpot = Histogram("llm_tpot_seconds", "Time per output token after the first.",
                                  buckets=(0.001, 0.002, 0.003, 0.005, 0.0075, 0.01, 0.02, 0.05, 0.1, 0.25),
                                  registry=r)
        self.llm_queue_wait = Histogram("llm_queue_wait_seconds",
                                        "Arrival to first admission into a prefill step.",
                                        buckets=HIGHR_BUCKETS, registry=r)
        self.llm_step = Histogram("llm_step_seconds", "Engine step time (launch or previous readback to "
                                  "readback) by phase.", ("phase",),
                                  buckets=(0.001, 0.002, 0.004, 0.006, 0.008, 0.01, 0.015, 0.02, 0.03, 0.05, 0.1,
                                           0.2, 0.5, 1.0), registry=r)
        self.llm_batch_size = Gauge("llm_batch_size", "Sequences in the last engine step.", registry=r)
        self.llm_queue_depth = Gauge("llm_queue_depth", "Requests waiting for the engine.", registry=r)
        self.llm_kv_blocks_used = Gauge("llm_kv_blocks_used", "Paged-KV blocks in use.", registry=r)
        self.llm_errors = Counter("llm_errors_total", "LLM failures by kind.", ("kind",), registry=r)
        self.rccl_allreduce = Histogram("rccl_allreduce_seconds",
                                        "Eager tensor-parallel all-reduce time (RCCL or one-shot IPC kernel).",
                                        buckets=(1e-5, 2.5e-5, 5e-5, 1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2,
                                                 5e-2), registry=r)
        self.rccl_allreduce_bytes = Counter("rccl_allreduce_bytes", "Bytes all-reduced across the TP group "
                                            "(eager and graph-captured calls at capture time).", registry=r)
        self.execute_duration = Histogram("execute_duration_seconds", "kubectl subprocess wall time.",
                                          buckets=HIGHR_BUCKETS, registry=r)
        self.loop_lag = Histogram("event_loop_lag_seconds", "asyncio event-loop scheduling delay (50 ms probe).",
                                  buckets=(0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0), registry=r)

        self.flush_hooks: List[Callable[[], None]] = []   # pending HTTP observations (PrometheusMiddleware)

    def render(self) -> bytes:
        for flush in self.flush_hooks:
            flush()
        mdir = os.environ.get("PROMETHEUS_MULTIPROC_DIR")
        if mdir:   # several API workers (parallel/workers.py): aggregate every worker's samples
            from prometheus_client import multiprocess
            reg = CollectorRegistry()
            multiprocess.MultiProcessCollector(reg, path=mdir)
            return generate_latest(reg)
        return generate_latest(self.registry)


_ROUTE_CACHE: dict = {}


def match_route(scope, routes):
    """(full_route, partial_route) for (method, path), memoised: the app's routes are static
    and the paths they match are exact (no path parameters in this service)."""
    key = (id(routes), scope.get("method"), scope.get("path"))
    hit = _ROUTE_CACHE.get(key)
    if hit is not None:
        return hit
    from starlette.routing import Match

    full = partial = None
    for route in routes:
        match, _ = route.matches(scope)
        if match == Match.FULL:
            full = route
            break
        if match == Match.PARTIAL and partial is None:
            partial = route
    if len(_ROUTE_CACHE) > 4096:
        _ROUTE_CACHE.clear()
    _ROUTE_CACHE[key] = (full, partial)
    return full, partial


def _route_name(scope, routes) -> str:
    full, partial = match_route(scope, routes)
    if full is not None:
        return full.path
    return partial.path if partial is not None else "none"


class PrometheusMiddleware:
    """Pure-ASGI HTTP instrumentation (the Instrumentator middleware's observable behaviour)."""

    def __init__(self, app, metrics: ServiceMetrics, routes: Callable[[], list]):
        self.app = app
        self.metrics = metrics
        self.routes = routes
        self._children = {}
        self._pending: list = []
        metrics.flush_hooks.append(self.flush)
        # KA_WORKER_HEADER=1 adds `x-ka-worker: <pid>` to every response (tests of the multi-worker
        # tier); off by default so the wire format stays the reference's
        self.worker_header = ((b"x-ka-worker", str(os.getpid()).encode())
                              if os.environ.get("KA_WORKER_HEADER") == "1" else None)

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            await self.app(scope, receive, send)
            return
        start = time.perf_counter()
        status = [500]
        resp_len = [0]

        async def send_wrapper(message):
            if message["type"] == "http.response.start":
                status[0] = message["status"]
                for k, v in message.get("headers", ()):
                    if k == b"content-length":
                        resp_len[0] = int(v)
                        break
                if self.worker_header is not None:   # opt-in diagnostics: which API worker answered
                    message = dict(message, headers=list(message.get("headers", ())) + [self.worker_header])
            await send(message)

        try:
            await self.app(scope, receive, send_wrapper)
        finally:
            dur = time.perf_counter() - start
            handler = _route_name(scope, self.routes())
            method = scope.get("method", "GET")
            req_len = 0
            for k, v in scope.get("headers", ()):
                if k == b"content-length":
                    try:
                        req_len = int(v)
                    except ValueError:
                        req_len = 0
                    break
            key = (method, status[0] // 100, handler)
            children = self._children.get(key)
            if children is None:   # labelled children are resolved once per (method, class, handler)
                m = self.metrics
                children = (m.requests_total.labels(method, "%dxx" % key[1], handler), m.request_size.labels(handler),
                            m.response_size.labels(handler), m.latency_lowr.labels(method, handler))
                if len(self._children) < 4096:
                    self._children[key] = children
            # recorded now, applied in bulk (every FLUSH_EVERY requests and before every /metrics
            # render): a request then costs one list append instead of a dozen lock-protected
            # counter / summary / histogram updates on the event loop
            self._pending.append((children, req_len, resp_len[0], dur))
            if len(self._pending) >= self.FLUSH_EVERY:
                self.flush()

    FLUSH_EVERY = 256

    def flush(self) -> None:
        """Apply the pending observations: per labelled child one count / sum increment and one
        increment per touched histogram bucket (the same values prometheus_client's observe()
        would have produced one by one; bucket = first upper bound >= the value)."""
        pend, self._pending = self._pending, []
        if not pend:
            return
        agg = {}
        hr = self.metrics.latency_highr
        hr_bounds = hr._upper_bounds
        hr_counts = [0] * len(hr_bounds)
        hr_sum = 0.0
        for children, req_len, resp_len, dur in pend:
            a = agg.get(id(children))
            if a is None:
                a = agg[id(children)] = [children, 0, 0.0, 0.0, 0.0, [0] * len(children[3]._upper_bounds)]
            a[1] += 1
            a[2] += req_len
            a[3] += resp_len
            a[4] += dur
            a[5][bisect.bisect_left(children[3]._upper_bounds, dur)] += 1
            hr_counts[bisect.bisect_left(hr_bounds, dur)] += 1
            hr_sum += dur
        for children, n, req_sum, resp_sum, dur_sum, counts in agg.values():
            children[0]._value.inc(n)
            for summ, total in ((children[1], req_sum), (children[2], resp_sum)):
                summ._count.inc(n)
                summ._sum.inc(total)
            lowr = children[3]
            lowr._sum.inc(dur_sum)
            for i, c in enumerate(counts):
                if c:
                    lowr._buckets[i].inc(c)
        hr._sum.inc(hr_sum)
        for i, c in enumerate(hr_counts):
            if c:
                hr._buckets[i].inc(c)
