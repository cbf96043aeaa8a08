"""Fixed-window, in-memory, per-client rate limiting.

Re-implements the behaviour of `slowapi.Limiter(key_func=get_remote_address,
default_limits=[RATE_LIMIT])` + `SlowAPIMiddleware` + `@limiter.limit(RATE_LIMIT)` as wired at
`/root/reference/app.py:128,132-134,298,368`:

* limit strings: `"N/unit"`, `"N per unit"`, `"N per M units"`; several joined by `;`, `,` or `|`;
  units second/minute/hour/day/month(30d)/year(360d), optional plural `s`;
* fixed window that starts at the first hit of a (limit, client, scope) key and lasts the unit;
  every hit increments (also over the limit), limits are evaluated in order and evaluation stops
  at the first one that is exceeded;
* key = client IP (`request.client.host`, `127.0.0.1` when absent) + route scope;
* the two decorated POST routes are checked *inside* the endpoint (after auth 401 and body 422)
  and are skipped by the middleware; every other FULL-matched route gets the default limits from
  the middleware; unmatched paths / method mismatches are never limited;
* 429 body: `{"error":"Rate limit exceeded: 10 per 1 minute"}`, no `X-RateLimit-*` headers.
"""
from __future__ import annotations

import re
import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

_GRANULARITY = {
    "second": 1,
    "minute": 60,
    "hour": 3600,
    "day": 86400,
    "month": 2592000,
    "year": 31104000,
}
_SEPARATORS = re.compile(r"[,;|]{1}")
_SINGLE = re.compile(
    r"^\s*([0-9]+)\s*(?:/|\s*per\s*)\s*([0-9]+)*\s*(hour|minute|second|day|month|year)s?\s*$",
    re.IGNORECASE,
)


@dataclass(frozen=True)
class RateLimitItem:
    amount: int
    multiples: int
    granularity: str

    @property
    def expiry(self) -> int:
        return _GRANULARITY[self.granularity] * self.multiples

    def __str__(self) -> str:  # `limits` RateLimitItem.__repr__ format, used in the 429 body
        return "%d per %d %s" % (self.amount, self.multiples, self.granularity)


def parse_many(spec: str) -> List[RateLimitItem]:
    if not spec or not spec.strip():
        raise ValueError("empty rate limit string")
    items = []
    for part in _SEPARATORS.split(spec):
        m = _SINGLE.match(part)
        if not m:
            raise ValueError("couldn't parse rate limit string '%s'" % spec)
        amount, mult, gran = m.groups()
        items.append(RateLimitItem(int(amount), int(mult or 1), gran.lower()))
    return items


class RateLimitExceeded(Exception):
    def __init__(self, limit: RateLimitItem):
        super().__init__(str(limit))
        self.limit = limit
        self.detail = str(limit)


class FixedWindowLimiter:
    """Memory-storage fixed window keyed by (limit, client, scope)."""

    def __init__(self, default_limits: Sequence[RateLimitItem], timer: Callable[[], float] = time.time,
                 enabled: bool = True):
        self.default_limits = list(default_limits)
        self.timer = timer
        self.enabled = enabled
        self._counts: Dict[Tuple, List[float]] = {}   # key -> [count, window_end]
        self._lock = threading.Lock()
        self._last_gc = 0.0

    def _gc(self, now: float) -> None:
        if now - self._last_gc < 1.0:
            return
        self._last_gc = now
        dead = [k for k, v in self._counts.items() if v[1] <= now]
        for k in dead:
            del self._counts[k]

    def hit(self, item: RateLimitItem, client: str, scope: str) -> bool:
        """One fixed-window hit; True while within the limit (limits.FixedWindowRateLimiter.hit)."""
        now = self.timer()
        key = (item.amount, item.multiples, item.granularity, client, scope)
        with self._lock:
            self._gc(now)
            ent = self._counts.get(key)
            if ent is None or ent[1] <= now:
                ent = [0, now + item.expiry]
                self._counts[key] = ent
            ent[0] += 1
            return ent[0] <= item.amount

    def check(self, client: str, scope: str, limits: Optional[Iterable[RateLimitItem]] = None) -> None:
        """Evaluate limits in order; raise RateLimitExceeded at the first violated one."""
        if not self.enabled:
            return
        for item in (self.default_limits if limits is None else limits):
            if not self.hit(item, client, scope):
                raise RateLimitExceeded(item)

    def reset(self) -> None:
        with self._lock:
            self._counts.clear()


def client_address(scope) -> str:
    """slowapi.util.get_remote_address: request.client.host or 127.0.0.1."""
    client = scope.get("client")
    if client and client[0]:
        return client[0]
    return "127.0.0.1"


def rate_limit_body(exc: RateLimitExceeded) -> bytes:
    return ('{"error":"Rate limit exceeded: %s"}' % exc.detail).encode()


class RateLimitMiddleware:
    """Pure-ASGI equivalent of SlowAPIMiddleware (default limits for non-decorated routes)."""

    def __init__(self, app, limiter: FixedWindowLimiter, exempt_endpoints: Callable[[], set],
                 routes: Callable[[], list]):
        self.app = app
        self.limiter = limiter
        self.exempt_endpoints = exempt_endpoints
        self.routes = routes

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http" or not self.limiter.enabled:
            await self.app(scope, receive, send)
            return
        from .metrics import match_route

        full, _ = match_route(scope, self.routes())
        handler = getattr(full, "endpoint", None)
        if handler is not None:
            name = "%s.%s" % (handler.__module__, handler.__name__)
            if name not in self.exempt_endpoints():
                try:
                    self.limiter.check(client_address(scope), name)
                except RateLimitExceeded as exc:
                    body = rate_limit_body(exc)
                    await send({"type": "http.response.start", "status": 429,
                                "headers": [(b"content-length", str(len(body)).encode()),
                                            (b"content-type", b"application/json")]})
                    await send({"type": "http.response.body", "body": body})
                    return
        await self.app(scope, receive, send)
