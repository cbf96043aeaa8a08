"""Service state shared by several API worker processes (response cache + rate-limit windows).

The reference runs one uvicorn worker with a process-local `TTLCache` and an in-memory slowapi
limiter (`/root/reference/app.py:125,128,400`).  One worker tops out near 1.3k req/s on this host
(profiles/service_plumbing_gpu_box.log), so serving several GPUs needs several API workers — and
then the cache and the limiter must stay global: a query answered by worker A has to be
`from_cache: true` on worker B (`app.py:312-322`), and a client's `10/minute` is one budget, not
one per worker.  Both live in one POSIX shared-memory segment managed by the C++ runtime
(`runtime/shared_state.h`, robust process-shared mutex); this module gives them the exact
interfaces of `cache.TTLCache` and `ratelimit.FixedWindowLimiter` so the service code is unchanged.

Enable with `SHARED_STATE=<name>` (serve.py sets it for `WORKERS > 1`).  Every process opening the
same name attaches to the same segment; the first one creates it.
"""
from __future__ import annotations

import hashlib
import os
import time
from typing import Any, Callable, Optional, Sequence

from .ratelimit import FixedWindowLimiter, RateLimitItem

VALUE_MAX = int(os.environ.get("SHARED_STATE_VALUE_MAX", "4096"))   # bytes of one cached command
LIMITER_KEYS = int(os.environ.get("SHARED_STATE_LIMITER_KEYS", "65536"))


def _native():
    from .runtime import native
    if native._native is None:
        raise RuntimeError("SHARED_STATE needs the native runtime (python -c 'import __graft_entry__ as g; g.build()')")
    return native._native


def digest(text: str) -> bytes:
    """128-bit BLAKE2b of the key text: any query length maps to a fixed, collision-resistant key."""
    return hashlib.blake2b(text.encode("utf-8", "surrogatepass"), digest_size=16).digest()


def shm_name(name: str) -> str:
    return name if name.startswith("/") else "/" + name


class SharedStore:
    """One named segment: `cache_capacity` cache entries + the limiter table."""

    def __init__(self, name: str, cache_capacity: int, value_max: int = VALUE_MAX, limiter_keys: int = LIMITER_KEYS,
                 recreate: bool = True):
        """Create or attach.  A segment left behind by an earlier run with another layout (a changed
        VALUE_MAX / capacity / version) is replaced instead of failing every worker (`recreate`)."""
        self.name = shm_name(name)
        args = (self.name, max(1, int(cache_capacity)), int(value_max), int(limiter_keys))
        try:
            self._s = _native().SharedState(*args)
        except RuntimeError as e:
            if not recreate or "incompatible layout" not in str(e):
                raise
            self.unlink(self.name)
            self._s = _native().SharedState(*args)

    @property
    def raw(self):
        return self._s

    def stats(self) -> dict:
        return self._s.stats()

    # DP routing load (parallel/dp.py): in-flight requests per (API worker, replica)
    def load_set(self, worker: int, replica: int, value: int) -> None:
        self._s.load_set(int(worker), int(replica), int(value))

    def load_clear_worker(self, worker: int) -> None:
        self._s.load_clear_worker(int(worker))

    def load_total(self, replica: int) -> int:
        return self._s.load_total(int(replica))

    def load_pick(self, n: int, live_mask: int) -> int:
        """Least-loaded live replica over every worker's in-flight counts (-1: none live)."""
        return self._s.load_pick(int(n), int(live_mask))

    @staticmethod
    def unlink(name: str) -> None:
        """Remove the segment name (processes that still map it keep working)."""
        try:
            _native().SharedState.unlink(shm_name(name))
        except Exception:  # pragma: no cover
            pass


class SharedTTLCache:
    """`cache.TTLCache` semantics over the shared segment (LRU at `maxsize`, per-item TTL stamped
    on every set, expired items invisible and purged on mutation, `get`/`in` count as a use).
    A value longer than the segment's value slot is not stored (the request is served uncached)."""

    def __init__(self, store: SharedStore, maxsize: int, ttl: float, timer: Callable[[], float] = time.monotonic):
        self.store = store
        self._s = store.raw
        self.maxsize = int(maxsize)
        self.ttl = ttl
        self.timer = timer
        self.hits = 0
        self.misses = 0

    def get(self, key, default: Any = None) -> Any:
        v = self._s.cache_get(digest(key), self.timer())
        if v is None:
            self.misses += 1
            return default
        self.hits += 1
        return v.decode("utf-8", "surrogatepass")

    def __contains__(self, key) -> bool:
        return self._s.cache_contains(digest(key), self.timer())

    def __getitem__(self, key):
        v = self._s.cache_get(digest(key), self.timer())
        if v is None:
            raise KeyError(key)
        return v.decode("utf-8", "surrogatepass")

    def __setitem__(self, key, value) -> None:
        if self.maxsize < 1:
            raise ValueError("value too large")
        self._s.cache_set(digest(key), str(value).encode("utf-8", "surrogatepass"), self.timer(), float(self.ttl),
                          self.maxsize)

    def __delitem__(self, key) -> None:
        if not self._s.cache_delete(digest(key)):
            raise KeyError(key)

    def __len__(self) -> int:
        return self._s.cache_len(self.timer())

    def clear(self) -> None:
        self._s.cache_clear()

    @property
    def currsize(self) -> int:
        return len(self)


class SharedFixedWindowLimiter(FixedWindowLimiter):
    """`ratelimit.FixedWindowLimiter` whose windows live in the shared segment: every worker
    counts against the same (limit, client, scope) window."""

    def __init__(self, store: SharedStore, default_limits: Sequence[RateLimitItem],
                 timer: Callable[[], float] = time.time, enabled: bool = True):
        super().__init__(default_limits, timer=timer, enabled=enabled)
        self._s = store.raw

    def hit(self, item: RateLimitItem, client: str, scope: str) -> bool:
        key = digest("%d|%d|%s|%s|%s" % (item.amount, item.multiples, item.granularity, client, scope))
        return self._s.limiter_hit(key, item.amount, float(item.expiry), self.timer())

    def reset(self) -> None:
        self._s.limiter_reset()


def open_from_settings(settings) -> Optional[SharedStore]:
    """Attach to the segment the supervisor created (serve.py / parallel/workers.run_workers owns it
    and replaces stale layouts itself).  An attaching worker never recreates it: a layout mismatch
    fails loudly instead of silently unlinking the live segment and serving from a private one."""
    name = getattr(settings, "SHARED_STATE", "") or ""
    if not name:
        return None
    return SharedStore(name, settings.CACHE_MAXSIZE, recreate=False)
