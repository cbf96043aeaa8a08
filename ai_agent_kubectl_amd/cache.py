"""TTL + LRU response cache.

Re-implements the `cachetools.TTLCache(maxsize, ttl)` semantics the reference relies on
(`/root/reference/app.py:125`, used at `:312` and `:322`):

* timer is `time.monotonic` (injectable for tests);
* every set stamps `expires = now + ttl` and makes the key most-recently-used;
* expired items are purged on mutation and are invisible to `get`, `in` and `[]`;
* when full, the least-recently-used live item is evicted; `get`/`in` count as a use;
* `maxsize == 0` rejects every insert with `ValueError("value too large")` (cachetools' message).

Key = sanitised query, value = generated command (only successful generations are stored).
"""
from __future__ import annotations

import collections
import time
from typing import Any, Callable, Hashable, Optional


class TTLCache:
    __slots__ = ("maxsize", "ttl", "timer", "_data", "_exp", "hits", "misses")

    def __init__(self, maxsize: int, ttl: float, timer: Callable[[], float] = time.monotonic):
        self.maxsize = int(maxsize)
        self.ttl = ttl
        self.timer = timer
        # key -> [value, expires]; order = LRU (first) ... MRU (last)
        self._data: "collections.OrderedDict[Hashable, list]" = collections.OrderedDict()
        # (expires, key) in stamp order: with a constant ttl and a monotonic timer the stamps are
        # non-decreasing, so expiry pops from the left instead of scanning every entry per insert
        self._exp: "collections.deque" = collections.deque()
        self.hits = 0
        self.misses = 0

    # -- internals -----------------------------------------------------------------------
    def _live(self, key, now: float) -> Optional[list]:
        ent = self._data.get(key)
        if ent is None:
            return None
        if not now < ent[1]:
            return None
        self._data.move_to_end(key)
        return ent

    def expire(self, now: Optional[float] = None) -> None:
        now = self.timer() if now is None else now
        exp, data = self._exp, self._data
        while exp and not now < exp[0][0]:
            t, k = exp.popleft()
            ent = data.get(k)
            if ent is not None and ent[1] == t:   # stale stamps (key re-set or evicted) are skipped
                del data[k]
        if len(exp) > 4 * max(16, len(data)):     # drop stale stamps left by re-sets / evictions
            self._exp = collections.deque(sorted(((e[1], k) for k, e in data.items()), key=lambda x: x[0]))

    # -- mapping API -----------------------------------------------------------------------
    def get(self, key, default: Any = None) -> Any:
        ent = self._live(key, self.timer())
        if ent is None:
            self.misses += 1
            return default
        self.hits += 1
        return ent[0]

    def __contains__(self, key) -> bool:
        return self._live(key, self.timer()) is not None

    def __getitem__(self, key):
        ent = self._live(key, self.timer())
        if ent is None:
            raise KeyError(key)
        return ent[0]

    def __setitem__(self, key, value) -> None:
        now = self.timer()
        self.expire(now)
        if self.maxsize < 1:
            raise ValueError("value too large")
        if key in self._data:
            ent = self._data[key]
            ent[0] = value
            ent[1] = now + self.ttl
            self._data.move_to_end(key)
            self._exp.append((ent[1], key))
            return
        while len(self._data) >= self.maxsize:
            self._data.popitem(last=False)
        self._data[key] = [value, now + self.ttl]
        self._exp.append((now + self.ttl, key))

    def __delitem__(self, key) -> None:
        del self._data[key]

    def __len__(self) -> int:
        now = self.timer()
        return sum(1 for e in self._data.values() if now < e[1])

    def clear(self) -> None:
        self._data.clear()
        self._exp.clear()

    @property
    def currsize(self) -> int:
        return len(self)
