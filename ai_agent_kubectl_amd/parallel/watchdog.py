"""Worker liveness for tensor / expert parallel engines (SURVEY.md §5.3 'watchdog on worker
processes').

With TP/EP > 1, rank 0 runs the scheduler and every other rank mirrors its steps inside
`ModelRunner.worker_loop()`; a dead or wedged worker leaves rank 0 blocked in an RCCL collective
until the process-group timeout (minutes).  Two cheap signals catch that much earlier:

* `Heartbeat` (every worker rank): a daemon thread stamps `ka/hb/<rank>` = wall time in the
  process group's key-value store (the c10d TCPStore the ranks rendezvoused through) every
  `interval` seconds.  It is independent of the GPU stream, so a rank whose process died stops
  beating while one that is merely busy keeps beating;
* `Watchdog` (rank 0): a daemon thread that reads every worker's stamp and the engine's
  in-progress step start time; a stamp older than `hb_timeout` or a step running longer than
  `step_timeout` marks the engine unhealthy (`/ready` and new cache misses answer 503, the
  reference's degraded-mode status, `/root/reference/app.py:179-180`) and records why.

The reference has no counterpart (it is single-process, `/root/reference/app.py:400`).
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Callable, Optional, Sequence

logger = logging.getLogger("app.watchdog")


def default_store():
    """The default process group's store (None when torch.distributed is not initialised)."""
    try:
        import torch.distributed as dist

        if not dist.is_initialized():
            return None
        return dist.distributed_c10d._get_default_store()
    except Exception:  # pragma: no cover - private API moved
        return None


def _key(rank: int) -> str:
    return f"ka/hb/{rank}"


class Heartbeat:
    def __init__(self, store, rank: int, interval: float = 1.0):
        self.store, self.rank, self.interval = store, rank, interval
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def beat(self) -> None:
        self.store.set(_key(self.rank), repr(time.time()))

    def start(self) -> "Heartbeat":
        self.beat()
        self._thread = threading.Thread(target=self._run, name=f"ka-heartbeat-{self.rank}", daemon=True)
        self._thread.start()
        return self

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            try:
                self.beat()
            except Exception:  # store gone (rank 0 exited): nothing left to report to
                return

    def stop(self) -> None:
        self._stop.set()


class Watchdog:
    def __init__(self, store, worker_ranks: Sequence[int], on_fail: Callable[[str], None],
                 hb_timeout: float = 30.0, step_timeout: float = 120.0, interval: float = 1.0,
                 step_started: Optional[Callable[[], Optional[float]]] = None):
        self.store = store
        self.ranks = list(worker_ranks)
        self.on_fail = on_fail
        self.hb_timeout, self.step_timeout, self.interval = hb_timeout, step_timeout, interval
        self.step_started = step_started
        self.failed: Optional[str] = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._t0 = time.time()

    def check(self, now: Optional[float] = None) -> Optional[str]:
        """One scan; returns the failure reason (also passed to on_fail once) or None."""
        now = time.time() if now is None else now
        reason = None
        for r in self.ranks:
            k = _key(r)
            try:
                seen = float(self.store.get(k)) if self.store.check([k]) else None
            except Exception as e:  # store unreachable
                reason = f"heartbeat store unreachable: {e}"
                break
            last = seen if seen is not None else self._t0   # grace period until the first beat
            if now - last > self.hb_timeout:
                reason = f"TP/EP worker rank {r} heartbeat lost ({now - last:.1f} s > {self.hb_timeout:.0f} s)"
                break
        if reason is None and self.step_started is not None:
            t = self.step_started()
            if t is not None and time.perf_counter() - t > self.step_timeout:
                reason = f"engine step stalled for {time.perf_counter() - t:.1f} s (> {self.step_timeout:.0f} s)"
        if reason is not None and self.failed is None:
            self.failed = reason
            logger.error(reason)
            self.on_fail(reason)
        return reason

    def start(self) -> "Watchdog":
        self._thread = threading.Thread(target=self._run, name="ka-watchdog", daemon=True)
        self._thread.start()
        return self

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            if self.check() is not None:
                return

    def stop(self) -> None:
        self._stop.set()
