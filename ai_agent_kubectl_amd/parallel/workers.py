"""Multi-worker HTTP tier: W API worker processes on one port + the engine replicas they share.

The reference serves from one uvicorn worker (`/root/reference/app.py:400`, `Dockerfile:33`); one
worker's HTTP + JSON handling caps near 1.3k req/s on this host, below what one MI355X engine
completes, and far below 8 GPUs' worth.  `serve.py` with WORKERS > 1 runs this supervisor:

  supervisor (no GPU use)
   ├─ shared-memory segment: response cache + rate-limit windows (shared_state.py), so
   │  `from_cache` (app.py:312-322) and 429 (app.py:298,368) stay global across workers
   ├─ DP engine replicas (dp.ReplicaSupervisor), each a TP group of TP devices, each serving all
   │  W workers over its Unix socket; a replica that dies is respawned
   └─ W API workers: each binds HOST:PORT with SO_REUSEPORT (the kernel spreads connections),
      runs the full app (auth, validation, limiter, cache, Prometheus) under uvicorn and routes
      its misses to the least-loaded replica.  /metrics aggregates every worker
      (prometheus_client multiprocess mode: PROMETHEUS_MULTIPROC_DIR).

A dead API worker is respawned too (its socket is re-bound with SO_REUSEPORT; the kernel stops
routing to the dead one's).  SIGTERM / SIGINT stop everything and remove the shared-memory segment
and the metrics directory.
"""
from __future__ import annotations

import dataclasses
import logging
import os
import shutil
import signal
import socket
import tempfile
import time

log = logging.getLogger("app")

MAX_WORKERS = 64   # rows of the shared load table (runtime/shared_state.h kMaxWorkers)


def bind_reuseport(host: str, port: int) -> socket.socket:
    """The worker's listening socket.  Created with proto=IPPROTO_TCP, as getaddrinfo's sockets are:
    asyncio turns Nagle off (TCP_NODELAY) only on accepted sockets whose proto says TCP, and with
    Nagle on, uvicorn's two writes per response (head, then body) wait for the client's delayed ACK
    — +40 ms on every request (profiles/r3/README.md)."""
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(fam, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    s.set_inheritable(True)
    return s


def _api_worker(idx: int, settings_dict: dict, host: str, port: int, endpoints, metrics_dir: str) -> None:
    """One API worker process (spawned): the app + uvicorn on a SO_REUSEPORT socket."""
    from ..utils.runtime import set_proc_name
    set_proc_name(f"ka-api-{idx}")
    if metrics_dir:   # before prometheus_client is imported: multiprocess value storage
        os.environ["PROMETHEUS_MULTIPROC_DIR"] = metrics_dir
    import asyncio

    import uvicorn

    from ..api import create_app
    from ..config import Settings
    from ..llm.base import build_backend

    settings = Settings(**settings_dict)
    logging.basicConfig(level=settings.log_level, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    if endpoints is not None:
        from .dp import DPRouterLLM
        backend = DPRouterLLM(settings, len(endpoints.addresses), endpoints=endpoints, client_id=idx)
    else:
        try:
            backend = build_backend(settings)
        except Exception:
            logging.getLogger("app").exception("Failed to initialize LLM backend.")
            backend = None
    app = create_app(settings, backend=backend)
    sock = bind_reuseport(host, port)
    config = uvicorn.Config(app, log_level=settings.LOG_LEVEL.lower(),
                            timeout_keep_alive=int(os.environ.get("KEEP_ALIVE_S", "75")))
    server = uvicorn.Server(config)
    asyncio.run(server.serve(sockets=[sock]))


def run_workers(settings, host: str, port: int) -> int:
    import multiprocessing as mp

    from ..shared_state import SharedStore
    from .dp import ReplicaSupervisor

    W = max(1, int(settings.WORKERS))
    if W > MAX_WORKERS:   # the shared load table has one row per worker (runtime/shared_state.h)
        raise ValueError(f"WORKERS={W} exceeds the shared state's {MAX_WORKERS} worker rows")
    name = settings.SHARED_STATE or "/ka_state_%d" % os.getpid()
    SharedStore.unlink(name)   # this supervisor owns the segment: never inherit an earlier run's cache
    store = SharedStore(name, settings.CACHE_MAXSIZE, recreate=True)   # created before any worker attaches
    metrics_dir = tempfile.mkdtemp(prefix="ka_prom_")
    sd = dataclasses.asdict(settings)
    sd["SHARED_STATE"] = store.name
    directory = None
    sup = None
    if settings.LLM_BACKEND.lower() == "engine":
        sup = ReplicaSupervisor(settings).start()
        directory = sup.directory
        log.info("DP=%d replicas (TP=%d each: %s) serving %d API workers", len(sup.specs), settings.TP,
                 " | ".join(",".join(d) for d in sup.devices), W)
    ctx = mp.get_context("spawn")

    def spawn_worker(i):
        p = ctx.Process(target=_api_worker, args=(i, sd, host, port, directory, metrics_dir), daemon=False)
        p.start()
        return p

    workers = [spawn_worker(i) for i in range(W)]
    restarts = [0] * W
    gone = set()   # workers that stay down (restart cap reached / stopping)
    log.info("Started %d API workers on %s:%d (shared state %s)", W, host, port, store.name)

    stop = {"flag": False}

    def _stop(signum, frame):
        stop["flag"] = True

    signal.signal(signal.SIGTERM, _stop)
    signal.signal(signal.SIGINT, _stop)
    rc = 0
    try:
        while not stop["flag"]:
            for i, p in enumerate(workers):
                if p.is_alive() or i in gone:
                    continue
                # a dead worker's in-flight counts must not skew everyone else's routing
                store.load_clear_worker(i)
                if not stop["flag"] and restarts[i] < 5:
                    log.error("API worker %d exited (status %s): respawning", i, p.exitcode)
                    restarts[i] += 1
                    workers[i] = spawn_worker(i)
                else:
                    gone.add(i)
            if all(not p.is_alive() for p in workers):
                rc = 1
                break
            time.sleep(0.2)
    finally:
        for p in workers:
            if p.is_alive():
                p.terminate()
        for p in workers:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
        if sup is not None:
            sup.stop()
        SharedStore.unlink(store.name)
        shutil.rmtree(metrics_dir, ignore_errors=True)
    return rc
