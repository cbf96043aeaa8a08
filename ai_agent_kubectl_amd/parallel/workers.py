"""Multi-worker HTTP tier: W API worker processes on one port + the engine replicas they share.

The reference serves from one uvicorn worker (`/root/reference/app.py:400`, `Dockerfile:33`); one
worker's HTTP + JSON handling caps near 1.3k req/s on this host, below what one MI355X engine
completes, and far below 8 GPUs' worth.  `serve.py` with WORKERS > 1 runs this supervisor:

  supervisor (no GPU use)
   ├─ shared-memory segment: response cache + rate-limit windows (shared_state.py), so
   │  `from_cache` (app.py:312-322) and 429 (app.py:298,368) stay global across workers
   ├─ DP engine replicas, one process per device, each serving all W workers (dp.spawn_replicas)
   └─ W API workers: each binds HOST:PORT with SO_REUSEPORT (the kernel spreads connections),
      runs the full app (auth, validation, limiter, cache, Prometheus) under uvicorn and routes
      its misses to the least-loaded replica.  /metrics aggregates every worker
      (prometheus_client multiprocess mode: PROMETHEUS_MULTIPROC_DIR).

The supervisor restarts nothing; a dead worker is logged and the rest keep serving (the kernel
stops routing to a closed SO_REUSEPORT socket).  SIGTERM / SIGINT stop everything and remove the
shared-memory segment and the metrics directory.
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


def bind_reuseport(host: str, port: int) -> socket.socket:
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(fam, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    s.set_inheritable(True)
    return s


def _api_worker(idx: int, settings_dict: dict, host: str, port: int, endpoints, metrics_dir: str) -> None:
    """One API worker process (spawned): the app + uvicorn on a SO_REUSEPORT socket."""
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
        backend = DPRouterLLM(settings, len(endpoints.senders), endpoints=endpoints)
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
    from .dp import engine_devices, spawn_replicas

    W = max(1, int(settings.WORKERS))
    name = settings.SHARED_STATE or "/ka_state_%d" % os.getpid()
    store = SharedStore(name, settings.CACHE_MAXSIZE)   # created before any worker attaches
    metrics_dir = tempfile.mkdtemp(prefix="ka_prom_")
    sd = dataclasses.asdict(settings)
    sd["SHARED_STATE"] = store.name
    endpoints = [None] * W
    replicas = []
    if settings.LLM_BACKEND.lower() == "engine":
        if settings.TP > 1:
            raise SystemExit("WORKERS > 1 serves DP replicas (TP = 1); run TP > 1 with one API worker")
        devices = engine_devices(settings, max(1, settings.DP))
        replicas, endpoints = spawn_replicas(settings, devices, W)
        log.info("DP replicas on %s serving %d API workers", ",".join(devices), W)
    ctx = mp.get_context("spawn")
    workers = [ctx.Process(target=_api_worker, args=(i, sd, host, port, endpoints[i], metrics_dir), daemon=False)
               for i in range(W)]
    for p in workers:
        p.start()
    log.info("Started %d API workers on %s:%d (shared state %s)", W, host, port, store.name)

    stop = {"flag": False}

    def _stop(signum, frame):
        stop["flag"] = True

    signal.signal(signal.SIGTERM, _stop)
    signal.signal(signal.SIGINT, _stop)
    rc = 0
    try:
        while not stop["flag"]:
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
        for p in replicas:
            p.join(timeout=10)   # replicas exit once every worker has disconnected
            if p.is_alive():
                p.terminate()
        SharedStore.unlink(store.name)
        shutil.rmtree(metrics_dir, ignore_errors=True)
    return rc
