"""Service entry point (replaces `python app.py` / `uvicorn app:app`, `/root/reference/app.py:392-400`).

    python -m ai_agent_kubectl_amd.serve                       # stub or single-GPU engine
    LLM_BACKEND=engine DP=8 python -m ai_agent_kubectl_amd.serve          # 8 replicas, 1 API process
    LLM_BACKEND=engine DP=8 WORKERS=8 python -m ai_agent_kubectl_amd.serve   # 8 replicas, 8 API workers
                                                               # (shared cache + limiter, parallel/workers.py)
    LLM_BACKEND=engine DP=4 TP=2 WORKERS=4 python -m ai_agent_kubectl_amd.serve   # 4 replicas of 2 GPUs each
    LLM_BACKEND=engine TP=8 MODEL=llama3-70b python -m ai_agent_kubectl_amd.serve          # one TP=8 replica
    LLM_BACKEND=engine TP=8 MODEL=llama3-70b torchrun --nproc-per-node 8 -m ai_agent_kubectl_amd.serve

Settings come from the environment and `./.env` (same variables and defaults as the reference, plus
the engine flags of SURVEY.md §5.6).  Engine replicas (parallel/dp.py) are TP groups: the replica
process is TP rank 0 and spawns the other ranks.  Under torchrun (WORLD_SIZE = TP > 1) this process
is rank 0 itself: it runs the API + scheduler and every other rank mirrors its steps in
`ModelRunner.worker_loop()` (RCCL collectives inside each forward).
HOST/PORT are honoured (the reference's Dockerfile ignored them, quirk Q10).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys


def main(argv=None) -> int:
    from .config import Settings

    settings = Settings.from_env()
    # a serving process exits after an unrecoverable engine fault so that its supervisor (docker's
    # restart policy, torchrun, the DP supervisor) restarts it (engine/engine.py)
    os.environ.setdefault("KA_EXIT_ON_FATAL", "1")
    ap = argparse.ArgumentParser(description="MI355X kubectl agent service")
    ap.add_argument("--host", default=settings.HOST)
    ap.add_argument("--port", type=int, default=settings.PORT)
    args = ap.parse_args(argv)
    logging.basicConfig(level=settings.log_level, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    log = logging.getLogger("app")

    if settings.LLM_BACKEND == "engine" and settings.TP > 1 and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from .engine.builder import EngineOptions, build_engine
        from .parallel.launch import init_tp

        comm, rank = init_tp(settings.TP)
        if rank != 0:
            opts = EngineOptions.from_settings(settings)
            opts.tp_rank = rank
            if opts.device.startswith("cuda"):
                opts.device = f"cuda:{os.environ.get('LOCAL_RANK', rank)}"
            eng = build_engine(opts, comm=comm)
            eng.runner.capture_graphs()
            eng.runner.worker_loop()
            return 0

    if settings.WORKERS > 1:
        from .parallel.workers import run_workers
        return run_workers(settings, args.host, args.port)

    import uvicorn

    from .api import create_app

    app = create_app(settings)
    log.info(f"Starting Uvicorn server on {args.host}:{args.port}")
    # keep-alive longer than common client/LB pools so idle pooled connections are not reset
    # under the client's feet (uvicorn's default is 5 s)
    uvicorn.run(app, host=args.host, port=args.port, reload=False, log_level=settings.LOG_LEVEL.lower(),
                workers=1, timeout_keep_alive=int(os.environ.get("KEEP_ALIVE_S", "75")))
    return 0


if __name__ == "__main__":
    sys.exit(main())
