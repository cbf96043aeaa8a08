"""Headline benchmark: requests/sec + p50 end-to-end latency of POST /kubectl-command backed by
Llama-3-8B (bf16, random-init weights, synthetic queries) on N MI355X GPUs (BASELINE.json metric).

One process per GPU (torchrun); every rank is a data-parallel replica: this process runs the full
ASGI app (auth, limiter, cache, Prometheus middleware, JSON) and the load generator, the engine runs
in its own process on the rank's GPU (`--in-process` keeps it in this one).  Load is a closed loop
of `--concurrency` clients per GPU, each sending its next distinct cache-miss query as soon as the
previous reply arrives (BASELINE.md's concurrency-N method).  A "step" is C completed requests: W
warm-up steps, then barrier + device sync, exactly K*C timed completions, sync + barrier; the job
value is total timed requests / max-over-ranks elapsed (weak scaling: per-GPU work is fixed).
`--waves` runs lock-step waves instead (C requests start together; the next wave after the last).

  python bench.py                                   # 1 GPU, defaults
  torchrun --nproc-per-node 8 bench.py --gpus 8     # driver form
"""
import argparse
import asyncio
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "requests/sec + p50 e2e latency, /kubectl-command Llama-3-8B 1/2/4/8 GPU"
# reference app.py, cache-miss /kubectl-command at concurrency 32 = 354 req/s
# (plumbing floor with an instant stub LLM; the reference publishes no OpenAI-backed number).
BASELINE_RPS = 354.0

VERBS = ["list", "show", "get", "display", "find"]
RES = ["pods", "services", "deployments", "nodes", "configmaps", "secrets", "jobs", "ingresses", "events",
       "statefulsets", "daemonsets", "replicasets", "namespaces", "cronjobs", "endpoints"]
MODS = ["in namespace", "with label app", "sorted by age in", "that are failing in", "running in cluster"]


def make_query(rank, step, i):
    """Distinct natural-language query; the unique part comes first (request index before step
    and rank) so that requests share only the instruction template's full KV blocks — the
    computed token count per request is then independent of arrival timing and process mode."""
    v = VERBS[(step + i) % len(VERBS)]
    r = RES[(i * 7 + step) % len(RES)]
    m = MODS[(i + rank) % len(MODS)]
    return f"{i}.{step}.{rank} team: {v} all {r} {m} prod"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--concurrency", type=int, default=int(os.environ.get("BENCH_CONCURRENCY", 256)))
    ap.add_argument("--model", default=os.environ.get("BENCH_MODEL", "llama3-8b"))
    ap.add_argument("--max-new-tokens", type=int, default=16)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--in-process", action="store_true",
                    help="run the engine in this process (default: its own process on the same GPU)")
    ap.add_argument("--ramp-s", type=float, default=float(os.environ.get("BENCH_RAMP_S", 0.0)),
                    help="closed loop: client start times spread uniformly over this many seconds")
    ap.add_argument("--waves", action="store_true",
                    help="lock-step waves (all C requests start together, the next wave after the "
                         "slowest) instead of the default closed loop of C clients")
    ap.add_argument("--client", choices=["asgi", "httpx"], default="asgi",
                    help="asgi: minimal in-process ASGI client (default); httpx: httpx.ASGITransport")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    C = args.concurrency
    buckets = tuple(b for b in (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 160, 192, 256, 320, 384, 448, 512)
                    if b <= max(C, 1))
    if C not in buckets:
        buckets = tuple(sorted(set(buckets) | {C}))

    from ai_agent_kubectl_amd.api import create_app
    from ai_agent_kubectl_amd.config import Settings

    settings = Settings(RATE_LIMIT="100000000/minute", CACHE_MAXSIZE=100, LLM_TIMEOUT=600, LOG_LEVEL="WARNING",
                        LLM_BACKEND="engine", MODEL=args.model, MAX_BATCH=max(C, 1), MAX_NEW_TOKENS=args.max_new_tokens,
                        IGNORE_EOS=True, MAX_NUM_BATCHED_TOKENS=16384,
                        HIPGRAPH_BUCKETS=",".join(str(b) for b in buckets))
    os.environ.setdefault("KV_CACHE_TOKENS", str(max(65536, C * 256)))
    os.environ.setdefault("MAX_MODEL_LEN", "512")
    t_build = time.perf_counter()
    if not args.in_process:
        # Engine in its own process on cuda:LOCAL_RANK (spawned before this process touches the
        # GPU); this process runs the ASGI app + load generator, so HTTP handling and the GPU loop
        # never share a GIL.  Barriers use gloo; the device sync runs inside the engine process.
        from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM
        backend = DPRouterLLM(settings, 1, devices=[os.environ.get("BENCH_DEVICE", f"cuda:{local}")])
        if world > 1:
            dist.init_process_group("gloo")
        backend.wait_ready()
        if not any(r.up for r in backend.replicas):
            raise RuntimeError("engine process failed to start")
        eng = None
        cap_s = 0.0
    else:
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)
        from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
        from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
        opts = EngineOptions(model=args.model, device=str(dev), max_batch=max(C, 1), graph_buckets=buckets,
                             kv_cache_tokens=max(65536, C * 256), max_model_len=512,
                             use_graphs=not args.no_graphs, ignore_eos=True, max_batched_tokens=16384)
        eng = build_engine(opts)
        cap_s = eng.runner.capture_graphs()
        backend = EngineLLM(eng, max_new_tokens=args.max_new_tokens, ignore_eos=True)
    t_build = time.perf_counter() - t_build
    import logging
    logging.getLogger("app").setLevel(logging.WARNING)
    app = create_app(settings, backend=backend)
    import httpx

    lat = []
    headers = [(b"host", b"bench"), (b"content-type", b"application/json")]

    async def asgi_post(path, body: bytes):
        """Minimal in-process ASGI client: one HTTP/1.1 request through the full app stack
        (Prometheus + rate-limit middleware, routing, auth dep, validation, handler, JSON)."""
        scope = {"type": "http", "asgi": {"version": "3.0"}, "http_version": "1.1", "method": "POST",
                 "scheme": "http", "path": path, "raw_path": path.encode(), "query_string": b"",
                 "root_path": "", "headers": headers + [(b"content-length", str(len(body)).encode())],
                 "client": ("127.0.0.1", 40000), "server": ("bench", 80)}
        done = [False]

        async def receive():
            if not done[0]:
                done[0] = True
                return {"type": "http.request", "body": body, "more_body": False}
            await asyncio.sleep(3600)
            return {"type": "http.disconnect"}

        out = {"status": 0, "body": []}

        async def send(msg):
            if msg["type"] == "http.response.start":
                out["status"] = msg["status"]
            elif msg["type"] == "http.response.body":
                out["body"].append(msg.get("body", b""))

        await app(scope, receive, send)
        return out["status"], b"".join(out["body"])

    async def one(client, q, record):
        """One request; returns the reply (raw JSON bytes on the ASGI path, parsed on demand by
        `command_of`).  The load generator shares this process's CPU with the service, so the
        client side stays lean: the reply is checked on its bytes (200, a generated command,
        from_cache false; the app emits compact JSON) instead of being parsed per request."""
        t0 = time.perf_counter()
        if client is None:
            status, raw = await asgi_post("/kubectl-command", b'{"query":' + json.dumps(q).encode() + b"}")
            ok = status == 200 and raw.startswith(b'{"kubectl_command":"kubectl ') and b'"from_cache":false' in raw
            body = raw
        else:
            r = await client.post("/kubectl-command", json={"query": q})
            status, body = r.status_code, r.json()
            ok = status == 200 and body["from_cache"] is False
        dt = time.perf_counter() - t0
        if not ok:
            raise RuntimeError(f"{status}: {body}")
        if record:
            lat.append(dt)
        return body

    def command_of(reply):
        return json.loads(reply)["kubectl_command"] if isinstance(reply, bytes) else reply["kubectl_command"]

    async def wave(client, step, record):
        return await asyncio.gather(*[one(client, make_query(rank, step, i), record) for i in range(C)])

    async def sync_all():
        """barrier + device synchronize: every engine's queued GPU work is complete"""
        if eng is None:
            st = (await backend.control("sync"))[0]
        else:
            torch.cuda.synchronize()
            st = dict(eng.runner.stats, prefix_hits=eng.bm.hits, prefix_queries=eng.bm.queries,
                      partial_tokens=getattr(eng.bm, "partial_tokens", 0), chained_steps=eng.chained_steps,
                      engine_idle_s=eng.idle_s)
        if world > 1:
            dist.barrier()
        return st

    async def sync_barrier():
        """device sync + cross-rank barrier, run off the event loop so in-flight load keeps moving"""
        loop = asyncio.get_running_loop()
        if eng is None:
            st = (await backend.control("sync"))[0]
        else:
            await loop.run_in_executor(None, torch.cuda.synchronize)
            st = dict(eng.runner.stats, prefix_hits=eng.bm.hits, prefix_queries=eng.bm.queries,
                      partial_tokens=getattr(eng.bm, "partial_tokens", 0), chained_steps=eng.chained_steps,
                      engine_idle_s=eng.idle_s)
        if world > 1:
            await loop.run_in_executor(None, dist.barrier)
        return st

    async def closed_loop(client):
        """C concurrent clients, each sending its next request as soon as the previous reply
        arrives (the closed-loop method BASELINE.md's concurrency-32 rows use).  W*C completions
        warm up; then barrier + device sync, exactly K*C completions are timed, sync + barrier."""
        import random
        state = {"done": 0, "target": args.warmup * C, "record": False, "stop": False}
        reached = asyncio.Event()
        sample = []

        async def worker(i):
            await asyncio.sleep(random.Random(i).uniform(0, args.ramp_s))   # de-phase the first arrivals
            n = 0
            while not state["stop"]:
                t_start = time.perf_counter()
                cmd = await one(client, make_query(rank, n, i), False)
                n += 1
                if state["stop"]:
                    break
                if not sample:
                    sample.append(cmd)
                state["done"] += 1
                if state["record"]:
                    lat.append(time.perf_counter() - t_start)
                if state["done"] >= state["target"] and not reached.is_set():
                    reached.set()

        tasks = [asyncio.ensure_future(worker(i)) for i in range(C)]
        if state["target"] > 0:
            await reached.wait()
        st0 = await sync_barrier()
        reached.clear()
        state.update(done=0, target=args.steps * C, record=True)
        t0 = time.perf_counter()
        await reached.wait()
        state["record"] = False
        st1 = await sync_barrier()
        el = time.perf_counter() - t0
        state["stop"] = True
        await asyncio.gather(*tasks)
        return el, sample, st0, st1

    async def waves(client):
        sample = None
        for s in range(args.warmup):
            sample = await wave(client, s, False)
        st0 = await sync_all()
        t0 = time.perf_counter()
        for s in range(args.steps):
            await wave(client, args.warmup + s, True)
        st1 = await sync_all()
        return time.perf_counter() - t0, sample, st0, st1

    async def run():
        await backend.start()
        limits = httpx.Limits(max_connections=None, max_keepalive_connections=None)
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://bench",
                                     limits=limits, timeout=600) as hc:
            client = hc if args.client == "httpx" else None
            el, sample, st0, st1 = await (waves(client) if args.waves else closed_loop(client))
        await backend.close()
        return el, sample, {k: st1[k] - st0[k] for k in st1 if isinstance(st1[k], (int, float))}

    if os.environ.get("KA_PROFILE_API"):
        import cProfile
        import pstats
        prof = cProfile.Profile()
        prof.enable()
        elapsed, sample, st = asyncio.run(run())
        prof.disable()
        with open(os.environ["KA_PROFILE_API"], "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(50)
    else:
        elapsed, sample, st = asyncio.run(run())
    n_req = C * args.steps
    p50 = statistics.median(lat) * 1e3
    if world > 1:
        t = torch.tensor([elapsed, p50], dtype=torch.float64,
                         device="cpu" if eng is None else torch.device(f"cuda:{local}"))
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        elapsed = max(g[0].item() for g in gathered)
        p50 = statistics.median([g[1].item() for g in gathered])
    value = n_req * world / elapsed
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "req/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": round(value / BASELINE_RPS, 3),
            "dtype": "bf16", "data": "synthetic queries, random-init weights",
            "config": {"model": "Llama-3-8B-Instruct" if args.model == "llama3-8b" else args.model,
                       "global_batch": C * world, "seq_len": len(backend.prompt_ids(make_query(0, 0, 0))) +
                       args.max_new_tokens, "parallelism": f"dp{world}"},
            "p50_ms": round(p50, 2),
            "detail": {"concurrency_per_gpu": C, "new_tokens": args.max_new_tokens,
                       "load": "waves" if args.waves else "closed-loop",
                       "p99_ms": round(sorted(lat)[int(0.99 * (len(lat) - 1))] * 1e3, 2) if lat else None,
                       "decode_steps": st.get("decode_steps"), "prefill_steps": st.get("prefill_steps"),
                       "decode_ms_per_step": round(st["decode_ms"] / max(1, st["decode_steps"]), 3),
                       "prefill_ms_per_step": round(st["prefill_ms"] / max(1, st["prefill_steps"]), 3),
                       "prefill_tokens": st.get("prefill_tokens"), "graph_replays": st.get("graph_replays"),
                       "prefix_cache_hit_rate": round(st.get("prefix_hits", 0) / max(1, st.get("prefix_queries", 0)), 3),
                       "sub_block_reused_tokens": st.get("partial_tokens", 0),
                       "overlapped_decode_steps": st.get("chained_steps", 0),
                       "engine_idle_ms_per_step": round(st.get("engine_idle_s", 0.0) * 1e3 / args.steps, 2),
                       "build_s": round(t_build, 1), "engine_process": eng is None,
                       "sample_reply": command_of(sample[0]) if sample else None,
                       "baseline": "BASELINE.md reference plumbing floor, cache-miss conc 32 = 354 req/s"},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
