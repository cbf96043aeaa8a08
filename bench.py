"""Headline benchmark: requests/sec + p50 end-to-end latency of POST /kubectl-command backed by
Llama-3-8B (bf16, random-init weights, synthetic queries) on N MI355X GPUs (BASELINE.json metric).

One process per GPU (torchrun); every rank is a data-parallel replica with its own engine process
on its GPU.  A "step" is C completed requests: W warm-up steps, then barrier + device sync,
exactly K*C timed completions, sync + barrier; the job value is total timed requests / max-over-
ranks elapsed (weak scaling: per-GPU work is fixed).

Transports (`--transport`):
  tcp   the production topology over real sockets: ONE `python -m ai_agent_kubectl_amd.serve` with
        DP = N engine replicas (one process per GPU) behind `--api-workers` x N uvicorn workers on
        one port (SO_REUSEPORT, one shared cache + limiter, parallel/workers.py), and
        `--client-procs` load-generator processes per rank speaking HTTP/1.1 keep-alive.  This is
        what the reference's 354 req/s plumbing floor (uvicorn over TCP) measures, so
        the headline `value` and `vs_baseline` come from it.
  asgi  the full ASGI app (Prometheus + rate-limit middleware, routing, auth, validation, cache,
        JSON) driven in-process by a minimal ASGI client — no sockets; the engine runs in its own
        process on the rank's GPU (one app + engine per rank).
  both  (default) tcp for the headline, then asgi, then asgi with the prefix cache off; the last two
        are reported in `detail.asgi` / `detail.prefix_cache_off`.

Load (`--load`): `closed` (default) C clients per GPU, each sending its next distinct cache-miss
query as soon as the previous reply arrives (BASELINE.md's concurrency-N method); `open` Poisson
arrivals at `--rate` req/s per GPU (latency under an arrival rate instead of a fixed population).
`--mix` runs BASELINE config #5 instead of pure misses: cache hits, concurrent /execute calls
(fake kubectl on PATH), and /metrics scrapes, with per-class counts and p50s in `detail`.

  python bench.py                                   # 1 GPU, defaults (driver form)
  python bench.py --gpus 8                          # spawns 8 ranks itself (torch.distributed.run)
  torchrun --nproc-per-node 8 bench.py --gpus 8     # driver form for N > 1
  python bench.py --transport asgi                  # in-process transport only
  python bench.py --gpus 8 --tp 8 --model llama3-70b --concurrency 8   # config #3: one TP=8 replica
  python bench.py --gpus 8 --tp 8 --model mixtral-8x7b                 # config #4: EP=8 (experts over TP)
"""
import argparse
import asyncio
import json
import os
import random
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "requests/sec + p50 e2e latency, /kubectl-command Llama-3-8B 1/2/4/8 GPU"
# reference app.py, cache-miss /kubectl-command at concurrency 32 = 354 req/s
# (plumbing floor with an instant stub LLM over TCP; the reference publishes no OpenAI-backed number).
BASELINE_RPS = 354.0
MODEL_NAMES = {"llama3-8b": "Llama-3-8B-Instruct", "llama3-70b": "Llama-3-70B-Instruct",
               "mixtral-8x7b": "Mixtral-8x7B-Instruct"}

VERBS = ["list", "show", "get", "display", "find"]
RES = ["pods", "services", "deployments", "nodes", "configmaps", "secrets", "jobs", "ingresses", "events",
       "statefulsets", "daemonsets", "replicasets", "namespaces", "cronjobs", "endpoints"]
MODS = ["in namespace", "with label app", "sorted by age in", "that are failing in", "running in cluster"]
FAKE_KUBECTL = "#!/bin/sh\nprintf 'NAME      READY   STATUS    RESTARTS   AGE\\nnginx-1   1/1     Running   0          5m\\n'\n"


def make_query(rank, step, i):
    """Distinct natural-language query; the unique part comes first (request index before step
    and rank) so that requests share only the instruction template's full KV blocks — the
    computed token count per request is then independent of arrival timing and process mode."""
    v = VERBS[(step + i) % len(VERBS)]
    r = RES[(i * 7 + step) % len(RES)]
    m = MODS[(i + rank) % len(MODS)]
    return f"{i}.{step}.{rank} team: {v} all {r} {m} prod"


def hot_query(rank, j):
    return f"hot {j}.{rank}: list all {RES[j % len(RES)]} in namespace prod"


def cache_size(args):
    """The reference default (100) for the miss-only headline; with --mix the cache holds the
    working set (the hit class re-asks 32 hot queries while misses keep inserting)."""
    return 50000 if args.mix else 100


def prompt_len(model: str) -> int:
    """Prompt tokens of a bench query (CPU only: tokenizer + chat template, as the engine sees it)."""
    from ai_agent_kubectl_amd.engine.tokenizer import get_tokenizer
    from ai_agent_kubectl_amd.models.config import get_config
    from ai_agent_kubectl_amd.prompt import PROMPT_PREFIX, PROMPT_SUFFIX
    cfg = get_config(model)
    tok = get_tokenizer(cfg.vocab_size, cfg.tokenizer, None)
    before, after = tok.chat_prefix_suffix()
    return len(before + tok.encode(PROMPT_PREFIX) + tok.encode(make_query(0, 0, 0) + PROMPT_SUFFIX) + after)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--concurrency", type=int, default=int(os.environ.get("BENCH_CONCURRENCY", 256)))
    ap.add_argument("--model", default=os.environ.get("BENCH_MODEL", "llama3-8b"))
    ap.add_argument("--max-new-tokens", type=int, default=16)
    ap.add_argument("--max-batched-tokens", type=int,
                    default=int(os.environ.get("BENCH_MAX_BATCHED_TOKENS", 0)),
                    help="engine token budget per step (prefill chunks + decode rows); 0: the model's default")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--in-process", action="store_true",
                    help="asgi transport: run the engine in this process (default: its own process on the GPU)")
    ap.add_argument("--transport", choices=["asgi", "tcp", "both"], default=os.environ.get("BENCH_TRANSPORT", "both"))
    ap.add_argument("--api-workers", type=int, default=int(os.environ.get("BENCH_API_WORKERS", 2)),
                    help="tcp: uvicorn API worker processes sharing the port, per GPU")
    ap.add_argument("--no-prefix-off-pass", action="store_true",
                    help="both: skip the asgi pass with the prefix cache off")
    ap.add_argument("--client-procs", type=int, default=int(os.environ.get("BENCH_CLIENT_PROCS", 2)),
                    help="tcp: load-generator processes")
    ap.add_argument("--load", choices=["closed", "open"], default="closed")
    ap.add_argument("--rate", type=float, default=0.0, help="open loop: arrivals per second per GPU")
    ap.add_argument("--mix", action="store_true", help="BASELINE config #5: hits + misses + /execute + scrapes")
    ap.add_argument("--hit-frac", type=float, default=0.5)
    ap.add_argument("--exec-frac", type=float, default=0.1)
    ap.add_argument("--ramp-s", type=float, default=float(os.environ.get("BENCH_RAMP_S", 0.0)),
                    help="closed loop: client start times spread uniformly over this many seconds")
    ap.add_argument("--variable-len", action="store_true",
                    help="EOS-terminated replies (IGNORE_EOS=0) instead of exactly --max-new-tokens")
    ap.add_argument("--tp", type=int, default=int(os.environ.get("BENCH_TP", 1)),
                    help="tensor-parallel degree of each engine replica (BASELINE configs #3 / #4: "
                         "--model llama3-70b --tp 8, --model mixtral-8x7b --tp 8 = EP 8); the server runs "
                         "DP = gpus / tp replicas, each a TP group of consecutive GPUs (tcp transport)")
    args = ap.parse_args(argv)
    if args.tp < 1 or args.gpus % args.tp:
        ap.error(f"--tp {args.tp} must divide --gpus {args.gpus}")
    if args.tp > 1 and args.transport != "tcp":
        # a TP group spans several ranks' GPUs: only the one-server tcp topology (serve.py with
        # DP x TP) places it; the per-rank in-process asgi transport has one GPU per rank
        args.transport = "tcp"
    return args


def parallelism(args, world: int) -> str:
    """config.parallelism: dp{N} (one replica per GPU), dp{d}tp{t} for tensor-parallel replicas, or
    dp{d}ep{t} for a MoE model (experts sharded over the tensor-parallel group: EP = TP)."""
    if args.tp == 1:
        return f"dp{world}"
    from ai_agent_kubectl_amd.models.config import get_config
    kind = "ep" if get_config(args.model).is_moe else "tp"
    return f"dp{world // args.tp}{kind}{args.tp}"


# ---------------------------------------------------------------------------------------------
# request classes for --mix (one draw per request)
def pick_kind(rng, args):
    if not args.mix:
        return "miss"
    x = rng.random()
    if x < args.exec_frac:
        return "exec"
    if x < args.exec_frac + args.hit_frac:
        return "hit"
    return "miss"


def body_for(kind, rank, n, i, rng):
    if kind == "exec":
        return "/execute", b'{"execute":"kubectl get pods -n prod"}'
    q = hot_query(rank, rng.randrange(32)) if kind == "hit" else make_query(rank, n, i)
    return "/kubectl-command", b'{"query":' + json.dumps(q).encode() + b"}"


def reply_ok(kind, status, raw):
    if kind == "exec":
        return status == 200 and raw.startswith(b'{"kubectl_command":"kubectl get pods')
    if status != 200 or not raw.startswith(b'{"kubectl_command":"kubectl '):
        return False
    return (b'"from_cache":true' in raw) if kind == "hit" else (b'"from_cache":false' in raw)


# ---------------------------------------------------------------------------------------------
# HTTP/1.1 keep-alive client (tcp transport)
class HttpConn:
    def __init__(self, host, port):
        self.host, self.port = host, port
        self.r = self.w = None

    async def open(self):
        self.r, self.w = await asyncio.open_connection(self.host, self.port)
        sock = self.w.get_extra_info("socket")
        if sock is not None:
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    async def request(self, method, path, body=b""):
        if self.w is None:
            await self.open()
        head = b"%s %s HTTP/1.1\r\nhost: bench\r\ncontent-type: application/json\r\ncontent-length: %d\r\n\r\n" % (
            method.encode(), path.encode(), len(body))
        self.w.write(head + body)
        hdr = await self.r.readuntil(b"\r\n\r\n")
        status = int(hdr[9:12])
        low = hdr.lower()
        i = low.find(b"content-length:")
        n = int(low[i + 15:low.index(b"\r\n", i)]) if i >= 0 else 0
        return status, await self.r.readexactly(n)

    def close(self):
        if self.w is not None:
            self.w.close()


def _client_proc(cid, nproc, args, rank, port, C, shared, out_q):
    """One load-generator process of the tcp transport: C/nproc closed-loop connections (or its
    share of the open-loop arrival rate).  `shared`: phase (0 warm-up, 1 record, 2 stop) and a
    completion counter the parent polls."""
    phase, done = shared

    async def run():
        rng = random.Random(1000 * rank + cid)
        lat = {"miss": [], "hit": [], "exec": []}
        errors = []

        async def one(conn, kind, path, body):
            t0 = time.perf_counter()
            status, raw = await conn.request("POST", path, body)
            if not reply_ok(kind, status, raw):
                errors.append(f"{kind} {status}: {raw[:200]!r}")
                return
            if phase.value == 1:
                lat[kind].append(time.perf_counter() - t0)
            with done.get_lock():
                done.value += 1

        if args.load == "closed":
            conns = [i for i in range(C) if i % nproc == cid]

            async def worker(i):
                await asyncio.sleep(random.Random(i).uniform(0, args.ramp_s))
                conn = HttpConn("127.0.0.1", port)
                n = 0
                while phase.value < 2 and not errors:
                    kind = pick_kind(rng, args)
                    path, body = body_for(kind, rank, n, i, rng)
                    n += 1
                    await one(conn, kind, path, body)
                conn.close()

            tasks = [asyncio.ensure_future(worker(i)) for i in conns]
        else:
            idle = []
            rate = args.rate / nproc
            tasks = []

            async def arrival(n):
                conn = idle.pop() if idle else HttpConn("127.0.0.1", port)
                kind = pick_kind(rng, args)
                path, body = body_for(kind, rank, n, cid, rng)
                await one(conn, kind, path, body)
                idle.append(conn)

            async def arrivals():
                n = 0
                t_next = time.perf_counter()
                while phase.value < 2 and not errors:
                    t_next += rng.expovariate(rate)
                    await asyncio.sleep(max(0.0, t_next - time.perf_counter()))
                    tasks.append(asyncio.ensure_future(arrival(n)))
                    n += 1

            tasks.append(asyncio.ensure_future(arrivals()))
        if args.mix and cid == 0:
            async def scraper():
                conn = HttpConn("127.0.0.1", port)
                while phase.value < 2:
                    t0 = time.perf_counter()
                    await conn.request("GET", "/metrics")
                    if phase.value == 1:
                        lat.setdefault("scrape", []).append(time.perf_counter() - t0)
                    await asyncio.sleep(1.0)
                conn.close()
            tasks.append(asyncio.ensure_future(scraper()))
        while phase.value < 2 and not errors:
            await asyncio.sleep(0.05)
        await asyncio.sleep(0.2)
        for t in tasks:
            t.cancel()
        out_q.put((cid, lat, errors[:5]))

    asyncio.run(run())


# ---------------------------------------------------------------------------------------------
def _barrier(dist):
    """A barrier that leaves the GPU alone on gloo: dist.barrier() resolves the accelerator
    (torch._C._get_accelerator) and so opens the device in every rank, though the ranks issue no
    GPU work (scripts/kfd_probe.py); on a box with a per-GPU process limit, N ranks + N replicas +
    torchrun then exceed it at N = 8.  A CPU all-reduce synchronises the same way."""
    if dist.get_backend() == "gloo":
        import torch
        dist.all_reduce(torch.zeros(1))
    else:
        dist.barrier()


def bench_devices(world):
    """Engine devices of the N replicas: cuda:0..N-1, or BENCH_DEVICE (one device for every replica,
    e.g. `cpu` for the CPU test of this path, or a comma list)."""
    dev = os.environ.get("BENCH_DEVICE", "")
    if not dev:
        return [f"cuda:{i}" for i in range(world)]
    devs = [d.strip() for d in dev.split(",") if d.strip()]
    return devs if len(devs) >= world else [devs[0]] * world


def service_env(args, C, buckets, world, port, kubectl_dir):
    """serve.py's environment: DP = world / tp replicas (each a TP group of tp consecutive GPUs, one
    process per GPU), api_workers x world API workers.  A replica serves the C clients of each of its
    tp GPUs' ranks: batch up to C x tp."""
    tp = args.tp
    rb = max(C, 1) * tp
    env = dict(os.environ, LLM_BACKEND="engine", MODEL=args.model, DP=str(world // tp), TP=str(tp),
        ENGINE_DEVICES=",".join(bench_devices(world)), WORKERS=str(args.api_workers * world), HOST="127.0.0.1",
        PORT=str(port),
        RATE_LIMIT="100000000/minute", CACHE_MAXSIZE=str(cache_size(args)), LLM_TIMEOUT="600", LOG_LEVEL="WARNING",
        MAX_BATCH=str(rb), MAX_NEW_TOKENS=str(args.max_new_tokens), IGNORE_EOS="0" if args.variable_len else "1",
        MAX_NUM_BATCHED_TOKENS=str(args.max_batched_tokens), HIPGRAPH_BUCKETS=",".join(str(b) for b in buckets),
        KV_CACHE_TOKENS=os.environ.get("KV_CACHE_TOKENS", str(max(65536, rb * 528))),
        MAX_MODEL_LEN=os.environ.get("MAX_MODEL_LEN", "512"), PYTHONPATH=ROOT,
        PATH=kubectl_dir + os.pathsep + os.environ.get("PATH", ""))
    env.pop("API_AUTH_KEY", None)
    for k in list(env):
        # the server is not a rank of this job: none of torchrun's variables may leak into it (with
        # TORCHELASTIC_USE_AGENT_STORE a TP replica's rank 0 would wait for an agent store that does
        # not exist instead of hosting its group's rendezvous)
        if k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                 "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT") or k.startswith("TORCHELASTIC_"):
            env.pop(k, None)
    if args.no_graphs:
        env["HIPGRAPH_BUCKETS"] = ""
    return env


async def scrape_engine_metrics(port):
    """Engine step / queue-wait histogram sums and counts from the server's /metrics (aggregated
    over the API workers): the TCP transport's view of the engine (llm_step_seconds{phase},
    llm_queue_wait_seconds)."""
    conn = HttpConn("127.0.0.1", port)
    try:
        st, body = await conn.request("GET", "/metrics")
    finally:
        conn.close()
    out = {}
    if st != 200:
        return out
    for line in body.decode().splitlines():
        for name, key in (('llm_step_seconds_sum{phase="decode"}', "decode_sum"),
                          ('llm_step_seconds_count{phase="decode"}', "decode_count"),
                          ('llm_step_seconds_sum{phase="prefill"}', "prefill_sum"),
                          ('llm_step_seconds_count{phase="prefill"}', "prefill_count"),
                          ("llm_queue_wait_seconds_sum", "qwait_sum"), ("llm_queue_wait_seconds_count", "qwait_count")):
            if line.startswith(name + " "):
                out[key] = out.get(key, 0.0) + float(line.rsplit(" ", 1)[1])
    return out


def cpu_snapshot(pids_by_role):
    """CPU seconds (user + system) of every process of the server tree and of the load generators,
    keyed by process name (serve.py names its processes ka-api-<i> / ka-replica-<i> / ka-tp-<i>.<r>)."""
    import psutil
    out = {}
    for role, pid in pids_by_role:
        try:
            root = psutil.Process(pid)
            procs = [root] + (root.children(recursive=True) if role == "server" else [])
        except psutil.Error:
            continue
        for p in procs:
            try:
                t = p.cpu_times()
                name = p.name() if role == "server" else f"client-{pid}"
                out[(name, p.pid)] = t.user + t.system
            except psutil.Error:
                pass
    return out


def cpu_util(s0, s1, elapsed):
    """Cores used per process over the timed region (1.0 = one core busy all the time)."""
    util = {}
    for key, v in s1.items():
        name = key[0]
        util[name] = round(util.get(name, 0.0) + (v - s0.get(key, v)) / max(elapsed, 1e-9), 3)
    return dict(sorted(util.items(), key=lambda kv: -kv[1]))


def run_tcp(args, rank, local, world, C, buckets, dist):
    """tcp transport: rank 0 starts ONE production server (DP = world replicas, shared cache and
    limiter across its API workers, one port); every rank drives C closed-loop clients at it from
    its own load-generator processes and times its own K*C completions."""
    import multiprocessing as mp

    kdir = tempfile.mkdtemp(prefix="ka_bench_bin_")
    with open(os.path.join(kdir, "kubectl"), "w") as f:
        f.write(FAKE_KUBECTL)
    os.chmod(os.path.join(kdir, "kubectl"), 0o755)
    t_build = time.perf_counter()
    srv, log, log_path = None, None, None
    if rank == 0:
        port = _free_port()
        log_path = os.path.join(tempfile.gettempdir(), f"ka_bench_serve_{os.getpid()}.log")
        log = open(log_path, "w")
        srv = subprocess.Popen([sys.executable, "-m", "ai_agent_kubectl_amd.serve"], env=service_env(
            args, C, buckets, world, port, kdir), stdout=log, stderr=subprocess.STDOUT, start_new_session=True,
            cwd=kdir)
    else:
        port = 0
    if world > 1:
        box = [port]
        dist.broadcast_object_list(box, src=0)
        port = box[0]

    async def health():
        conn = HttpConn("127.0.0.1", port)
        try:
            st, _ = await conn.request("GET", "/health")
            return st == 200
        finally:
            conn.close()

    try:
        if rank == 0:
            deadline = time.time() + 1500
            while True:
                if srv.poll() is not None:
                    raise RuntimeError("server exited: " + open(log_path).read()[-3000:])
                try:
                    if asyncio.run(health()):
                        break
                except OSError:
                    pass
                if time.time() > deadline:
                    raise RuntimeError("server did not come up")
                time.sleep(1.0)

            # the first request of each API worker waits for every engine replica (start + autotune
            # + hipGraph capture): prime every worker before timing anything
            async def prime():
                conns = [HttpConn("127.0.0.1", port) for _ in range(4 * args.api_workers * world)]
                rs = await asyncio.gather(*[c.request("POST", "/kubectl-command", b'{"query":"prime %d"}' % j)
                                            for j, c in enumerate(conns)])
                if args.mix:   # hot queries for the hit class, inserted through ONE worker: the other
                    for r in range(world):   # workers' hits prove the cache is shared
                        rs += [await conns[0].request("POST", "/kubectl-command", b'{"query":' + json.dumps(
                            hot_query(r, j)).encode() + b"}") for j in range(32)]
                for c in conns:
                    c.close()
                return rs
            rs = asyncio.run(prime())
            bad = [r for r in rs if r[0] != 200]
            if bad:
                raise RuntimeError(f"priming failed: {bad[:2]}")
        if world > 1:
            _barrier(dist)
        t_build = time.perf_counter() - t_build

        ctx = mp.get_context("spawn")
        phase, done = ctx.Value("i", 0), ctx.Value("l", 0)
        out_q = ctx.Queue()
        P = max(1, min(args.client_procs, C if args.load == "closed" else 64))
        procs = [ctx.Process(target=_client_proc, args=(c, P, args, rank, port, C, (phase, done), out_q))
                 for c in range(P)]
        for p in procs:
            p.start()
        warm_target = args.warmup * C
        while done.value < warm_target:
            time.sleep(0.005)
        if world > 1:
            _barrier(dist)
        m0 = asyncio.run(scrape_engine_metrics(port)) if rank == 0 else {}
        roles = ([("server", srv.pid)] if srv is not None else []) + [("client", p.pid) for p in procs]
        c0 = cpu_snapshot(roles)
        with done.get_lock():
            done.value = 0
        phase.value = 1
        t0 = time.perf_counter()
        target = args.steps * C
        while done.value < target:
            time.sleep(0.001)
        elapsed = time.perf_counter() - t0
        c1 = cpu_snapshot(roles)
        phase.value = 2
        m1 = asyncio.run(scrape_engine_metrics(port)) if rank == 0 else {}
        if world > 1:
            _barrier(dist)
        lat = {}
        errors = []
        for _ in procs:
            _, l, e = out_q.get(timeout=120)
            errors += e
            for k, v in l.items():
                lat.setdefault(k, []).extend(v)
        for p in procs:
            p.join(timeout=30)
        if world > 1:
            _barrier(dist)   # every rank's clients are done before rank 0 stops the server
        if errors:
            raise RuntimeError("bad replies: %s" % errors[:3])
        d = {k: m1.get(k, 0.0) - m0.get(k, 0.0) for k in m1}
        st = {"decode_steps": int(d.get("decode_count", 0)), "decode_ms": d.get("decode_sum", 0.0) * 1e3,
              "prefill_steps": int(d.get("prefill_count", 0)), "prefill_ms": d.get("prefill_sum", 0.0) * 1e3,
              "queue_wait_ms_mean": round(d.get("qwait_sum", 0.0) * 1e3 / max(1.0, d.get("qwait_count", 0.0)), 2),
              "cpu_cores": cpu_util(c0, c1, elapsed)}
        return elapsed, lat, st, t_build, None
    finally:
        if srv is not None:
            if srv.poll() is None:
                os.killpg(srv.pid, 15)
                try:
                    srv.wait(60)
                except subprocess.TimeoutExpired:
                    os.killpg(srv.pid, 9)
            log.close()


def run_asgi(args, rank, local, world, C, buckets, dist, prefix_caching=True):
    """asgi transport: the full app in this process, driven by a minimal in-process ASGI client."""
    import torch

    from ai_agent_kubectl_amd.api import create_app
    from ai_agent_kubectl_amd.config import Settings

    kdir = tempfile.mkdtemp(prefix="ka_bench_bin_")
    with open(os.path.join(kdir, "kubectl"), "w") as f:
        f.write(FAKE_KUBECTL)
    os.chmod(os.path.join(kdir, "kubectl"), 0o755)
    os.environ["PATH"] = kdir + os.pathsep + os.environ.get("PATH", "")
    settings = Settings(RATE_LIMIT="100000000/minute", CACHE_MAXSIZE=cache_size(args), LLM_TIMEOUT=600,
                        LOG_LEVEL="WARNING",
                        LLM_BACKEND="engine", MODEL=args.model, MAX_BATCH=max(C, 1), MAX_NEW_TOKENS=args.max_new_tokens,
                        IGNORE_EOS=not args.variable_len, MAX_NUM_BATCHED_TOKENS=args.max_batched_tokens,
                        HIPGRAPH_BUCKETS=",".join(str(b) for b in buckets), PREFIX_CACHING=prefix_caching)
    os.environ.setdefault("KV_CACHE_TOKENS", str(max(65536, C * 528)))
    os.environ.setdefault("MAX_MODEL_LEN", "512")
    t_build = time.perf_counter()
    if not args.in_process:
        # engine in its own process on cuda:LOCAL_RANK (spawned before this process touches the
        # GPU); this process runs the ASGI app + load generator, so HTTP handling and the GPU loop
        # never share a GIL.  Barriers use gloo; the device sync runs inside the engine process.
        from ai_agent_kubectl_amd.parallel.dp import DPRouterLLM
        backend = DPRouterLLM(settings, 1, devices=[bench_devices(world)[local]])
        if world > 1 and not dist.is_initialized():
            dist.init_process_group("gloo")
        backend.wait_ready()
        if not any(r.up for r in backend.replicas):
            raise RuntimeError("engine process failed to start")
        eng = None
    else:
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
        if world > 1 and not dist.is_initialized():
            dist.init_process_group("nccl", device_id=dev)
        from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
        from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
        opts = EngineOptions(model=args.model, device=str(dev), max_batch=max(C, 1), graph_buckets=buckets,
                             kv_cache_tokens=max(65536, C * 528), max_model_len=512, prefix_caching=prefix_caching,
                             use_graphs=not args.no_graphs, ignore_eos=not args.variable_len, max_batched_tokens=args.max_batched_tokens)
        eng = build_engine(opts)
        eng.runner.capture_graphs()
        backend = EngineLLM(eng, max_new_tokens=args.max_new_tokens, ignore_eos=not args.variable_len)
    t_build = time.perf_counter() - t_build
    import logging
    logging.getLogger("app").setLevel(logging.WARNING)
    app = create_app(settings, backend=backend)
    lat = {"miss": [], "hit": [], "exec": []}
    headers = [(b"host", b"bench"), (b"content-type", b"application/json")]

    async def asgi_call(method, path, body: bytes):
        """Minimal in-process ASGI client: one HTTP/1.1 request through the full app stack
        (Prometheus + rate-limit middleware, routing, auth dep, validation, handler, JSON)."""
        scope = {"type": "http", "asgi": {"version": "3.0"}, "http_version": "1.1", "method": method,
                 "scheme": "http", "path": path, "raw_path": path.encode(), "query_string": b"",
                 "root_path": "", "headers": headers + [(b"content-length", str(len(body)).encode())],
                 "client": ("127.0.0.1", 40000), "server": ("bench", 80)}
        sent = [False]

        async def receive():
            if not sent[0]:
                sent[0] = True
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
            await loop.run_in_executor(None, _barrier, dist)
        return st

    async def run():
        await backend.start()
        if args.mix:
            for j in range(32):
                st, raw = await asgi_call("POST", "/kubectl-command", b'{"query":' + json.dumps(
                    hot_query(rank, j)).encode() + b"}")
                assert st == 200, raw
        state = {"done": 0, "target": args.warmup * C, "record": False, "stop": False}
        reached = asyncio.Event()
        sample = []
        errors = []
        rng = random.Random(rank)

        async def one(kind, path, body):
            t_start = time.perf_counter()
            status, raw = await asgi_call("POST", path, body)
            if not reply_ok(kind, status, raw):
                errors.append(f"{kind} {status}: {raw[:200]!r}")
                reached.set()
                return
            if not sample and kind == "miss":
                sample.append(raw)
            state["done"] += 1
            if state["record"]:
                lat[kind].append(time.perf_counter() - t_start)
            if state["done"] >= state["target"] and not reached.is_set():
                reached.set()

        tasks = []
        if args.load == "closed":
            async def worker(i):
                await asyncio.sleep(random.Random(i).uniform(0, args.ramp_s))   # de-phase the first arrivals
                n = 0
                while not state["stop"] and not errors:
                    kind = pick_kind(rng, args)
                    path, body = body_for(kind, rank, n, i, rng)
                    n += 1
                    await one(kind, path, body)
            tasks = [asyncio.ensure_future(worker(i)) for i in range(C)]
        else:
            async def arrivals():
                n = 0
                t_next = time.perf_counter()
                while not state["stop"] and not errors:
                    t_next += rng.expovariate(args.rate)
                    await asyncio.sleep(max(0.0, t_next - time.perf_counter()))
                    kind = pick_kind(rng, args)
                    path, body = body_for(kind, rank, n, n % 997, rng)
                    n += 1
                    tasks.append(asyncio.ensure_future(one(kind, path, body)))
            tasks.append(asyncio.ensure_future(arrivals()))
        if args.mix:
            async def scraper():
                while not state["stop"]:
                    t0 = time.perf_counter()
                    await asgi_call("GET", "/metrics", b"")
                    if state["record"]:
                        lat.setdefault("scrape", []).append(time.perf_counter() - t0)
                    await asyncio.sleep(1.0)
            tasks.append(asyncio.ensure_future(scraper()))
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
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)
        await backend.close()
        if errors:
            raise RuntimeError("bad replies: %s" % errors[:3])
        stats = {k: st1[k] - st0[k] for k in st1 if isinstance(st1[k], (int, float))}
        return el, sample, stats

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
    reply = json.loads(sample[0])["kubectl_command"] if sample else None
    return elapsed, lat, st, t_build, (reply, backend.prompt_ids(make_query(0, 0, 0)))


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: spawn the N ranks ourselves, before anything touches a GPU,
        # as a child torch.distributed.run job (one process per GPU), and exit with its status
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} does not match WORLD_SIZE={world}")
    if args.load == "open" and args.rate <= 0:
        sys.exit("bench.py: --load open needs --rate")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    C = args.concurrency
    rb = max(C, 1) * args.tp   # a replica's largest batch (tp ranks' clients)
    buckets = tuple(b for b in (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 160, 192, 256, 320, 384, 448, 512)
                    if b <= rb)
    if rb not in buckets and rb <= 512:
        buckets = tuple(sorted(set(buckets) | {rb}))

    import torch.distributed as dist

    if world > 1 and not (args.transport == "asgi" and args.in_process):
        dist.init_process_group("gloo")   # barriers / gathers only (no rank touches a GPU itself)
    passes = {"tcp": ["tcp"], "asgi": ["asgi"],
              "both": ["tcp", "asgi"] + ([] if args.no_prefix_off_pass else ["asgi-prefix-off"])}[args.transport]
    results = {}
    for name in passes:
        if name == "tcp":
            r = run_tcp(args, rank, local, world, C, buckets, dist)
            seq_len = prompt_len(args.model) + args.max_new_tokens
        else:
            r = run_asgi(args, rank, local, world, C, buckets, dist, prefix_caching=name == "asgi")
            seq_len = len(r[4][1]) + args.max_new_tokens
        results[name] = summarize(args, name, world, C, dist, r, seq_len)
    if rank == 0:
        head = results[passes[0]]
        out = dict(head["out"])
        detail = out["detail"]
        for name in passes[1:]:
            key = "asgi" if name == "asgi" else "prefix_cache_off"
            detail[key] = results[name]["compact"]
        for name in passes:
            if name in ("tcp", "asgi"):
                out[f"{name}_value"] = results[name]["out"]["value"]
                out[f"{name}_p50_ms"] = results[name]["out"]["p50_ms"]
        if "tcp" in results and "asgi" in results:
            detail["tcp_vs_asgi"] = round(results["tcp"]["out"]["value"] / results["asgi"]["out"]["value"], 3)
        print(json.dumps(out), flush=True)
    if world > 1:
        _barrier(dist)
        dist.destroy_process_group()


def summarize(args, name, world, C, dist, r, seq_len):
    """One pass's JSON (headline form) and compact form; elapsed is the max over ranks."""
    elapsed, lat, st, t_build, extra = r
    rank = int(os.environ.get("RANK", "0"))
    transport = "tcp" if name == "tcp" else "asgi"
    reply = extra[0] if extra else None
    n_req = C * args.steps
    allv = [v for k in ("miss", "hit", "exec") for v in lat.get(k, [])]
    if world > 1:
        # the slowest rank's elapsed time; p50 / p99 over every rank's latencies merged (per-class
        # lists too), so both percentiles describe the same population
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        elapsed = max(g[0].item() for g in gathered)
        lats = [None] * world
        dist.all_gather_object(lats, {k: list(v) for k, v in lat.items()})
        lat = {}
        for d in lats:
            for k, v in d.items():
                lat.setdefault(k, []).extend(v)
        allv = [v for k in ("miss", "hit", "exec") for v in lat.get(k, [])]
    p50 = statistics.median(allv) * 1e3 if allv else float("nan")
    value = n_req * world / elapsed

    def pct(v, q):
        return round(sorted(v)[int(q * (len(v) - 1))] * 1e3, 2) if v else None

    detail = {"concurrency_per_gpu": C, "new_tokens": args.max_new_tokens, "transport": transport,
              "load": args.load + (f"@{args.rate}/s" if args.load == "open" else ""),
              "p99_ms": pct(allv, 0.99), "build_s": round(t_build, 1), "sample_reply": reply,
              "baseline": "BASELINE.md reference plumbing floor, cache-miss conc 32 = 354 req/s (uvicorn, TCP)"}
    if transport == "tcp":
        tp = f" of TP={args.tp}" if args.tp > 1 else ""
        detail.update(topology=f"one server: DP={world // args.tp} replicas{tp}, {args.api_workers * world} API "
                               f"workers, one port",
                      api_workers=args.api_workers * world, client_procs_per_rank=args.client_procs)
    if name == "asgi-prefix-off":
        detail["prefix_caching"] = False
    if args.mix:
        detail["mix"] = {k: {"n": len(v), "p50_ms": pct(v, 0.5), "p99_ms": pct(v, 0.99)} for k, v in lat.items()}
    if st and transport == "tcp":   # from the server's Prometheus histograms
        detail.update({
            "decode_steps": st["decode_steps"], "prefill_steps": st["prefill_steps"],
            "decode_ms_per_step": round(st["decode_ms"] / max(1, st["decode_steps"]), 3),
            "prefill_ms_per_step": round(st["prefill_ms"] / max(1, st["prefill_steps"]), 3),
            "queue_wait_ms_mean": st["queue_wait_ms_mean"], "engine_stats_from": "/metrics",
            "cpu_cores": st.get("cpu_cores")})
    elif st:
        detail.update({
            "decode_steps": st.get("decode_steps"), "prefill_steps": st.get("prefill_steps"),
            "decode_ms_per_step": round(st["decode_ms"] / max(1, st["decode_steps"]), 3),
            "prefill_ms_per_step": round(st["prefill_ms"] / max(1, st["prefill_steps"]), 3),
            "prefill_tokens": st.get("prefill_tokens"), "graph_replays": st.get("graph_replays"),
            "prefix_cache_hit_rate": round(st.get("prefix_hits", 0) / max(1, st.get("prefix_queries", 0)), 3),
            "sub_block_reused_tokens": st.get("partial_tokens", 0),
            "overlapped_decode_steps": st.get("chained_steps", 0),
            "engine_idle_ms_per_step": round(st.get("engine_idle_s", 0.0) * 1e3 / args.steps, 2),
            "engine_process": not args.in_process})
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "req/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": round(value / BASELINE_RPS, 3),
        "dtype": "bf16", "data": "synthetic queries, random-init weights",
        "config": {"model": MODEL_NAMES.get(args.model, args.model),
                   "global_batch": C * world, "seq_len": seq_len, "parallelism": parallelism(args, world)},
        "p50_ms": round(p50, 2), "detail": detail,
    }
    if args.mix:
        out["config"]["mix"] = f"hit {args.hit_frac} exec {args.exec_frac} miss {1 - args.hit_frac - args.exec_frac}"
    compact = {"value": out["value"], "p50_ms": out["p50_ms"], "p99_ms": detail["p99_ms"],
               "ms_per_step": out["ms_per_step"]}
    for k in ("decode_ms_per_step", "prefill_ms_per_step", "prefill_steps", "decode_steps", "prefill_tokens",
              "prefix_cache_hit_rate"):
        if k in detail:
            compact[k] = detail[k]
    return {"out": out, "compact": compact}


if __name__ == "__main__":
    main()
