"""Data parallelism for serving: N engine replicas behind the API process(es), each replica a
tensor-parallel group of t GPUs (DP x TP <= 8 per node).

SURVEY.md §2.5 DP row: the API tier keeps the single TTL cache and rate limiter (so `from_cache`
semantics match `/root/reference/app.py:312-322` exactly — process-local with one API worker, in
shared memory with several: shared_state.py) and every API worker routes its cache misses to the
replica with the fewest of its in-flight requests.  Tokenisation and detokenisation stay in the API
process; only int lists cross the process boundary.

Topology
  supervisor (the API process with DP > 1, or serve.py's WORKERS > 1 supervisor; never touches a GPU)
   └─ replica i (multiprocessing "spawn", started before anything touches a GPU), TP rank 0 of its
      group: binds devices[i][0], spawns its t - 1 TP worker ranks (ModelRunner.worker_loop) on
      devices[i][1:], builds the engine, then listens on a Unix socket `replica<i>.sock`.
API clients (one per API worker process) connect to every replica's socket: one duplex connection
carries the client's requests and the replica's batched completions.

Faults.  A replica that dies — a crash, or the engine's fatal-fault exit
(engine.py: a one-shot collective timeout, a HIP fault, a lost TP worker) — closes its sockets: each
client fails that replica's in-flight requests with LLMUnavailableError (HTTP 503), routes new ones
to the live replicas and keeps reconnecting.  The supervisor respawns the replica in a fresh process
(same devices and socket, exponential backoff, at most `max_restarts` in 10 minutes); the clients
reconnect and it serves again.  Nothing is ever re-exec'ed in a process that touched a GPU.
"""
from __future__ import annotations

import asyncio
import dataclasses
import itertools
import logging
import multiprocessing as mp
import os
import secrets
import socket
import sys
import tempfile
import threading
import time
from multiprocessing.connection import Client, Listener, wait as _wait
from typing import Dict, List, Optional

from ..llm.base import LLMBackend, LLMUnavailableError

FLUSH_EVERY = 16   # requests per engine-bound IPC message within one event-loop tick

logger = logging.getLogger("app.dp")


class _Obs:
    """Histogram stand-in: records observations for shipping to the API process."""

    def __init__(self, sink: list):
        self.sink = sink

    def observe(self, v: float) -> None:
        self.sink.append(v)


class _Labelled:
    """`metric.labels(phase).observe(v)` recorded as (phase, v)."""

    def __init__(self, sink: list):
        self.sink = sink

    def labels(self, phase):
        sink = self.sink

        class _O:
            @staticmethod
            def observe(v):
                sink.append((phase, v))
        return _O


class _Gauge:
    def __init__(self, store: dict, name: str):
        self.store, self.name = store, name

    def set(self, v) -> None:
        self.store[self.name] = v


class EngineMetricsProxy:
    """The engine's metrics interface inside a replica process.  TTFT / TPOT observations and the
    batch / queue / KV gauges ride back to the API process on the batched completion messages and
    are replayed into its Prometheus registry (DPRouterLLM._apply_obs), so /metrics shows the engine
    even though it runs in another process."""

    def __init__(self):
        self.ttft: list = []
        self.tpot: list = []
        self.qwait: list = []
        self.steps: list = []      # (phase, seconds)
        self.gauges: dict = {}
        self.llm_ttft = _Obs(self.ttft)
        self.llm_tpot = _Obs(self.tpot)
        self.llm_queue_wait = _Obs(self.qwait)
        self.llm_step = _Labelled(self.steps)
        self.llm_batch_size = _Gauge(self.gauges, "llm_batch_size")
        self.llm_queue_depth = _Gauge(self.gauges, "llm_queue_depth")
        self.llm_kv_blocks_used = _Gauge(self.gauges, "llm_kv_blocks_used")

    def take(self):
        if not (self.ttft or self.tpot or self.qwait or self.steps or self.gauges):
            return None
        out = {"ttft": self.ttft[:], "tpot": self.tpot[:], "qwait": self.qwait[:], "steps": self.steps[:],
               "gauges": dict(self.gauges)}
        for lst in (self.ttft, self.tpot, self.qwait, self.steps):
            lst.clear()
        self.gauges.clear()
        return out


# ---------------------------------------------------------------------------------------------
@dataclasses.dataclass
class ReplicaSpec:
    """What a replica process needs: its index, its TP group's devices and rendezvous port, and
    the socket its clients connect to."""
    idx: int
    devices: List[str]
    address: str
    master_port: int = 0
    incarnation: int = 0        # 0 = first start, k = k-th respawn
    mem_share: float = 1.0      # this replica's share of each of its GPUs (several replicas on one GPU)

    @property
    def tp(self) -> int:
        return len(self.devices)


@dataclasses.dataclass
class ReplicaDirectory:
    """What an API client holds to reach every replica (picklable: handed to spawned API workers)."""
    addresses: List[str]
    authkey: bytes


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def engine_devices(settings, dp: int, tp: int = 1) -> List[List[str]]:
    """Devices of the dp replicas, t per replica: ENGINE_DEVICES (comma list; `cpu` repeats) or
    cuda:0 .. cuda:dp*t-1 in order (replica i = cuda:i*t .. cuda:i*t+t-1)."""
    devs = [d.strip() for d in (getattr(settings, "ENGINE_DEVICES", "") or "").split(",") if d.strip()]
    n = dp * tp
    if len(devs) < n:
        devs = devs * n if devs and all(d == "cpu" for d in devs) else [f"cuda:{i}" for i in range(n)]
    return [devs[i * tp:(i + 1) * tp] for i in range(dp)]


def _exit_with_parent(parent: int) -> None:
    """A replica / TP worker ends when the process that spawned it is gone (no orphan keeps a GPU)."""
    def watch():
        while True:
            time.sleep(0.5)
            if os.getppid() != parent:
                os._exit(0)
    threading.Thread(target=watch, name="parent-watch", daemon=True).start()


def _tp_env(spec: ReplicaSpec, rank: int) -> None:
    """torch.distributed rendezvous of the replica's TP group (every GPU stays visible: RCCL and the
    IPC-mapped one-shot collectives reach the peers; LOCAL_RANK = the rank's device index)."""
    dev = spec.devices[rank]
    local = dev.split(":")[1] if dev.startswith("cuda") and ":" in dev else "0"
    os.environ.update(RANK=str(rank), LOCAL_RANK=local, WORLD_SIZE=str(spec.tp), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(spec.master_port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    # the group's rank 0 hosts its own store on MASTER_PORT: a torchrun agent store inherited from a
    # launcher (TORCHELASTIC_USE_AGENT_STORE) would make it wait for a server that never comes
    os.environ.pop("TORCHELASTIC_USE_AGENT_STORE", None)


def _tp_worker_main(spec: ReplicaSpec, rank: int, settings_dict: dict, parent: int) -> None:
    """TP rank > 0 of a replica: mirror rank 0's steps until it stops (or dies)."""
    from ..utils.runtime import set_proc_name
    set_proc_name(f"ka-tp-{spec.idx}.{rank}")
    _exit_with_parent(parent)
    _tp_env(spec, rank)
    os.environ["KA_GPU_MEM_SHARE"] = repr(spec.mem_share)
    dev = spec.devices[rank]
    from ..config import Settings
    from ..engine.builder import EngineOptions, build_engine
    from .launch import init_tp

    s = Settings(**settings_dict)
    comm, r = init_tp(spec.tp, backend="gloo" if dev == "cpu" else None)
    opts = EngineOptions.from_settings(s)
    opts.device, opts.tp_rank, opts.tp_size = dev, r, spec.tp
    eng = build_engine(opts, comm=comm)
    if opts.use_graphs and dev.startswith("cuda"):
        eng.runner.capture_graphs()
    eng.runner.worker_loop()


def _replica_main(spec: ReplicaSpec, settings_dict: dict, authkey: bytes, parent: int) -> None:
    """Entry point of one replica process (TP rank 0 of its group)."""
    from ..utils.runtime import set_proc_name
    set_proc_name(f"ka-replica-{spec.idx}")
    _exit_with_parent(parent)
    os.environ.setdefault("KA_EXIT_ON_FATAL", "1")   # a fatal engine fault ends the replica: respawned
    # fault injection (tests): KA_FAULT_STEP applies to replica KA_FAULT_REPLICA's
    # first incarnation only (its respawn serves normally)
    target = os.environ.get("KA_FAULT_REPLICA")
    if target is not None and (int(target) != spec.idx or spec.incarnation > 0):
        os.environ.pop("KA_FAULT_STEP", None)
    os.environ["KA_GPU_MEM_SHARE"] = repr(spec.mem_share)
    dead_path = spec.address + ".dead"
    if os.path.exists(dead_path):
        os.unlink(dead_path)
    if spec.tp > 1:
        # the TP worker ranks are spawned before this process touches a GPU
        ctx = mp.get_context("spawn")
        for r in range(1, spec.tp):
            ctx.Process(target=_tp_worker_main, args=(spec, r, settings_dict, os.getpid()), daemon=True).start()
        _tp_env(spec, 0)
    dev = spec.devices[0]
    import torch  # noqa: F401  (first GPU use happens here, in the child)

    from ..config import Settings
    from ..engine.builder import EngineOptions, build_engine
    from ..engine.safe_decode import forced_prefix
    from ..engine.sequence import SamplingParams

    cpus = []
    if dev.startswith("cuda"):
        from ..utils.runtime import pin_to_device_numa
        cpus = pin_to_device_numa(int(dev.split(":")[1]) if ":" in dev else 0)
    try:
        s = Settings(**settings_dict)
        opts = EngineOptions.from_settings(s)
        opts.device = dev
        comm = None
        if spec.tp > 1:
            from .launch import init_tp
            comm, _ = init_tp(spec.tp, backend="gloo" if dev == "cpu" else None)
            opts.tp_rank, opts.tp_size = 0, spec.tp
        eng = build_engine(opts, comm=comm)
        eng.metrics = EngineMetricsProxy()
        if opts.use_graphs and dev.startswith("cuda"):
            eng.runner.capture_graphs()
        from ..utils.runtime import tune_gc
        tune_gc()
        eng.start()
        params = SamplingParams(max_new_tokens=s.MAX_NEW_TOKENS, ignore_eos=s.IGNORE_EOS, safe_decode=s.SAFE_DECODE)
        forced = forced_prefix(eng.tokenizer) if s.SAFE_DECODE else []
        if os.path.exists(spec.address):
            os.unlink(spec.address)
        listener = Listener(spec.address, family="AF_UNIX", authkey=authkey)
    except Exception as e:  # reported to the clients through the .dead file, then respawned
        logger.exception("DP replica %d failed to start", spec.idx)
        with open(dead_path, "w") as f:
            f.write(repr(e))
        os._exit(3)

    conns: Dict[int, object] = {}          # connection id -> Connection
    send_locks: Dict[int, threading.Lock] = {}
    conns_lock = threading.Lock()
    new_conn = threading.Event()
    cid_of: Dict[int, int] = {}            # connection id -> client id (hello)

    def accept_loop():
        ids = itertools.count()
        while True:
            try:
                c = listener.accept()
            except Exception:   # a client that failed the handshake, or the listener closed
                if listener._listener is None:   # pragma: no cover
                    return
                continue
            k = next(ids)
            with conns_lock:
                conns[k] = c
                send_locks[k] = threading.Lock()
            new_conn.set()

    threading.Thread(target=accept_loop, name="replica-accept", daemon=True).start()

    def send(k: int, msg) -> None:
        c, lk = conns.get(k), send_locks.get(k)
        if c is None:
            return
        try:
            with lk:
                c.send(msg)
        except (OSError, ValueError):
            pass   # the client went away: its EOF is handled in the request loop

    # completions are batched: the engine thread appends, and one message per engine step and
    # client carries all of them back (a wave of 256 finishing together = 1 pickle + 1 socket write)
    done_buf: Dict[int, list] = {}
    done_lock = threading.Lock()

    def done(seq, key):
        err = repr(seq.error) if seq.error is not None else None
        with done_lock:
            done_buf.setdefault(key[0], []).append((key[1], (seq.output_ids, err, seq.finish_reason)))

    last_obs = [0.0]

    def flush():
        nonlocal done_buf
        now = time.perf_counter()
        if done_buf or now - last_obs[0] > 0.05:
            obs = eng.metrics.take()   # engine-level observations go to ONE client (counted once)
            if done_buf or obs is not None:
                with done_lock:
                    bufs, done_buf = done_buf, {}
                last_obs[0] = now
                with conns_lock:
                    ks = sorted(conns)
                obs_k = min(ks, key=lambda k: cid_of.get(k, 1 << 30)) if ks else None
                for k in ks:
                    batch, o = bufs.get(k, []), (obs if k == obs_k else None)
                    if batch or o is not None:
                        send(k, ("done_batch", spec.idx, (batch, o)))

    eng.step_end_hooks.append(flush)

    live: Dict[tuple, object] = {}
    told_healthy: Dict[int, bool] = {}     # connection id -> the health last pushed to that client
    while True:
        with conns_lock:
            items = list(conns.items())
        if not items:
            new_conn.wait(0.5)
            new_conn.clear()
            continue
        # engine health changes (watchdog verdict, recoveries exhausted without exit_on_fatal) are
        # pushed to every client, which then routes around this replica while it is unhealthy
        healthy = bool(eng.healthy)
        for k, _ in items:
            if told_healthy.get(k, True) != healthy:
                told_healthy[k] = healthy
                send(k, ("health", spec.idx, healthy))
        ready = _wait([c for _, c in items], timeout=0.2)
        by_conn = {id(c): k for k, c in items}
        for c in ready:
            k = by_conn[id(c)]
            try:
                msg = c.recv()
            except (EOFError, OSError):
                msg = None
            if msg is None:   # client gone: abort its requests (capacity back to the others)
                with conns_lock:
                    conns.pop(k, None)
                    send_locks.pop(k, None)
                told_healthy.pop(k, None)
                for key in [key for key in live if key[0] == k]:
                    eng.abort(live.pop(key))
                continue
            msgs = msg[2] if msg[0] == "batch" else [msg]
            for op, rid, payload in msgs:
                key = (k, rid)
                if op == "gen":
                    if not eng.healthy:   # an unhealthy engine takes no work: the client answers 503
                        send(k, ("done_batch", spec.idx,
                                 ([(rid, ([], repr(RuntimeError(f"engine unhealthy: {eng.last_error}")), "error"))],
                                  None)))
                        continue
                    seq = eng.submit(payload, params, lambda sq, key=key: done(sq, key), forced_prefix=forced)
                    live[key] = seq
                elif op == "abort":
                    if key in live:
                        eng.abort(live.pop(key))
                elif op == "hello":
                    cid_of[k] = int(payload or 0)
                    send(k, ("ready", spec.idx, cpus))
                elif op == "sync":   # barrier helper: all queued GPU work of this replica is done
                    import torch as _t
                    if dev.startswith("cuda"):
                        _t.cuda.synchronize(dev)
                    send(k, ("ctl", rid, dict(eng.runner.stats, prefix_hits=eng.bm.hits,
                                              prefix_queries=eng.bm.queries,
                                              partial_tokens=getattr(eng.bm, "partial_tokens", 0),
                                              chained_steps=eng.chained_steps, engine_idle_s=eng.idle_s,
                                              build_s=getattr(eng, "build_seconds", 0.0))))
                elif op == "health":
                    send(k, ("ctl", rid, {"healthy": eng.healthy, "recoveries": eng.recoveries,
                                          "failures": eng.failures, "pid": os.getpid()}))
        if len(live) > 4096:
            live = {key: v for key, v in live.items() if not v.finished}


# ---------------------------------------------------------------------------------------------
class ReplicaSupervisor:
    """Spawns the replicas and keeps them alive: a replica process that exits is respawned (same
    devices, same socket) after an exponential backoff, at most `max_restarts` times in 10 minutes.
    Runs in a process that never touches a GPU (the API process with DP > 1, or serve.py's
    WORKERS > 1 supervisor)."""

    def __init__(self, settings, dp: Optional[int] = None, devices: Optional[List[List[str]]] = None,
                 run_dir: Optional[str] = None, respawn: Optional[bool] = None, max_restarts: int = 5):
        tp = max(1, int(getattr(settings, "TP", 1) or 1))
        dp = dp if dp is not None else max(1, int(getattr(settings, "DP", 1) or 1))
        self.devices = devices or engine_devices(settings, dp, tp)
        self.run_dir = run_dir or tempfile.mkdtemp(prefix="ka_dp_")
        self.authkey = secrets.token_bytes(16)
        sd = dataclasses.asdict(settings)
        sd.update(TP=1, DP=1)
        self.settings_dict = sd
        # ranks sharing a GPU split its memory (tests put a DP x TP layout on one device)
        per_dev: Dict[str, int] = {}
        for d in self.devices:
            for x in d:
                per_dev[x] = per_dev.get(x, 0) + 1
        self.specs = [ReplicaSpec(i, list(d), os.path.join(self.run_dir, f"replica{i}.sock"),
                                  _free_port() if len(d) > 1 else 0,
                                  mem_share=1.0 / max(per_dev[x] for x in d) if d[0] != "cpu" else 1.0)
                      for i, d in enumerate(self.devices)]
        self.respawn = (os.environ.get("KA_REPLICA_RESPAWN", "1") == "1") if respawn is None else respawn
        self.max_restarts = max_restarts
        self.ctx = mp.get_context("spawn")
        self.procs: List[Optional[mp.Process]] = [None] * len(self.specs)
        self.restarts: List[List[float]] = [[] for _ in self.specs]
        self._next_at = [0.0] * len(self.specs)
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.respawned = 0

    @property
    def directory(self) -> ReplicaDirectory:
        return ReplicaDirectory([s.address for s in self.specs], self.authkey)

    def _spawn(self, i: int) -> None:
        spec = self.specs[i]
        if self.procs[i] is not None:
            spec = self.specs[i] = dataclasses.replace(spec, incarnation=spec.incarnation + 1)
        p = self.ctx.Process(target=_replica_main, args=(spec, self.settings_dict, self.authkey, os.getpid()),
                             daemon=False, name=f"ka-replica-{i}")
        p.start()
        self.procs[i] = p

    def start(self) -> "ReplicaSupervisor":
        for i in range(len(self.specs)):
            self._spawn(i)
        self._thread = threading.Thread(target=self._watch, name="dp-supervisor", daemon=True)
        self._thread.start()
        return self

    def pids(self) -> List[Optional[int]]:
        return [p.pid if p is not None else None for p in self.procs]

    def _watch(self) -> None:
        while not self._stop.wait(0.2):
            self.poll()

    def poll(self) -> None:
        """One supervision pass: respawn replicas whose process has exited."""
        now = time.monotonic()
        for i, p in enumerate(self.procs):
            if p is None or p.is_alive() or self._stop.is_set():
                continue
            if self._next_at[i] == 0.0:
                logger.error("DP replica %d exited (status %s)", i, p.exitcode)
                hist = [t for t in self.restarts[i] if now - t < 600.0]
                self.restarts[i] = hist
                if not self.respawn or len(hist) >= self.max_restarts:
                    logger.error("DP replica %d stays down (%d restarts in 10 min)", i, len(hist))
                    self._next_at[i] = float("inf")
                    continue
                self._next_at[i] = now + min(30.0, 0.5 * (2 ** len(hist)))
            if now >= self._next_at[i]:
                self.restarts[i].append(now)
                self._next_at[i] = 0.0
                logger.warning("respawning DP replica %d on %s", i, ",".join(self.specs[i].devices))
                self._spawn(i)
                self.respawned += 1

    def stop(self, timeout: float = 30.0) -> None:
        self._stop.set()
        for p in self.procs:
            if p is not None and p.is_alive():
                p.terminate()
        for p in self.procs:
            if p is not None:
                p.join(timeout)
                if p.is_alive():
                    p.kill()


# ---------------------------------------------------------------------------------------------
@dataclasses.dataclass
class _Replica:
    idx: int
    address: str
    conn: object = None
    inflight: int = 0
    up: bool = False
    healthy: bool = True                  # the replica's engine health, pushed by the replica
    failed: Optional[str] = None          # startup failure reported by the replica (.dead file)
    outbox: list = dataclasses.field(default_factory=list)
    flush_scheduled: bool = False
    cpus: list = dataclasses.field(default_factory=list)
    next_try: float = 0.0
    lock: threading.Lock = dataclasses.field(default_factory=threading.Lock)

    def put(self, msg) -> None:
        c = self.conn
        if c is None:
            raise OSError("replica not connected")
        with self.lock:
            c.send(msg)


class DPRouterLLM(LLMBackend):
    """LLM backend that fans requests out over DP engine replicas."""

    name = "engine-dp"

    def __init__(self, settings, dp: int, devices: Optional[List] = None, start_timeout: float = 900,
                 endpoints: Optional[ReplicaDirectory] = None, client_id: int = 0):
        """Spawns (and supervises) its own `dp` replicas, or (`endpoints`) connects to replicas
        another process supervises for several API workers (serve.py WORKERS > 1).  `devices`: one
        device (TP = 1) or one device list (a TP group) per replica."""
        from ..engine.tokenizer import get_tokenizer, tokenizer_path
        from ..models.config import get_config
        from ..prompt import PROMPT_PREFIX

        cfg = get_config(settings.MODEL)
        self.tok = get_tokenizer(cfg.vocab_size, cfg.tokenizer, tokenizer_path(settings.WEIGHTS))
        before, after = self.tok.chat_prefix_suffix()
        self._prefix = before + self.tok.encode(PROMPT_PREFIX)
        self._after = after
        self.settings = settings
        self.client_id = client_id
        self.supervisor: Optional[ReplicaSupervisor] = None
        if endpoints is None:
            devs = None
            if devices is not None:
                devs = [list(d) if isinstance(d, (list, tuple)) else [d] for d in devices]
            self.supervisor = ReplicaSupervisor(settings, dp, devs).start()
            endpoints = self.supervisor.directory
        self.owner = self.supervisor is not None
        self.authkey = endpoints.authkey
        self.replicas: List[_Replica] = [_Replica(i, a) for i, a in enumerate(endpoints.addresses)]
        # several API workers in front of the same replicas (serve.py WORKERS > 1): least-loaded
        # routing over every worker's in-flight counts, kept in the shared state's load table
        # (each worker writes its own row); a single router balances on its own counts
        self.loads = None
        if not self.owner:
            from ..shared_state import open_from_settings
            try:
                self.loads = open_from_settings(settings)
            except Exception:   # pragma: no cover - no native runtime: local counts only
                self.loads = None
            if self.loads is not None:
                self.loads.load_clear_worker(client_id)   # a respawned worker's row starts at zero
        # the reply-reader thread must get the GIL promptly while the event loop is busy
        sys.setswitchinterval(min(sys.getswitchinterval(), 0.001))
        self._pending: Dict[int, tuple] = {}
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._ready = threading.Event()
        self._metrics = None
        self._gauges: Dict[int, dict] = {}
        self._closing = False
        self.reconnects = 0
        self._reader = threading.Thread(target=self._read_loop, name="dp-router", daemon=True)
        self._reader.start()
        self._start_timeout = start_timeout

    # -----------------------------------------------------------------------------------------
    def _try_connect(self, r: _Replica) -> None:
        now = time.monotonic()
        if now < r.next_try:
            return
        r.next_try = now + 0.25
        try:
            c = Client(r.address, family="AF_UNIX", authkey=self.authkey)
        except (OSError, EOFError):
            dead = r.address + ".dead"
            if os.path.exists(dead) and not r.failed:
                try:
                    with open(dead) as f:
                        r.failed = f.read() or "startup failed"
                except OSError:
                    r.failed = "startup failed"
                logger.error("DP replica %d failed to start: %s", r.idx, r.failed)
                self._check_ready()
            return
        r.failed = None
        try:
            c.send(("hello", 0, self.client_id))
        except OSError:
            c.close()
            return
        r.conn = c   # up once its "ready" arrives

    def _on_down(self, r: _Replica, why: str) -> None:
        was_up = r.up
        r.up = False
        c, r.conn = r.conn, None
        if c is not None:
            try:
                c.close()
            except OSError:
                pass
        r.outbox = []
        if was_up and not self._closing:
            logger.error("DP replica %d down: %s", r.idx, why)
        self._fail_replica(r)

    def _check_ready(self) -> None:
        if all(r.up or r.failed for r in self.replicas):
            self._ready.set()

    def _read_loop(self) -> None:
        while not self._closing:
            for r in self.replicas:
                if r.conn is None:
                    self._try_connect(r)
            conns = {id(r.conn): r for r in self.replicas if r.conn is not None}
            if not conns:
                time.sleep(0.05)
                continue
            try:
                ready = _wait([r.conn for r in conns.values()], timeout=0.1)
            except (OSError, ValueError):
                ready = []
            for c in ready:
                r = conns.get(id(c))
                if r is None or r.conn is not c:
                    continue
                try:
                    kind, a, b = c.recv()
                except (EOFError, OSError, ValueError):
                    self._on_down(r, "connection closed")
                    continue
                self._dispatch(r, kind, a, b)

    def _dispatch(self, r: _Replica, kind, a, b) -> None:
        if kind == "ready":
            if not r.up and self._ready.is_set():
                self.reconnects += 1
                logger.warning("DP replica %d is back", r.idx)
            r.up = True
            r.healthy = True   # a (re)started replica reports a change of health itself
            r.cpus = list(b or [])
            if len(self.replicas) == 1 and r.cpus and self.owner:
                # one replica (a bench rank, or DP=1 serving): the API process joins its engine on
                # the GPU's NUMA node
                from ..utils.runtime import pin_process
                pin_process(r.cpus)
            self._check_ready()
        elif kind == "done_batch":
            items, obs = b
            if obs is not None and self._metrics is not None:
                self._apply_obs(a, obs)
            by_loop = {}
            with self._lock:
                for rid, payload in items:
                    ent = self._pending.pop(rid, None)
                    if ent is not None:
                        ent[2].inflight -= 1
                        by_loop.setdefault(ent[0], []).append((ent[1], payload))
                self._publish_load(r)
            for loop, lst in by_loop.items():
                loop.call_soon_threadsafe(_set_many, lst)
        elif kind == "ctl":
            with self._lock:
                ent = self._pending.pop(a, None)
            if ent is not None:
                ent[0].call_soon_threadsafe(_set, ent[1], b)
        elif kind == "health":
            if r.healthy != bool(b):
                logger.error("DP replica %d reports its engine %s", r.idx, "healthy" if b else "UNHEALTHY")
            r.healthy = bool(b)

    def attach_metrics(self, metrics) -> None:
        self._metrics = metrics

    def _apply_obs(self, idx: int, obs: dict) -> None:
        m = self._metrics
        for v in obs["ttft"]:
            m.llm_ttft.observe(v)
        for v in obs["tpot"]:
            m.llm_tpot.observe(v)
        for v in obs.get("qwait", ()):
            m.llm_queue_wait.observe(v)
        for phase, v in obs.get("steps", ()):
            m.llm_step.labels(phase).observe(v)
        if obs["gauges"]:
            self._gauges[idx] = {**self._gauges.get(idx, {}), **obs["gauges"]}
            for name in ("llm_batch_size", "llm_queue_depth", "llm_kv_blocks_used"):
                getattr(m, name).set(sum(g.get(name, 0) for g in self._gauges.values()))

    def _publish_load(self, r) -> None:
        if self.loads is not None and isinstance(r, _Replica):
            self.loads.load_set(self.client_id, r.idx, r.inflight)

    def _pick(self, live: List["_Replica"]) -> "_Replica":
        """Least-loaded live replica: over every API worker's in-flight requests when they share a
        load table, else over this router's own."""
        if self.loads is not None and len(self.replicas) > 1:
            mask = 0
            for r in live:
                mask |= 1 << r.idx
            i = self.loads.load_pick(len(self.replicas), mask)
            if i >= 0:
                return self.replicas[i]
        return min(live, key=lambda r: r.inflight)

    def _fail_replica(self, r) -> None:
        """Fail every pending request and control op routed to `r` (503)."""
        with self._lock:
            dead = [(k, v) for k, v in self._pending.items() if v[2] is r]
            for k, _ in dead:
                self._pending.pop(k)
            r.inflight = 0
            self._publish_load(r)
        for _, (loop, fut, *_rest) in dead:
            loop.call_soon_threadsafe(_set_exc, fut, LLMUnavailableError(f"replica {r.idx} died"))

    def wait_ready(self, timeout: Optional[float] = None) -> bool:
        return self._ready.wait(timeout if timeout is not None else self._start_timeout)

    async def start(self) -> None:
        loop = asyncio.get_running_loop()
        await loop.run_in_executor(None, self.wait_ready)

    async def close(self) -> None:
        """Disconnect from every replica; an owning router also stops its replicas."""
        self._closing = True
        for r in self.replicas:
            c, r.conn = r.conn, None
            r.up = False
            if c is not None:
                try:
                    c.close()
                except OSError:
                    pass
        if self.supervisor is not None:
            loop = asyncio.get_running_loop()
            await loop.run_in_executor(None, self.supervisor.stop)

    def healthy(self) -> bool:
        return any(r.up and r.healthy for r in self.replicas)

    def stats(self):
        return {f"replica{r.idx}_inflight": r.inflight for r in self.replicas}

    def _send(self, rep, msg, loop) -> None:
        """Queue a message for a replica; all messages queued in one event-loop tick go out as
        one `batch` message (a burst of concurrent requests = one pickle + one socket write)."""
        rep.outbox.append(msg)
        if len(rep.outbox) >= FLUSH_EVERY:
            # a burst larger than this is handed over in chunks so the engine starts on the first
            # requests while this process is still parsing the rest (the scheduler re-batches)
            self._flush(rep)
        elif not rep.flush_scheduled:
            rep.flush_scheduled = True
            loop.call_soon(self._flush, rep)

    def _flush(self, rep) -> None:
        rep.flush_scheduled = False
        if rep.outbox:
            batch, rep.outbox = rep.outbox, []
            try:
                rep.put(("batch", 0, batch) if len(batch) > 1 else batch[0])
            except (OSError, ValueError) as e:   # replica died: fail what was just routed to it
                logger.error("DP replica %d unreachable: %s", rep.idx, e)
                rep.up = False
                self._fail_replica(rep)

    async def control(self, op: str = "sync") -> List[dict]:
        """Send a control op to every live replica and gather the replies (sync = device barrier
        + engine stats; health = engine health, recovery counters and pid)."""
        loop = asyncio.get_running_loop()
        futs = []
        for r in self.replicas:
            if not r.up:
                continue
            rid = next(self._ids)
            fut = loop.create_future()
            with self._lock:
                # registered with the real replica, so its death fails the op (_fail_replica); the
                # "ctl" reply pops it without touching the request in-flight counts
                self._pending[rid] = (loop, fut, r, "ctl")
            try:
                r.put((op, rid, None))
            except (OSError, ValueError) as e:
                with self._lock:
                    self._pending.pop(rid, None)
                fut.set_exception(LLMUnavailableError(f"replica {r.idx} unreachable: {e}"))
            futs.append(fut)
        return list(await asyncio.gather(*futs))

    # -----------------------------------------------------------------------------------------
    def prompt_ids(self, query: str) -> List[int]:
        from ..prompt import PROMPT_SUFFIX
        return self._prefix + self.tok.encode(query + PROMPT_SUFFIX) + self._after

    async def generate(self, query: str) -> str:
        if not self._ready.is_set():
            await self.start()
        live = [r for r in self.replicas if r.up and r.healthy]
        if not live:
            raise LLMUnavailableError("no live DP replica")
        rep = self._pick(live)
        rid = next(self._ids)
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with self._lock:
            self._pending[rid] = (loop, fut, rep)
            rep.inflight += 1
            self._publish_load(rep)
        self._send(rep, ("gen", rid, self.prompt_ids(query)), loop)
        try:
            out_ids, err, reason = await fut
        except asyncio.CancelledError:
            try:
                self._send(rep, ("abort", rid, None), loop)
            except Exception:
                pass
            with self._lock:
                if self._pending.pop(rid, None) is not None:
                    rep.inflight -= 1
                    self._publish_load(rep)
            raise
        if err is not None:
            raise LLMUnavailableError(err) if reason == "error" else RuntimeError(err)
        return self.tok.decode([t for t in out_ids if not self.tok.is_eos(t)])


def _set_many(lst):
    for fut, val in lst:
        if not fut.done():
            fut.set_result(val)


def _set(fut, val):
    if not fut.done():
        fut.set_result(val)


def _set_exc(fut, exc):
    if not fut.done():
        fut.set_exception(exc)
