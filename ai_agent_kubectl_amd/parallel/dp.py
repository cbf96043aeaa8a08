"""Data parallelism for serving: N engine replicas (one process per GPU) behind the API process(es).

SURVEY.md §2.5 DP row: the API tier keeps the single TTL cache and rate limiter (so `from_cache`
semantics match `/root/reference/app.py:312-322` exactly — process-local with one API worker,
in shared memory with several: shared_state.py) and every API worker routes its cache misses to
the replica with the fewest of its in-flight requests.  A replica serves several API workers:
one request pipe per (replica, worker) and one reply queue per worker (`spawn_replicas`).  Replicas are spawned (multiprocessing "spawn")
BEFORE the API process touches the GPU; each binds `cuda:i`, builds its engine (random-init or
safetensors weights, hipGraph capture) and serves token-id requests from a queue.  Tokenisation
and detokenisation stay in the API process; only int lists cross the process boundary.

A replica that dies (or fails to start) is marked down; its in-flight requests fail with
LLMUnavailableError (HTTP 503) and new requests go to the remaining replicas.
"""
from __future__ import annotations

import asyncio
import dataclasses
import itertools
import logging
import multiprocessing as mp
import os
import sys
import threading
import time
from typing import Dict, List, Optional

from ..llm.base import LLMBackend, LLMUnavailableError

FLUSH_EVERY = 16   # requests per engine-bound IPC message within one event-loop tick

logger = logging.getLogger("app.dp")


class _PipeSender:
    """Request channel API process -> replica.  `put` pickles and writes on the calling thread
    (mp.Queue hands both to a feeder thread, which waits for the GIL while the event loop turns a
    burst of replies into new requests: measured as ~15 ms of engine idle per wave)."""

    def __init__(self, conn):
        self.conn = conn
        self.lock = threading.Lock()

    def put(self, obj) -> None:
        with self.lock:
            self.conn.send(obj)


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


def _replica_main(idx: int, device: str, settings_dict: dict, req_conns, resp_qs) -> None:
    """Entry point of one replica process.  `req_conns[c]` / `resp_qs[c]` are the request pipe and
    the reply queue of API client c (one per API worker process)."""
    if not isinstance(req_conns, (list, tuple)):
        req_conns, resp_qs = [req_conns], [resp_qs]
    os.environ.setdefault("KA_EXIT_ON_FATAL", "1")   # a fatal engine fault ends the replica: respawned
    import torch  # noqa: F401  (first CUDA use happens here, in the child)

    from ..config import Settings
    from ..engine.builder import EngineOptions, build_engine
    from ..engine.safe_decode import forced_prefix
    from ..engine.sequence import SamplingParams

    cpus = []
    if device.startswith("cuda"):
        from ..utils.runtime import pin_to_device_numa
        cpus = pin_to_device_numa(int(device.split(":")[1]) if ":" in device else 0)
    try:
        s = Settings(**settings_dict)
        opts = EngineOptions.from_settings(s)
        opts.device = device
        eng = build_engine(opts)
        eng.metrics = EngineMetricsProxy()
        if opts.use_graphs and device.startswith("cuda"):
            eng.runner.capture_graphs()
        from ..utils.runtime import tune_gc
        tune_gc()
        eng.start()
        params = SamplingParams(max_new_tokens=s.MAX_NEW_TOKENS, ignore_eos=s.IGNORE_EOS, safe_decode=s.SAFE_DECODE)
        forced = forced_prefix(eng.tokenizer) if s.SAFE_DECODE else []
        for q in resp_qs:
            q.put(("ready", idx, cpus))
    except Exception as e:  # pragma: no cover - reported to the router
        for q in resp_qs:
            q.put(("dead", idx, repr(e)))
        return

    # completions are batched: the engine thread appends, and one message per engine step and
    # client carries all of them back (a wave of 256 finishing together = 1 pickle + 1 pipe write)
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
            obs = eng.metrics.take()   # engine-level observations go to client 0 only (counted once)
            if done_buf or obs is not None:
                with done_lock:
                    bufs, done_buf = done_buf, {}
                last_obs[0] = now
                for c in range(len(resp_qs)):
                    batch, o = bufs.get(c, []), (obs if c == 0 else None)
                    if batch or o is not None:
                        resp_qs[c].put(("done_batch", idx, (batch, o)))

    eng.step_end_hooks.append(flush)

    from multiprocessing.connection import wait as _wait

    def requests():
        conns = list(req_conns)
        client_of = {id(cn): c for c, cn in enumerate(req_conns)}
        while conns:
            for cn in _wait(conns):
                try:
                    msg = cn.recv()
                except EOFError:   # that API process went away
                    msg = None
                if msg is None:
                    conns.remove(cn)
                    continue
                c = client_of[id(cn)]
                if msg[0] == "batch":
                    for m in msg[2]:
                        yield c, m
                else:
                    yield c, msg

    live = {}
    for client, msg in requests():
        op, rid, payload = msg
        key = (client, rid)
        if op == "sync":           # barrier helper: all queued GPU work of this replica is done
            import torch as _t
            if device.startswith("cuda"):
                _t.cuda.synchronize(device)
            resp_qs[client].put(("ctl", rid, dict(eng.runner.stats, prefix_hits=eng.bm.hits,
                                                  prefix_queries=eng.bm.queries,
                                                  partial_tokens=getattr(eng.bm, "partial_tokens", 0),
                                                  chained_steps=eng.chained_steps, engine_idle_s=eng.idle_s,
                                                  build_s=getattr(eng, "build_seconds", 0.0))))
            continue
        if op == "gen":
            seq = eng.submit(payload, params, lambda sq, key=key: done(sq, key), forced_prefix=forced)
            live[key] = seq
        elif op == "abort" and key in live:
            eng.abort(live.pop(key))
        if len(live) > 4096:
            live = {k: v for k, v in live.items() if not v.finished}
    eng.shutdown()


@dataclasses.dataclass
class ReplicaEndpoints:
    """What one API client (worker process) holds to talk to every replica."""
    senders: list          # per replica: the write end of this client's request pipe
    resp_q: object         # this client's reply queue (shared by all replicas)
    pids: List[int]


def engine_devices(settings, dp: int) -> List[str]:
    devs = [d.strip() for d in (getattr(settings, "ENGINE_DEVICES", "") or "").split(",") if d.strip()]
    return devs[:dp] if len(devs) >= dp else [f"cuda:{i}" for i in range(dp)]


def spawn_replicas(settings, devices: List[str], n_clients: int):
    """Start one engine replica process per device, each serving `n_clients` API clients.
    Must run before the calling process touches the GPU (spawned children bind the devices)."""
    ctx = mp.get_context("spawn")
    resp_qs = [ctx.Queue() for _ in range(n_clients)]
    sd = dataclasses.asdict(settings)
    sd.update(TP=1, DP=1)
    procs, senders = [], [[] for _ in range(n_clients)]
    for i, dev in enumerate(devices):
        r_ends = []
        for c in range(n_clients):
            r_end, w_end = ctx.Pipe(duplex=False)
            r_ends.append(r_end)
            senders[c].append(w_end)
        p = ctx.Process(target=_replica_main, args=(i, dev, sd, r_ends, resp_qs), daemon=True)
        p.start()
        for r_end in r_ends:
            r_end.close()
        procs.append(p)
    pids = [p.pid for p in procs]
    return procs, [ReplicaEndpoints(senders[c], resp_qs[c], pids) for c in range(n_clients)]


def _pid_alive(pid: Optional[int]) -> bool:
    if not pid:
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:  # pragma: no cover
        return True
    return True


@dataclasses.dataclass
class _Replica:
    idx: int
    proc: Optional[mp.Process]   # None when another process (serve.py's supervisor) owns it
    req_q: object
    inflight: int = 0
    up: bool = False
    outbox: list = dataclasses.field(default_factory=list)
    flush_scheduled: bool = False
    cpus: list = dataclasses.field(default_factory=list)   # NUMA-local CPUs the replica pinned to
    pid: Optional[int] = None

    def alive(self) -> bool:
        return self.proc.is_alive() if self.proc is not None else _pid_alive(self.pid)


class DPRouterLLM(LLMBackend):
    """LLM backend that fans requests out over DP engine replicas."""

    name = "engine-dp"

    def __init__(self, settings, dp: int, devices: Optional[List[str]] = None, start_timeout: float = 900,
                 endpoints: Optional[ReplicaEndpoints] = None):
        """Spawns its own `dp` replicas, or (`endpoints`) attaches to replicas another process
        spawned for several API workers (serve.py WORKERS > 1)."""
        from ..engine.tokenizer import get_tokenizer, tokenizer_path
        from ..models.config import get_config
        from ..prompt import PROMPT_PREFIX

        cfg = get_config(settings.MODEL)
        self.tok = get_tokenizer(cfg.vocab_size, cfg.tokenizer, tokenizer_path(settings.WEIGHTS))
        before, after = self.tok.chat_prefix_suffix()
        self._prefix = before + self.tok.encode(PROMPT_PREFIX)
        self._after = after
        self.settings = settings
        self.owner = endpoints is None
        if endpoints is None:
            self.devices = devices or engine_devices(settings, dp)
            procs, eps = spawn_replicas(settings, self.devices, 1)
            endpoints = eps[0]
        else:
            self.devices = [f"replica{i}" for i in range(len(endpoints.senders))]
            procs = [None] * len(endpoints.senders)
        self.resp_q = endpoints.resp_q
        self.replicas: List[_Replica] = [_Replica(i, procs[i], _PipeSender(w), pid=endpoints.pids[i])
                                         for i, w in enumerate(endpoints.senders)]
        # the reply-reader thread must get the GIL promptly while the event loop is busy
        sys.setswitchinterval(min(sys.getswitchinterval(), 0.001))
        self._pending: Dict[int, tuple] = {}
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._ready = threading.Event()
        self._n_ready = 0
        self._metrics = None
        self._gauges: Dict[int, dict] = {}
        self._reader = threading.Thread(target=self._read_loop, name="dp-router", daemon=True)
        self._reader.start()
        self._start_timeout = start_timeout

    # -----------------------------------------------------------------------------------------
    def _read_loop(self) -> None:
        while True:
            try:
                kind, a, b = self.resp_q.get(timeout=1.0)
            except Exception:
                self._check_alive()
                continue
            if kind == "ready":
                self.replicas[a].up = True
                self.replicas[a].cpus = list(b or [])
                if len(self.replicas) == 1 and self.replicas[a].cpus:
                    # one replica (a bench rank, or DP=1 serving): the API process joins its
                    # engine on the GPU's NUMA node
                    from ..utils.runtime import pin_process
                    pin_process(self.replicas[a].cpus)
                self._n_ready += 1
                if self._n_ready == len(self.replicas):
                    self._ready.set()
            elif kind == "dead":
                logger.error("DP replica %d failed to start: %s", a, b)
                self.replicas[a].up = False
                self._n_ready += 1
                if self._n_ready == len(self.replicas):
                    self._ready.set()
            elif kind in ("done", "done_batch"):
                if kind == "done_batch":
                    items, obs = b
                    if obs is not None and self._metrics is not None:
                        self._apply_obs(a, obs)
                else:
                    items = [(a, b)]
                by_loop = {}
                with self._lock:
                    for rid, payload in items:
                        ent = self._pending.pop(rid, None)
                        if ent is not None:
                            ent[2].inflight -= 1
                            by_loop.setdefault(ent[0], []).append((ent[1], payload))
                for loop, lst in by_loop.items():
                    loop.call_soon_threadsafe(_set_many, lst)
            elif kind == "ctl":
                with self._lock:
                    ent = self._pending.pop(a, None)
                if ent is not None:
                    ent[0].call_soon_threadsafe(_set, ent[1], b)
            elif kind == "stop":
                return

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

    def _check_alive(self) -> None:
        for r in self.replicas:
            if r.up and not r.alive():
                logger.error("DP replica %d died (exit %s)", r.idx, r.proc.exitcode if r.proc is not None else "?")
                r.up = False
                self._fail_replica(r)

    def _fail_replica(self, r) -> None:
        with self._lock:
            dead = [(k, v) for k, v in self._pending.items() if v[2] is r]
            for k, _ in dead:
                self._pending.pop(k)
        for _, (loop, fut, _) in dead:
            loop.call_soon_threadsafe(_set_exc, fut, LLMUnavailableError(f"replica {r.idx} died"))

    def wait_ready(self, timeout: Optional[float] = None) -> bool:
        return self._ready.wait(timeout if timeout is not None else self._start_timeout)

    async def start(self) -> None:
        loop = asyncio.get_running_loop()
        await loop.run_in_executor(None, self.wait_ready)

    async def close(self) -> None:
        """Disconnect from every replica; an owning router also waits for its replicas to exit
        (a replica serving several API workers exits when the last one disconnects)."""
        for r in self.replicas:
            try:
                r.req_q.put(None)
            except Exception:
                pass
        for r in self.replicas:
            if r.proc is None:
                continue
            r.proc.join(timeout=30)
            if r.proc.is_alive():
                r.proc.terminate()
        self.resp_q.put(("stop", 0, None))

    def healthy(self) -> bool:
        return any(r.up for r in self.replicas)

    def stats(self):
        return {f"replica{r.idx}_inflight": r.inflight for r in self.replicas}

    def _send(self, rep, msg, loop) -> None:
        """Queue a message for a replica; all messages queued in one event-loop tick go out as
        one `batch` message (a burst of concurrent requests = one pickle + one pipe write)."""
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
                rep.req_q.put(("batch", 0, batch) if len(batch) > 1 else batch[0])
            except (OSError, ValueError) as e:   # replica died: fail what was just routed to it
                logger.error("DP replica %d unreachable: %s", rep.idx, e)
                rep.up = False
                self._fail_replica(rep)

    async def control(self, op: str = "sync") -> List[dict]:
        """Send a control op to every live replica and gather the replies (sync = device barrier
        + engine stats)."""
        loop = asyncio.get_running_loop()
        futs = []
        for r in self.replicas:
            if not r.up:
                continue
            rid = next(self._ids)
            fut = loop.create_future()
            with self._lock:
                self._pending[rid] = (loop, fut, _Dummy())
            r.req_q.put((op, rid, None))
            futs.append(fut)
        return list(await asyncio.gather(*futs))

    # -----------------------------------------------------------------------------------------
    def prompt_ids(self, query: str) -> List[int]:
        from ..prompt import PROMPT_SUFFIX
        return self._prefix + self.tok.encode(query + PROMPT_SUFFIX) + self._after

    async def generate(self, query: str) -> str:
        if not self._ready.is_set():
            await self.start()
        live = [r for r in self.replicas if r.up]
        if not live:
            raise LLMUnavailableError("no live DP replica")
        rep = min(live, key=lambda r: r.inflight)
        rid = next(self._ids)
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with self._lock:
            self._pending[rid] = (loop, fut, rep)
            rep.inflight += 1
        self._send(rep, ("gen", rid, self.prompt_ids(query)), loop)
        try:
            out_ids, err, reason = await fut
        except asyncio.CancelledError:
            self._send(rep, ("abort", rid, None), loop)
            with self._lock:
                if self._pending.pop(rid, None) is not None:
                    rep.inflight -= 1
            raise
        if err is not None:
            raise LLMUnavailableError(err) if reason == "error" else RuntimeError(err)
        return self.tok.decode([t for t in out_ids if not self.tok.is_eos(t)])


class _Dummy:
    inflight = 0


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
