"""LLMEngine: request queue -> scheduler -> runner loop on a dedicated thread.

The API process is asyncio (uvicorn); the GPU loop runs on one background thread so the event loop
keeps serving cache hits, `/execute` and `/metrics` while tokens are generated.  The two sides meet
through a thread-safe inbox and per-request callbacks (the asyncio side wraps them with
`loop.call_soon_threadsafe`, llm/engine_backend.py).  This replaces `chain.ainvoke`
(`/root/reference/app.py:184`).

Per step: drain inbox/aborts -> `Scheduler.schedule()` -> `ModelRunner.execute()` -> append tokens,
publish completed prefix blocks, stop on EOS / max_new_tokens -> callbacks.

Faults.  A step that raises fails every in-flight request (HTTP 503, the
reference's degraded-mode status, `/root/reference/app.py:179-180`) instead of hanging, then:
* recoverable (a host-side error, a transient allocation failure): the engine drops its transient
  state (KV block tables were freed with the requests, the prefix cache is reset), checks that the
  device still answers, and serves again — at most `max_recoveries` times per minute;
* fatal (a one-shot TP collective timed out, a HIP fault, a TP group, too many recoveries, or the
  TP watchdog's verdict: a lost worker rank / a stalled step, `mark_unhealthy`): the engine stays
  unhealthy (`/ready` 503, new requests rejected) and, with `exit_on_fatal` (serve.py / DP
  replicas), the process exits non-zero so its supervisor restarts it — the reference relies on the same
  process-level restart (`/root/reference/docker-compose.yml:14`, `restart: unless-stopped`).
Fault injection: KA_FAULT_STEP=<n>[:fatal|:exit] raises in step n (tests, `FAULT_*` of §5.3).
"""
from __future__ import annotations

import logging
import os
import queue
import sys
import threading
import time
from typing import Callable, Dict, List, Optional

from .block_manager import make_block_manager
from .runner import CollectiveTimeout, ModelRunner
from .scheduler import Scheduler
from .sequence import PLACEHOLDER, SamplingParams, Sequence, SeqStatus

logger = logging.getLogger("app.engine")

EXIT_FATAL = 75   # process exit status after an unrecoverable engine fault (supervisors restart on it)
_FATAL_MARKERS = ("hiperror", "hip error", "illegal memory access", "device-side assert", "launch failure",
                  "unspecified launch", "gpu hang", "ecc error", "device lost")


class InjectedFault(RuntimeError):
    """KA_FAULT_STEP fault injection (recoverable unless `fatal`)."""


class LLMEngine:
    def __init__(self, runner: ModelRunner, tokenizer, max_batch: int = 256, max_batched_tokens: int = 8192,
                 max_model_len: int = 4096, prefix_caching: bool = True, metrics=None):
        self.runner = runner
        self.tokenizer = tokenizer
        self.bm = make_block_manager(runner.num_blocks, runner.block_size, enable_prefix_caching=prefix_caching)
        self.scheduler = Scheduler(self.bm, max_batch=max_batch, max_batched_tokens=max_batched_tokens,
                                   max_model_len=max_model_len,
                                   gather_max_s=float(os.environ.get("KA_GATHER_MAX_MS", "15")) / 1000.0,
                                   gather_quiet_s=float(os.environ.get("KA_GATHER_QUIET_MS", "1.5")) / 1000.0)
        self.metrics = metrics
        self._inbox: "queue.SimpleQueue" = queue.SimpleQueue()
        self._wake = threading.Event()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.healthy = True
        self.last_error: Optional[BaseException] = None
        self.steps = 0
        self.step_end_hooks: List[Callable[[], None]] = []   # e.g. batched IPC flush (parallel/dp.py)
        # overlapped decode: one decode step in flight while the host applies the previous one
        self.overlap = os.environ.get("KA_OVERLAP", "1") == "1"
        self._inflight = None
        # every admitted, unfinished sequence (a step that raises may hold rows that are in none of
        # the scheduler's sets yet: admitted by schedule(), added to `running` only at readback)
        self._live: Dict[int, Sequence] = {}
        self.chained_steps = 0
        self.prefill_chains = 0    # decode steps queued behind a prefill before its readback
        # steps whose batch composition changes (admissions, finished rows, chunk continuations) are
        # scheduled from a provisional advance of the in-flight step and queued before its readback
        self.lookahead = os.environ.get("KA_LOOKAHEAD", "1") == "1"
        self.lookahead_steps = 0
        # ... but not earlier than needed: requests arriving while the in-flight step runs should
        # still make it into the next one, so the lookahead waits until the in-flight step is
        # expected to end within this margin (host-side schedule + pack + first launches), from
        # running estimates of the step durations (decode: ms per step; prefill / mixed: a fixed part
        # plus ms per token)
        self.lookahead_margin_s = float(os.environ.get("KA_LOOKAHEAD_MARGIN_MS", "8")) / 1000.0
        self.lookahead_poll_s = float(os.environ.get("KA_LOOKAHEAD_POLL_US", "300")) / 1e6
        self._est_decode_s = 0.007
        self._est_tok_s = 9e-6
        self._est_fixed_s = 0.005
        self.idle_s = 0.0          # time the loop slept with no work (waiting for requests)
        self.step_t0: Optional[float] = None   # perf_counter at the start of the running step
        self.watchdog = None       # parallel/watchdog.py (TP/EP > 1, rank 0)
        self._ar_bytes_seen = 0
        self._t_done = 0.0         # perf_counter of the last step readback (step-time metric)
        # fault handling (module docstring)
        self.exit_on_fatal = os.environ.get("KA_EXIT_ON_FATAL", "0") == "1"
        self.max_recoveries = int(os.environ.get("KA_MAX_RECOVERIES_PER_MIN", "3"))
        self.recoveries = 0
        self.failures = 0
        self._recovery_times: List[float] = []
        self._exit = os._exit      # replaced in tests
        spec = os.environ.get("KA_FAULT_STEP", "")
        n, _, kind = spec.partition(":")
        self.fault_step = int(n) if n.strip() else -1
        self.fault_kind = kind or "error"

    def mark_unhealthy(self, reason: str) -> None:
        """Watchdog verdict (worker heartbeat lost / step stalled): new requests get 503.

        A lost TP worker or a stalled step is fatal: rank 0 is typically blocked inside a collective
        that only the process-group timeout (minutes) would end.  With `exit_on_fatal` (serve.py, DP
        replicas) the in-flight requests are failed (503) and the process exits with EXIT_FATAL
        right away, so its supervisor respawns the whole TP group; the clients of a DP replica also
        see its sockets close and fail whatever was routed to it."""
        self.healthy = False
        self.last_error = RuntimeError(reason)
        if not self.exit_on_fatal:
            return
        logger.critical("fatal engine fault (%s): exiting (status %d) for the supervisor to restart the engine",
                        reason, EXIT_FATAL)
        try:
            # the engine thread may be blocked mid-step: fail what is tracked and push the replies out
            # best-effort (this process ends next either way)
            self._fail_all(self.last_error)
            for hook in self.step_end_hooks:
                hook()
        except Exception:  # pragma: no cover - racing the blocked engine thread
            logger.exception("failing in-flight requests before the fatal exit")
        finally:
            self._exit(EXIT_FATAL)

    # ------------------------------------------------------------------------------------------
    def start(self) -> None:
        # The GPU loop shares the GIL with the asyncio HTTP thread; the default 5 ms switch
        # interval would let request handling delay the next kernel launch by up to 5 ms after
        # every device sync.  A short interval hands the GIL back to the engine promptly.
        sys.setswitchinterval(float(os.environ.get("KA_SWITCH_INTERVAL", "0.0002")))
        if self._thread is None:
            self._stop.clear()
            self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
            self._thread.start()
        if self.watchdog is not None and self.watchdog._thread is None:
            self.watchdog.start()

    def shutdown(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()
        self._stop.set()
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None
        try:
            self.runner.stop_workers()
        except Exception:  # pragma: no cover
            pass

    def submit(self, prompt_ids: List[int], params: SamplingParams, callback: Callable[[Sequence], None],
               forced_prefix: Optional[List[int]] = None) -> Sequence:
        seq = Sequence(prompt_ids=list(prompt_ids), params=params, callback=callback,
                       forced_prefix=list(forced_prefix or []))
        self._inbox.put(("add", seq))
        self._wake.set()
        return seq

    def abort(self, seq: Sequence) -> None:
        self._inbox.put(("abort", seq))
        self._wake.set()

    # ------------------------------------------------------------------------------------------
    def _drain_inbox(self) -> None:
        while True:
            try:
                op, seq = self._inbox.get_nowait()
            except queue.Empty:
                return
            if op == "add":
                if seq.finished:
                    continue
                try:
                    self.scheduler.add(seq)
                    self._live[seq.seq_id] = seq
                except ValueError as e:
                    self._finish(seq, SeqStatus.ABORTED, "length", error=e)
            elif op == "abort" and not seq.finished:
                self.scheduler.abort(seq)
                seq.finish_reason = "abort"
                self._live.pop(seq.seq_id, None)

    def _finish(self, seq: Sequence, status: SeqStatus, reason: str, error: Optional[BaseException] = None):
        seq.status = status
        seq.finish_reason = reason
        seq.error = error
        seq.t_finish = time.perf_counter()
        self._live.pop(seq.seq_id, None)
        if seq.block_table:
            self.bm.free_table(seq.block_table)
        if seq.callback is not None:
            try:
                seq.callback(seq)
            except Exception:  # pragma: no cover
                logger.exception("request callback failed")

    def _apply(self, batch, tokens) -> None:
        """Append sampled tokens, publish prefix blocks, finish sequences (EOS / max_new_tokens): the
        lookahead path's advance + finalize back to back."""
        self._advance(batch)
        self._settle(batch, tokens)

    def _chain(self, prev):
        """The decode step after `prev` (in flight, tokens not applied), or None when the batch
        composition could change: an admission is due, a sequence reaches max_new_tokens with
        `prev`, a sequence finished / was aborted, or KV capacity for one more token is missing.
        (An EOS sampled by `prev` is only seen at collect: that row's next token is discarded.)"""
        sch = self.scheduler
        if prev.partial or (sch.waiting and sch._should_prefill()):
            return None
        for s in prev.seqs:
            if s.finished or s.num_generated + 1 >= s.params.max_new_tokens:
                return None
        try:
            for s in prev.seqs:
                self.bm.ensure_capacity(s.block_table, s.total_len + 1)
        except Exception:
            return None
        from .scheduler import Batch
        return Batch(list(prev.seqs), [1] * len(prev.seqs), is_decode=True)

    def _finish_step(self, batch, tokens, t_launch: float) -> None:
        self._apply(batch, tokens)
        self.scheduler.on_step_done(batch)
        self.steps += 1
        m = self.metrics
        # a step's share of the pipeline: from its launch (or the previous step's completion, when it
        # was queued behind it) to its readback
        now = time.perf_counter()
        self._observe_step(batch, now - max(t_launch, self._t_done))
        if m is not None:
            m.llm_step.labels("decode" if batch.is_decode else "prefill").observe(now - max(t_launch, self._t_done))
        self._t_done = now

    def _observe_step(self, batch, dur: float) -> None:
        """Running step-duration estimates for the lookahead timing (EMA, weight 1/4)."""
        if dur <= 0:
            return
        if batch.is_decode:
            self._est_decode_s += 0.25 * (dur - self._est_decode_s)
        elif batch.num_tokens >= 256:
            per_tok = max(0.0, dur - self._est_fixed_s) / batch.num_tokens
            self._est_tok_s += 0.25 * (per_tok - self._est_tok_s)

    def step(self) -> int:
        """Run one scheduler step; returns the number of sequences processed."""
        self._drain_inbox()
        if self.fault_step >= 0 and self.steps >= self.fault_step and self.scheduler.has_work():
            kind, self.fault_step = self.fault_kind, -1   # one shot
            if kind == "exit":
                self._exit(EXIT_FATAL)
            if kind == "fatal":
                raise CollectiveTimeout("injected collective timeout (KA_FAULT_STEP)")
            raise InjectedFault("injected engine step fault (KA_FAULT_STEP)")
        if self._inflight is not None:
            prev, handle, t_prev = self._inflight
            nxt = self._chain(prev)
            if nxt is None and self.lookahead and self.runner.can_lookahead():
                n = self._lookahead_step(prev, handle, t_prev)
                self._step_metrics(prev)
                return n
            t_nxt = time.perf_counter()
            nh = self.runner.launch_decode_async(nxt, chained=True) if nxt is not None else None
            self.chained_steps += nxt is not None
            self.prefill_chains += nxt is not None and not prev.is_decode
            self._finish_step(prev, self.runner.collect(handle), t_prev)
            self._inflight = (nxt, nh, t_nxt) if nxt is not None else None
            batch = prev
        else:
            if not self.scheduler.has_work():
                return 0
            batch = self.scheduler.schedule()
            if not batch.seqs:
                return 0
            t0 = time.perf_counter()
            if self.overlap and batch.is_decode and self.runner.can_overlap(len(batch.seqs)):
                self._inflight = (batch, self.runner.launch_decode_async(batch), t0)
                return len(batch.seqs)
            if (self.overlap and not batch.is_decode and self.runner.can_overlap_prefill(len(batch.seqs))
                    and (self.lookahead or len(batch.prefill_seqs) == len(batch.seqs))):
                # a prefill / mixed step is queued and left in flight: the next call queues the step
                # after it (a decode chain of the same rows, or a lookahead step) before reading it back
                self._inflight = (batch, self.runner.launch_prefill_async(batch), t0)
                return len(batch.seqs)
            self._finish_step(batch, self.runner.execute(batch), t0)
        self._step_metrics(batch)
        return len(batch.seqs)

    def _step_metrics(self, batch) -> None:
        m = self.metrics
        if m is not None:
            m.llm_batch_size.set(len(batch.seqs))
            m.llm_queue_depth.set(len(self.scheduler.waiting))
            m.llm_kv_blocks_used.set(self.bm.num_used)
            timer = getattr(self.runner.comm, "timer", None)
            if timer is not None and hasattr(m, "rccl_allreduce"):
                for sec in timer.drain():
                    m.rccl_allreduce.observe(sec)
                nbytes = self.runner.comm.allreduce_bytes
                if nbytes > self._ar_bytes_seen:
                    m.rccl_allreduce_bytes.inc(nbytes - self._ar_bytes_seen)
                    self._ar_bytes_seen = nbytes

    # ---- applying a step: advance (at launch for lookahead, at readback otherwise), then settle ----
    def _advance(self, batch) -> None:
        """Move `batch`'s sequences past its step: KV counts advance and every sampling row gets a
        PLACEHOLDER token (the sampled value is filled in by `_settle`)."""
        partial = batch.partial
        for row, (s, nq) in enumerate(zip(batch.seqs, batch.num_query)):
            if s.finished:
                continue
            s.num_computed += nq
            if id(s) in partial:
                continue
            s.output_ids.append(PLACEHOLDER)
            s.ph_row = row

    def _settle(self, batch, tokens) -> None:
        """Placeholders of an advanced `batch` get their sampled tokens; prefix blocks are published;
        EOS / max_new_tokens finish sequences (a row a lookahead step computed for a sequence
        finished here is discarded at that step's own readback)."""
        now = time.perf_counter()
        m = self.metrics
        prefill = {id(s) for s in batch.prefill_seqs}
        for s, tok in zip(batch.seqs, tokens):
            if s.finished:
                continue
            if id(s) in batch.partial:   # a chunk of a long prompt: its KV is cached, nothing sampled
                self.bm.register_computed(s.block_table, s.all_ids[:s.num_computed], s.block_hashes)
                continue
            if s.ph_row is None:   # not advanced (finished before the advance)
                continue
            s.output_ids[-1] = int(tok)
            s.ph_row = None
            if id(s) in prefill:
                self.bm.register_computed(s.block_table, s.all_ids[:s.num_computed], s.block_hashes)
                if s.t_first_token is None:
                    s.t_first_token = now
                    if m is not None:
                        m.llm_ttft.observe(now - s.t_arrival)
                        m.llm_queue_wait.observe((s.t_scheduled or now) - s.t_arrival)
            eos = (not s.params.ignore_eos) and self.tokenizer.is_eos(int(tok))
            if eos or s.num_generated >= s.params.max_new_tokens:
                if m is not None and s.t_first_token is not None and s.num_generated > 1:
                    m.llm_tpot.observe((now - s.t_first_token) / (s.num_generated - 1))
                self._finish(s, SeqStatus.FINISHED, "stop" if eos else "length")

    # ---- lookahead: the next step scheduled and queued before the in-flight one is read back ----
    def _provisional(self, batch) -> None:
        """Advance the in-flight `batch` as if it had been read back (its tokens are still on the
        device: the next step's inputs take them from there) and update the scheduler's sets."""
        self._advance(batch)
        self.scheduler.on_step_done(batch)

    def _finalize(self, batch, tokens, t_launch: float) -> None:
        """Readback of a `_provisional` batch: settle its tokens, then the step accounting."""
        self._settle(batch, tokens)
        self.scheduler.drop_finished()
        self.steps += 1
        now = time.perf_counter()
        self._observe_step(batch, now - max(t_launch, self._t_done))
        if self.metrics is not None:
            self.metrics.llm_step.labels("decode" if batch.is_decode else "prefill").observe(
                now - max(t_launch, self._t_done))
        self._t_done = now

    def _lookahead_step(self, prev, handle, t_prev: float) -> int:
        """The in-flight `prev` cannot be followed by a same-rows decode chain: advance it
        provisionally, schedule the next step from that state, queue it (its placeholder inputs
        fixed up on the device), then read `prev` back and finalize it.  A step that cannot be queued
        early (a decode batch above the largest graph bucket, ...) runs after the readback."""
        start = max(t_prev, self._t_done)   # the device starts `prev` when the step before it is done
        est = (self._est_decode_s if prev.is_decode
               else self._est_fixed_s + self._est_tok_s * max(1, prev.num_tokens))
        until = start + est - self.lookahead_margin_s
        ev = handle.event
        if handle.progress is not None:
            # an eager step marks its progress a few layers before its end: wait for that instead of
            # the estimate (step sizes vary too much for one)
            if self.lookahead_poll_s > 0:
                while not handle.progress.query() and not ev.query():
                    time.sleep(self.lookahead_poll_s)
            else:
                handle.progress.synchronize()
            until = 0.0
        # arrivals meanwhile queue in the inbox and join the next step; stop waiting as soon as `prev`
        # is done on the device (an estimate that runs long must not leave the GPU idle)
        while ev is not None and time.perf_counter() < until and not ev.query():
            time.sleep(min(0.0005, max(0.0, until - time.perf_counter())))
        self._drain_inbox()
        self._provisional(prev)
        batch, nh, t_nxt = None, None, 0.0
        if self.scheduler.has_work():
            self.scheduler.lookahead = True
            try:
                batch = self.scheduler.schedule()
            finally:
                self.scheduler.lookahead = False
            if batch.seqs:
                t_nxt = time.perf_counter()
                if batch.is_decode:
                    if self.runner.can_overlap(len(batch.seqs)):
                        fix = [(i, s.ph_row) for i, s in enumerate(batch.seqs) if s.ph_row is not None]
                        nh = self.runner.launch_decode_async(batch, fix=fix)
                elif self.runner.can_overlap_prefill(len(batch.seqs)):
                    nh = self.runner.launch_prefill_async(batch)
                self.lookahead_steps += nh is not None
        self._finalize(prev, self.runner.collect(handle), t_prev)
        if nh is not None:
            self._inflight = (batch, nh, t_nxt)
        else:
            self._inflight = None
            if batch is not None and batch.seqs:   # placeholders are real now: run it synchronously
                # rows whose sequence `prev` just finished (EOS) were scheduled from the provisional
                # state; `_finish` freed their block tables, so they must not reach the runner
                batch = self._without_finished(batch)
                if batch.seqs:
                    self._finish_step(batch, self.runner.execute(batch), t_nxt)
                else:
                    self.scheduler.on_step_done(batch)
        return len(prev.seqs)

    @staticmethod
    def _without_finished(batch):
        """`batch` minus the rows of finished sequences (same row order; chunk ids, block copies and the
        step kind kept: copies only belong to newly admitted rows, which cannot have finished)."""
        if not any(s.finished for s in batch.seqs):
            return batch
        from .scheduler import Batch
        keep = [(s, nq) for s, nq in zip(batch.seqs, batch.num_query) if not s.finished]
        return Batch([s for s, _ in keep], [nq for _, nq in keep], is_decode=batch.is_decode,
                     prefill_seqs=[s for s in batch.prefill_seqs if not s.finished], copies=list(batch.copies),
                     partial=batch.partial)

    def is_fatal(self, err: BaseException) -> bool:
        if isinstance(err, CollectiveTimeout) or self.runner.tp_size > 1:
            return True   # a TP group cannot be resynchronised from inside one rank
        msg = repr(err).lower()
        return any(m in msg for m in _FATAL_MARKERS)

    def _recover(self, err: BaseException) -> bool:
        """After `_fail_all`: drop transient state and serve again, unless the fault is fatal or
        recoveries come too often.  Returns whether the engine is healthy again."""
        now = time.monotonic()
        self._recovery_times = [t for t in self._recovery_times if now - t < 60.0]
        if self.is_fatal(err) or len(self._recovery_times) >= self.max_recoveries:
            return False
        try:
            self._inflight = None
            self.bm.reset_prefix_cache()    # a failed step may have left partly written KV behind
            self.runner.health_check()
        except Exception as e2:  # the device itself is gone
            logger.error("engine recovery failed: %r", e2)
            self.last_error = e2
            return False
        self._recovery_times.append(now)
        self.recoveries += 1
        self.healthy = True
        logger.warning("engine recovered from %r (recovery %d)", err, self.recoveries)
        return True

    def _fail_all(self, err: BaseException) -> None:
        self._inflight = None
        sch = self.scheduler
        seqs = list(sch.running) + list(sch.prefilling) + list(sch.waiting) + list(self._live.values())
        sch.running.clear()
        sch.prefilling.clear()
        sch.waiting.clear()
        self._live.clear()
        seen = set()
        for s in seqs:
            if not s.finished and s.seq_id not in seen:
                seen.add(s.seq_id)
                self._finish(s, SeqStatus.ABORTED, "error", error=err)

    def _loop(self) -> None:
        prof_path = os.environ.get("KA_PROFILE_ENGINE")
        if prof_path:  # cProfile of the engine thread (diagnostics only)
            import cProfile
            import pstats
            prof = cProfile.Profile()
            prof.enable()
            try:
                self._loop_body()
            finally:
                prof.disable()
                with open(prof_path, "w") as f:
                    pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(60)
            return
        self._loop_body()

    def _torch_profile_hook(self):
        """KA_TORCH_PROFILE=<trace.json>[:<steps>]: torch.profiler (CPU + GPU activities) over the
        first <steps> busy engine steps (default 50), exported as a Chrome trace."""
        spec = os.environ.get("KA_TORCH_PROFILE")
        if not spec:
            return None
        path, _, steps = spec.partition(":")
        import torch
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        prof = torch.profiler.profile(activities=acts)
        prof.start()
        state = {"left": int(steps or 50), "prof": prof}

        def on_step(n: int) -> None:
            if state["prof"] is None or n == 0:
                return
            state["left"] -= 1
            if state["left"] <= 0:
                state["prof"].stop()
                state["prof"].export_chrome_trace(path)
                state["prof"] = None
        return on_step

    def _loop_body(self) -> None:
        tprof = self._torch_profile_hook()
        while not self._stop.is_set():
            try:
                self.step_t0 = time.perf_counter()
                n = self.step()
                self.step_t0 = None
                if tprof is not None:
                    tprof(n)
            except Exception as e:  # engine fault: fail in-flight requests, then recover or stop
                logger.exception("engine step failed")
                self.step_t0 = None
                self.healthy = False
                self.last_error = e
                self.failures += 1
                self._fail_all(e)
                if not self._recover(e):
                    logger.critical("unrecoverable engine fault: %r", e)
                    if self.exit_on_fatal:
                        logger.critical("exiting (status %d) for the supervisor to restart the engine", EXIT_FATAL)
                        self._exit(EXIT_FATAL)
                n = 0
            for hook in self.step_end_hooks:
                hook()
            if n == 0 and not self.scheduler.has_work():
                t_idle = time.perf_counter()
                self._wake.wait(timeout=0.05)
                self._wake.clear()
                self.idle_s += time.perf_counter() - t_idle
            elif n == 0 and self.scheduler.gathering():   # let the arriving burst in (no busy spin)
                t_idle = time.perf_counter()
                self._wake.wait(timeout=self.scheduler.gather_quiet_s)
                self._wake.clear()
                self.idle_s += time.perf_counter() - t_idle
        if self._inflight is not None:   # stopping with a step in flight: finish it cleanly
            prev, handle, t_prev = self._inflight
            self._inflight = None
            try:
                self._finish_step(prev, self.runner.collect(handle), t_prev)
            except Exception:  # pragma: no cover
                logger.exception("in-flight step failed at shutdown")

    # ------------------------------------------------------------------------------------------
    def generate_blocking(self, prompt_ids_list: List[List[int]], params: SamplingParams,
                          forced_prefix: Optional[List[int]] = None) -> List[Sequence]:
        """Synchronous batch generation on the caller's thread (tests, benchmarks)."""
        seqs = [Sequence(prompt_ids=list(p), params=params, forced_prefix=list(forced_prefix or []))
                for p in prompt_ids_list]
        for s in seqs:
            self.scheduler.add(s)
        gather, self.scheduler.gather_max_s = self.scheduler.gather_max_s, 0.0   # everything is here
        try:
            while any(not s.finished for s in seqs):
                batch = self.scheduler.schedule()
                if not batch.seqs:
                    raise RuntimeError("scheduler produced an empty batch (out of KV blocks?)")
                tokens = self.runner.execute(batch)
                self._apply(batch, tokens)
                self.scheduler.on_step_done(batch)
        finally:
            self.scheduler.gather_max_s = gather
        return seqs
