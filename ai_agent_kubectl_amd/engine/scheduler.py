"""Continuous-batching scheduler.

Each engine step runs ONE forward over a batch:
* a prefill step when requests are waiting and KV blocks are available: as many waiting
  sequences as fit the token budget (`MAX_NUM_BATCHED_TOKENS`) and the batch limit, with their
  prefix-cache hits skipped (only the uncached tail of each prompt is computed), plus — so that
  running sequences do not stall behind arrivals — every running sequence's next decode token
  (a mixed varlen step; decode rows are one-token queries in the same paged prefill kernel);
* otherwise a decode step over all running sequences (hipGraph replay in the runner).

New sequences join the running set the step after their prefill; finished sequences leave
immediately and free their blocks, so the batch composition changes every step.

Chunked prefill: a prompt whose uncached tail exceeds the step's token budget is
prefilled in budget-sized chunks over consecutive mixed steps (`prefilling`), so a long context
(up to MAX_MODEL_LEN = 8192) neither blows the step's activation size nor stalls the running
decodes for a whole 8k-token forward.  A chunk row samples nothing; the row that computes the last
prompt token samples the first output token as usual.
"""
from __future__ import annotations

import collections
import os
import time
from dataclasses import dataclass, field
from typing import Deque, List, Optional

from .block_manager import BlockManager, NoFreeBlocks
from .sequence import Sequence, SeqStatus


@dataclass
class Batch:
    seqs: List[Sequence]
    num_query: List[int]                 # tokens computed this step per sequence
    is_decode: bool
    prefill_seqs: List[Sequence] = field(default_factory=list)
    copies: List[tuple] = field(default_factory=list)     # (src, dst) KV block copies before the step
    partial: frozenset = frozenset()     # id() of chunk rows: prompt not finished, nothing sampled

    @property
    def num_tokens(self) -> int:
        return sum(self.num_query)


class Scheduler:
    def __init__(self, block_manager: BlockManager, max_batch: int = 256, max_batched_tokens: int = 8192,
                 max_model_len: int = 4096, mix_decode_into_prefill: bool = True,
                 prefill_max_wait_s: Optional[float] = None, prefill_min_frac: Optional[float] = None,
                 partial_block_reuse: bool = True, gather_max_s: float = 0.0, gather_quiet_s: float = 0.0015,
                 hold_steps: Optional[int] = None, hold_max_s: Optional[float] = None,
                 chunked_prefill: Optional[bool] = None, min_chunk: int = 256):
        # Prefill batching under continuous arrivals: a prefill step is an eager (non-graph) step,
        # so while sequences are decoding, new arrivals are admitted together — when at least
        # max(4, prefill_min_frac * running) are waiting or the oldest has waited
        # prefill_max_wait_s — instead of turning every decode step into a mixed eager step.
        if prefill_max_wait_s is None:
            prefill_max_wait_s = float(os.environ.get("KA_PREFILL_MAX_WAIT_MS", "15")) / 1000.0
        if prefill_min_frac is None:
            prefill_min_frac = float(os.environ.get("KA_PREFILL_MIN_FRAC", "0.25"))
        self.prefill_max_wait_s = prefill_max_wait_s
        self.prefill_min_frac = prefill_min_frac
        # idle engine + a burst still arriving (the replies of a finished wave turn into new
        # requests over a few ms): gather while the newest arrival is younger than gather_quiet_s,
        # for at most gather_max_s, so the burst is prefilled as one large step instead of a
        # small, GEMM-inefficient first step followed by the rest
        self.gather_max_s = gather_max_s
        self.gather_quiet_s = gather_quiet_s
        self._idle_since = 0.0     # when the running set last became empty
        self._drained = 0          # sequences that left in the step that emptied the running set
        # after a large wave drains, its clients' next requests come back as a burst spread over
        # the API process's turnaround (~10 ms for 256 requests): a longer quiet gap keeps them in
        # one prefill; a lone request to an idle engine still waits only gather_quiet_s
        self.burst_quiet_s = float(os.environ.get("KA_GATHER_BURST_QUIET_MS", "4")) / 1000.0
        self.burst_min = int(os.environ.get("KA_GATHER_BURST_MIN", "32"))
        # Wave merging: arrivals that find every running sequence within `hold_steps` decode steps
        # of its token limit wait for that batch to drain (then gather with its clients' next
        # requests) instead of starting a second, half-size prefill wave beside it.  Two offset
        # waves cost a whole extra prefill step per cycle: at 256 requests of ~31 new tokens two
        # ~4k-token steps take 2 x 58 ms against 96 ms for one 8k-token step
        # (profiles/phase_profile_c256.txt).  Bounded by hold_max_s of waiting.  Off by default: with
        # EOS-terminated variable-length outputs and with open-loop arrivals it measured no better than
        # off (1158 vs 1135 req/s closed loop, p50 200 vs 209 ms open loop: profiles/r2/sched/).
        if hold_steps is None:
            hold_steps = int(os.environ.get("KA_PREFILL_HOLD_STEPS", "0"))
        if hold_max_s is None:
            hold_max_s = float(os.environ.get("KA_PREFILL_HOLD_MAX_MS", "100")) / 1000.0
        self.hold_steps = hold_steps
        self.hold_max_s = hold_max_s
        self.bm = block_manager
        self.max_batch = max_batch
        self.max_batched_tokens = max_batched_tokens
        self.max_model_len = max_model_len
        self.mix = mix_decode_into_prefill
        self.partial_reuse = partial_block_reuse and hasattr(block_manager, "reuse_partial")
        self.waiting: Deque[Sequence] = collections.deque()
        self.running: List[Sequence] = []
        if chunked_prefill is None:
            chunked_prefill = os.environ.get("KA_CHUNKED_PREFILL", "1") == "1"
        self.chunked = chunked_prefill
        self.min_chunk = min_chunk          # a later row is chunked only if this much budget is left
        self.prefilling: List[Sequence] = []   # admitted, prompt partially computed (chunked)
        # scheduling ahead of an in-flight step (engine._lookahead_step): sequences were advanced
        # provisionally, so no preemption (a victim's placeholder token would be re-prefilled)
        self.lookahead = False

    def add(self, seq: Sequence) -> None:
        if seq.total_len + seq.params.max_new_tokens > self.max_model_len:
            raise ValueError(f"prompt ({len(seq.prompt_ids)}) + max_new_tokens exceeds max_model_len "
                             f"{self.max_model_len}")
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self.prefilling)

    def abort(self, seq: Sequence) -> None:
        if seq in self.waiting:
            self.waiting.remove(seq)
        if seq in self.running:
            self.running.remove(seq)
        if seq in self.prefilling:
            self.prefilling.remove(seq)
        self.bm.free_table(seq.block_table)
        seq.status = SeqStatus.ABORTED

    # ------------------------------------------------------------------------------------------
    def _admit(self, copies: List[tuple]):
        """-> (rows, query lengths, partial ids): the chunked prompts first, then new arrivals."""
        admitted: List[Sequence] = []
        nqs: List[int] = []
        partial = set()
        budget = self.max_batched_tokens - (self._n_active() if self.mix else 0)
        for seq in self.prefilling:   # continue the chunked prompts (oldest first)
            rem = seq.total_len - seq.num_computed
            c = min(rem, budget)
            if c <= 0:
                break
            admitted.append(seq)
            nqs.append(c)
            if c < rem:
                partial.add(id(seq))
            budget -= c
        n_busy = self._n_active() + len(self.prefilling)
        n_cont = len(admitted)     # continued chunk rows are already counted in n_busy
        while self.waiting and budget > 0 and n_busy + len(admitted) - n_cont < self.max_batch:
            seq = self.waiting[0]
            try:
                table, cached, hashes = self.bm.allocate_prompt(seq.all_ids)
            except NoFreeBlocks:
                break
            part = self.bm.reuse_partial(table, seq.all_ids, cached, hashes) if self.partial_reuse else None
            q = seq.total_len - cached - (part[1] if part else 0)
            c = q
            if q > budget:
                if admitted and not (self.chunked and budget >= self.min_chunk):
                    if part:
                        self.bm.unpin(part[0])
                    self.bm.free_table(table)
                    break
                if self.chunked:
                    c = budget
            if part:   # sub-block reuse: copy the sibling's KV rows, skip its first r tokens
                copies.append((part[0], table[cached // self.bm.block_size]))
                cached += part[1]
            self.waiting.popleft()
            seq.block_table, seq.block_hashes = table, hashes
            seq.num_computed = cached
            seq.num_cached_prompt = cached
            seq.status = SeqStatus.RUNNING
            if seq.t_scheduled is None:
                seq.t_scheduled = time.perf_counter()
            admitted.append(seq)
            nqs.append(c)
            if c < q:
                partial.add(id(seq))
            budget -= c
        return admitted, nqs, partial

    def _n_active(self) -> int:
        """Running sequences still generating (a provisionally advanced one may already hold its
        last token, to be finished when that step is read back)."""
        return sum(1 for s in self.running if s.num_generated < s.params.max_new_tokens)

    def drop_finished(self) -> None:
        before = len(self.running)
        self.running = [s for s in self.running if not s.finished]
        if not self.running and before:
            self._idle_since = time.perf_counter()
            self._drained = before

    def gathering(self) -> bool:
        """Idle engine, requests still streaming in: hold the admission for a moment.  The window
        opens at the later of the first waiting arrival and the moment the engine went idle (held
        requests wait for the drained batch's clients to come back); it closes after a quiet gap of
        gather_quiet_s once something has arrived since then, or after gather_max_s."""
        if self.running or not self.waiting or self.gather_max_s <= 0 or len(self.waiting) >= self.max_batch:
            return False
        now = time.perf_counter()
        newest = self.waiting[-1].t_arrival
        # a large batch just drained (its clients' next requests are on their way): gather for up to
        # gather_max_s; otherwise (steady arrivals into an idle engine) only for two quiet gaps, so an
        # open-loop stream is not held back (profiles/r2/sched: p50 +10 ms at 900 req/s otherwise)
        burst = self._drained >= self.burst_min and newest - self._idle_since < self.gather_max_s
        if burst and len(self.waiting) >= self._drained:
            return False      # as many requests are back as just finished: the whole wave is here
        cap = self.gather_max_s if burst else min(self.gather_max_s, 2 * self.gather_quiet_s)
        if now - max(self.waiting[0].t_arrival, self._idle_since) >= cap:
            return False
        if newest < self._idle_since:
            return True
        quiet = max(self.gather_quiet_s, self.burst_quiet_s) if burst else self.gather_quiet_s
        return now - newest < quiet

    def _holding(self) -> bool:
        if self.hold_steps <= 0 or len(self.running) + len(self.waiting) > self.max_batch:
            return False
        if time.perf_counter() - self.waiting[0].t_arrival >= self.hold_max_s:
            return False
        left = max(s.params.max_new_tokens - s.num_generated for s in self.running)
        return left <= self.hold_steps

    def _should_prefill(self) -> bool:
        if self.prefilling:   # a chunked prompt continues every step
            return True
        if not self.waiting:
            return False
        if not self.running:
            return not self.gathering()
        if self._n_active() >= self.max_batch:
            return False
        if self._holding():
            return False
        if len(self.waiting) >= max(4, int(self.prefill_min_frac * len(self.running))):
            return True
        return time.perf_counter() - self.waiting[0].t_arrival >= self.prefill_max_wait_s

    def schedule(self) -> Batch:
        copies: List[tuple] = []
        admitted, nqs, partial = self._admit(copies) if self._should_prefill() else ([], [], set())
        # decode rows need a slot for their next token
        decodes: List[Sequence] = []
        if not admitted or self.mix:
            for seq in list(self.running):
                if seq.status is not SeqStatus.RUNNING:
                    continue  # preempted below while serving an earlier row
                if seq.num_generated >= seq.params.max_new_tokens:
                    continue  # holds its last token (provisional): finished at that step's readback
                ok = True
                while True:
                    try:
                        self.bm.ensure_capacity(seq.block_table, seq.total_len)
                        break
                    except NoFreeBlocks:
                        if self.lookahead:   # no preemption ahead of a readback: skip the row this step
                            ok = False
                            break
                        # preempt the newest running sequence (recomputed when re-admitted)
                        victim = self.running[-1]
                        self._preempt(victim)
                        if victim in decodes:
                            decodes.remove(victim)
                        if victim is seq:
                            break
                if ok and seq.status is SeqStatus.RUNNING:
                    decodes.append(seq)
        if admitted:
            seqs = decodes + admitted
            nq = [1] * len(decodes) + nqs
            return Batch(seqs, nq, is_decode=False, prefill_seqs=admitted, copies=copies,
                         partial=frozenset(partial))
        return Batch(decodes, [1] * len(decodes), is_decode=True)

    def _preempt(self, seq: Sequence) -> None:
        """Recompute-style preemption: drop the KV, requeue; re-admission prefills all_ids."""
        self.running.remove(seq)
        self.bm.free_table(seq.block_table)
        seq.block_hashes = []
        seq.num_computed = 0
        seq.status = SeqStatus.WAITING
        self.waiting.appendleft(seq)

    def on_step_done(self, batch: Batch) -> None:
        for src, _ in batch.copies:   # the copy is enqueued before the step's kernels: release the pin
            self.bm.unpin(src)
        for s in batch.prefill_seqs:
            chunk = id(s) in batch.partial
            if s.finished or not chunk:
                if s in self.prefilling:
                    self.prefilling.remove(s)
                if not s.finished:
                    self.running.append(s)
            elif s not in self.prefilling:
                self.prefilling.append(s)
        self.drop_finished()
