"""Request / sequence state shared by the scheduler, the runner and the engine loop."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

_ids = itertools.count()

# token id of an output whose value is still on the device: a step scheduled while the previous
# one is in flight (engine._lookahead_step) appends it; the readback replaces it, and until then the
# next step's packed inputs take that token from the device (runner fixups)
PLACEHOLDER = -1


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2
    ABORTED = 3


@dataclass
class SamplingParams:
    max_new_tokens: int = 24
    ignore_eos: bool = False
    safe_decode: bool = True      # SAFE_DECODE token mask (engine/safe_decode.py)


@dataclass(eq=False)   # identity semantics: `seq in list` / `remove` must not compare token lists
class Sequence:
    prompt_ids: List[int]
    params: SamplingParams
    callback: Optional[Callable[["Sequence"], None]] = None
    forced_prefix: List[int] = field(default_factory=list)   # jump-forward tokens (counted as output)
    seq_id: int = field(default_factory=lambda: next(_ids))
    status: SeqStatus = SeqStatus.WAITING
    output_ids: List[int] = field(default_factory=list)
    block_table: List[int] = field(default_factory=list)
    block_hashes: List[int] = field(default_factory=list)
    num_computed: int = 0           # tokens whose KV is in the cache
    num_cached_prompt: int = 0      # prompt tokens served by the prefix cache
    n_forced: int = 0
    finish_reason: Optional[str] = None
    error: Optional[BaseException] = None
    t_arrival: float = field(default_factory=time.perf_counter)
    t_scheduled: Optional[float] = None     # first admission into a prefill step (queue wait ends)
    t_first_token: Optional[float] = None
    t_finish: Optional[float] = None
    ph_row: Optional[int] = None            # row of the in-flight step whose token is the PLACEHOLDER

    def __post_init__(self):
        self.n_forced = len(self.forced_prefix)
        if self.forced_prefix:
            # jump-forward: deterministic constrained tokens are appended to the prompt and also
            # reported as the first output tokens (equivalent to decoding them under the mask).
            self.prompt_ids = list(self.prompt_ids) + list(self.forced_prefix)
            self.output_ids = list(self.forced_prefix)

    @property
    def generated(self) -> List[int]:
        return self.output_ids[self.n_forced:]

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids[self.n_forced:]

    @property
    def total_len(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids) - self.n_forced

    @property
    def num_generated(self) -> int:
        """Tokens produced by the model (excluding the jump-forward prefix)."""
        return len(self.output_ids) - self.n_forced

    @property
    def finished(self) -> bool:
        return self.status in (SeqStatus.FINISHED, SeqStatus.ABORTED)
