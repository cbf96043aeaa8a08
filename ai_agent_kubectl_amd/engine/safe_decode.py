"""SAFE_DECODE: a token-level grammar that makes every generation pass the reference validator.

Random-init weights produce arbitrary tokens, which would fail `is_safe_kubectl_command`
(`/root/reference/app.py:72-88`) and turn every request into a 422 (SURVEY.md §7.3 hard part 1).
The grammar is enforced inside the sampler (masked greedy argmax, csrc/sampling.hip):

  state FORCED : the reply starts with the token(s) spelling "kubectl" — deterministic, so they are
                 jump-forwarded into the prefill instead of spending decode steps on them;
  state FIRST  : a token that starts with one space followed by a safe non-space character
                 (the validator needs "kubectl " + something after strip());
  state BODY   : tokens made only of safe characters, or EOS.

Safe characters exclude everything in the validator's blacklist (`; & | \\` $ ( ) < >`), quotes
and backslashes (so `shlex.split` always succeeds) and newlines.  The validator itself still runs
unchanged on the detokenised text (api/app.py -> safety.parse_llm_output).
"""
from __future__ import annotations

import string
from typing import List, Tuple

import numpy as np

SAFE_CHARS = set(string.ascii_letters + string.digits + " -_./:=,@%+")
MASK_FIRST = 0
MASK_BODY = 1


def _safe_text(b: bytes) -> bool:
    try:
        s = b.decode("utf-8")
    except UnicodeDecodeError:
        return False
    return len(s) > 0 and all(c in SAFE_CHARS for c in s)


def build_masks(tokenizer, allow_eos: bool = True) -> np.ndarray:
    """Return uint32 bitmasks [2, ceil(V/32)]: row MASK_FIRST and row MASK_BODY."""
    V = tokenizer.vocab_size
    first = np.zeros(V, dtype=bool)
    body = np.zeros(V, dtype=bool)
    for tid in range(V):
        b = tokenizer.id_to_bytes[tid]
        if b is None or not _safe_text(b):
            continue
        body[tid] = True
        if len(b) >= 2 and b[0:1] == b" " and b[1:2] != b" ":
            first[tid] = True
    if allow_eos:
        for e in tokenizer.eos_ids:
            body[e] = True
    words = (V + 31) // 32
    out = np.zeros((2, words), dtype=np.uint32)
    for row, m in ((MASK_FIRST, first), (MASK_BODY, body)):
        padded = np.zeros(words * 32, dtype=bool)
        padded[:V] = m
        bits = padded.reshape(words, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)
        out[row] = bits.sum(axis=1).astype(np.uint32)
    return out


def forced_prefix(tokenizer) -> List[int]:
    return tokenizer.encode("kubectl")


def mask_index_for(num_generated: int, safe: bool) -> int:
    if not safe:
        return -1
    return MASK_FIRST if num_generated == 0 else MASK_BODY
