"""Query sanitiser, kubectl command safety validator and LLM output parser.

Behavioural parity:

* `sanitize_query`        — `/root/reference/app.py:60-68`: `\\n \\r \\t` -> space, whitespace runs
  collapsed, stripped.  The result is both the cache key and the LLM input.
* `is_safe_kubectl_command` — `app.py:72-88`: after `strip()` must start with `"kubectl "`, must not
  contain any of `; && || \\` $ ( ) < >` (a single `|`, `&`, `{}`, `*` and embedded newlines pass,
  Q3), and must `shlex.split` cleanly (unbalanced quotes fail).
* `parse_llm_output`      — `app.py:95-104`: strip; if the text starts AND ends with three
  backticks remove exactly three chars from each end and strip again (so a fenced
  "```bash\\n...```" block keeps "bash" and fails the check, Q4); then validate, raising
  `UnsafeCommandError` (a `ValueError`, like the reference's parser) on failure.

The blacklist is also consumed by the engine's constrained decoder (`engine/safe_decode.py`) so
that the GPU sampler can never emit a token the validator would reject.
"""
from __future__ import annotations

import logging
import shlex

logger = logging.getLogger("app")

# app.py:79 — order kept for log parity.
UNSAFE_SUBSTRINGS = (";", "&&", "||", "`", "$", "(", ")", "<", ">")
KUBECTL_PREFIX = "kubectl "


class UnsafeCommandError(ValueError):
    """Raised when generated text fails the safety checks (maps to HTTP 422, app.py:192-194)."""


def sanitize_query(query: str) -> str:
    normalized = query.replace("\n", " ").replace("\r", " ").replace("\t", " ")
    return " ".join(normalized.split()).strip()


def is_safe_kubectl_command(command: str) -> bool:
    command = command.strip()
    if not command.startswith(KUBECTL_PREFIX):
        logger.warning(f"Generated command does not start with 'kubectl ': {command}")
        return False
    for bad in UNSAFE_SUBSTRINGS:
        if bad in command:
            logger.warning(f"Generated command contains potentially unsafe characters: {command}")
            return False
    if "'" not in command and '"' not in command and "\\" not in command:
        return True   # shlex.split raises only on an unclosed quote or a trailing escape
    try:
        shlex.split(command)
    except ValueError as e:
        logger.warning(f"Generated command failed shlex parsing: {command} - Error: {e}")
        return False
    return True


def strip_code_fence(text: str) -> str:
    command = text.strip()
    if command.startswith("```") and command.endswith("```"):
        command = command[3:-3].strip()
    return command


def parse_llm_output(text: str) -> str:
    command = strip_code_fence(text)
    if not is_safe_kubectl_command(command):
        raise UnsafeCommandError(f"Generated command failed safety checks: {command}")
    return command
