"""Async, shell-free `kubectl` execution and output parsing.

Parity with `execute_command_async` (`/root/reference/app.py:205-281`):

* `shlex.split` the command, require `args[0] == "kubectl"`, spawn it with
  `asyncio.create_subprocess_exec` (never a shell), wait at most `EXECUTION_TIMEOUT` seconds;
* rc == 0: multi-line stdout becomes `{"type":"table","data":[{header.lower(): value, ...}]}` by
  whitespace splitting (quirk Q6: misaligned for multi-word cells, preserved), single-line stdout
  `{"type":"raw","data": stdout}`;
* rc != 0: `execution_error={"type":"kubectl_error","code":str(rc),"message":stderr}` and the
  metadata gains `error_type`/`error_code`;
* timeout -> terminate + wait <= 2 s.

Quirk Q1: on timeout / missing binary / bad command / unexpected error the reference
returns a dict *without* `metadata`, which makes the route crash with a plain-text 500.  By
default this build returns a structured error with real metadata (HTTP 200); set
`COMPAT_STRICT_500=1` to get the reference's exact dicts (and hence its 500).
"""
from __future__ import annotations

import asyncio
import datetime
import logging
import os
import shlex
import signal
import sys
import time
from typing import Any, Dict, List

logger = logging.getLogger("app")


if sys.version_info < (3, 12):
    def utcnow_iso() -> str:
        """`datetime.datetime.utcnow().isoformat()` (naive, no `Z`; quirk Q7) — twice per request."""
        return datetime.datetime.utcnow().isoformat()
else:  # utcnow() is deprecated from 3.12: same value through an aware datetime
    def utcnow_iso() -> str:
        """`datetime.datetime.utcnow().isoformat()` (naive, no `Z`; quirk Q7) without the deprecation."""
        return datetime.datetime.now(datetime.timezone.utc).replace(tzinfo=None).isoformat()


def parse_kubectl_output(stdout: str) -> Dict[str, Any]:
    """app.py:236-249 — whitespace table parse for multi-line output, raw otherwise."""
    try:
        if "\n" in stdout:
            lines = stdout.splitlines()
            headers = [h.lower() for h in lines[0].split()]
            items: List[Dict[str, str]] = []
            for line in lines[1:]:
                items.append(dict(zip(headers, line.split())))
            return {"type": "table", "data": items}
        return {"type": "raw", "data": stdout}
    except Exception as parse_err:  # pragma: no cover - mirrors app.py:245-247
        logger.warning(f"Failed to parse kubectl output: {parse_err}")
        return {"type": "raw", "data": stdout}


def _error_result(kind: str, message: str, start_iso: str, start_ts: float, strict: bool) -> Dict[str, Any]:
    if strict:
        return {"execution_error": message}
    return {
        "execution_error": {"type": kind, "message": message},
        "metadata": {
            "start_time": start_iso,
            "end_time": utcnow_iso(),
            "duration_ms": (time.time() - start_ts) * 1000,
            "success": False,
            "error_type": kind,
            "error_code": None,
        },
    }


def _signal_group(process, sig) -> None:
    """Signal the child's process group (it was started in its own session)."""
    try:
        os.killpg(process.pid, sig)
    except ProcessLookupError:
        pass


async def execute_command_async(command: str, timeout: float, kubectl_bin: str = "kubectl",
                                strict_compat: bool = False) -> Dict[str, Any]:
    start_time = utcnow_iso()
    start_ts = time.time()
    logger.info(f"Attempting to execute command: {command}")
    process = None
    try:
        args = shlex.split(command)
        if not args or args[0] != "kubectl":
            raise ValueError("invalid_command", "Command does not start with kubectl")
        if kubectl_bin != "kubectl":
            args[0] = kubectl_bin
        # own process group: a timeout stops kubectl's children too (exec credential plugins),
        # which would otherwise keep the pipes open after kubectl itself is gone
        process = await asyncio.create_subprocess_exec(
            *args, stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE, start_new_session=True)
        stdout, stderr = await asyncio.wait_for(process.communicate(), timeout=timeout)
        end_ts = time.time()
        metadata = {
            "start_time": start_time,
            "end_time": utcnow_iso(),
            "duration_ms": (end_ts - start_ts) * 1000,
            "success": process.returncode == 0,
        }
        result: Dict[str, Any] = {"metadata": metadata}
        if process.returncode == 0:
            out = stdout.decode().strip()
            logger.info(f"Command executed successfully. Output:\n{out}")
            result["execution_result"] = parse_kubectl_output(out)
        else:
            err = stderr.decode().strip()
            logger.error(f"Command execution failed with code {process.returncode}. Error:\n{err}")
            result["execution_error"] = {"type": "kubectl_error", "code": str(process.returncode),
                                         "message": err}
            metadata.update({"error_type": "kubectl_error", "error_code": str(process.returncode)})
        return result
    except asyncio.TimeoutError:
        logger.error(f"Command execution timed out after {timeout}s: {command}")
        # drain the pipes as well as reaping the child (communicate, not wait): the subprocess
        # transport closes only once both pipes hit EOF, else it outlives the request
        try:
            _signal_group(process, signal.SIGTERM)
            await asyncio.wait_for(process.communicate(), timeout=2)
        except Exception as kill_err:
            logger.error(f"Error terminating timed-out process: {kill_err!r}")
            try:
                _signal_group(process, signal.SIGKILL)
                await asyncio.wait_for(process.communicate(), timeout=2)
            except Exception:
                pass
        t = int(timeout) if float(timeout).is_integer() else timeout
        return _error_result("timeout", f"Command execution timed out after {t}s", start_time, start_ts,
                             strict_compat)
    except FileNotFoundError:
        logger.error("kubectl command not found. Is it installed and in PATH?")
        return _error_result("not_found", "kubectl command not found", start_time, start_ts, strict_compat)
    except ValueError as ve:
        logger.error(f"Invalid command for execution: {command} - {ve}")
        return _error_result("invalid_command", f"Invalid command format: {ve}", start_time, start_ts,
                             strict_compat)
    except Exception as e:
        logger.exception(f"Error executing command '{command}': {e}")
        return _error_result("internal", f"An unexpected error occurred during execution: {e}", start_time,
                             start_ts, strict_compat)
