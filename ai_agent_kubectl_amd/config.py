"""Configuration: `.env` loading plus typed settings.

Parity with the reference's config block (`/root/reference/app.py:23-36`) and the env template
(`/root/reference/.env-sample:1-25`): the same variable names, the same defaults and the same
`int()` parsing.  The reference calls `python-dotenv`'s `load_dotenv()` (`app.py:24`), which is
not installed here, so `load_dotenv` below re-implements the subset of its semantics the service
depends on (python-dotenv row):

* reads `./.env` (or an explicit path); missing file is not an error;
* never overrides a variable that is already set in the process environment;
* `KEY=VALUE`, optional `export ` prefix, blank lines and `#` comment lines ignored;
* unquoted values lose a trailing ` # comment` (whitespace before `#` required) and surrounding
  whitespace — `.env-sample` relies on this for lines such as `CACHE_TTL=300      # seconds`;
* single-quoted values are literal; double-quoted values understand `\\n`, `\\t`, `\\"`, `\\\\`.

Engine settings (LLM_BACKEND, MODEL, TP, ...) follow the same env-var style.
"""
from __future__ import annotations

import dataclasses
import os
import re
from typing import Dict, Mapping, MutableMapping, Optional

_LINE = re.compile(r"^\s*(?:export\s+)?([A-Za-z_][A-Za-z0-9_.\-]*)\s*=\s*(.*)$")


def _parse_value(raw: str) -> str:
    raw = raw.strip()
    if not raw:
        return ""
    q = raw[0]
    if q in ("'", '"'):
        end = raw.find(q, 1)
        while end != -1 and q == '"' and raw[end - 1] == "\\" and not raw[:end].endswith("\\\\"):
            end = raw.find(q, end + 1)
        if end != -1:
            body = raw[1:end]
            if q == '"':
                body = (body.replace("\\\\", "\x00").replace("\\n", "\n").replace("\\t", "\t")
                        .replace('\\"', '"').replace("\x00", "\\"))
            return body
    # unquoted: strip inline comment (" #" or "\t#") then whitespace
    m = re.search(r"\s#", raw)
    if m:
        raw = raw[: m.start()]
    return raw.strip()


def parse_dotenv(text: str) -> Dict[str, str]:
    """Parse `.env` text into an ordered dict (python-dotenv compatible subset)."""
    out: Dict[str, str] = {}
    for line in text.splitlines():
        s = line.strip()
        if not s or s.startswith("#"):
            continue
        m = _LINE.match(line)
        if not m:
            continue
        out[m.group(1)] = _parse_value(m.group(2))
    return out


def load_dotenv(path: Optional[str] = None, environ: Optional[MutableMapping[str, str]] = None,
                override: bool = False) -> bool:
    """Load `path` (default `./.env`) into `environ` without overriding existing keys.

    Returns True when a file was read (python-dotenv returns True if at least one var was set;
    here: file existed), mirroring `load_dotenv()` at `app.py:24`.
    """
    environ = os.environ if environ is None else environ
    path = path or os.path.join(os.getcwd(), ".env")
    if not os.path.isfile(path):
        return False
    with open(path, "r", encoding="utf-8") as f:
        values = parse_dotenv(f.read())
    for k, v in values.items():
        if override or k not in environ:
            environ[k] = v
    return True


@dataclasses.dataclass
class Settings:
    """All service + engine knobs.  Field defaults = reference defaults (`app.py:27-36`)."""

    # --- reference variables (app.py:27-36, 394-395) ---
    API_AUTH_KEY: Optional[str] = None
    CACHE_MAXSIZE: int = 100
    CACHE_TTL: int = 300
    LLM_TIMEOUT: int = 60
    EXECUTION_TIMEOUT: int = 30
    RATE_LIMIT: str = "10/minute"
    LOG_LEVEL: str = "INFO"
    OPENAI_API_KEY: Optional[str] = None
    OPENAI_MODEL: str = "gpt-3.5-turbo"
    OPENAI_BASE_URL: Optional[str] = None
    PORT: int = 8000
    HOST: str = "0.0.0.0"

    # --- behaviour flags ---
    COMPAT_STRICT_500: bool = False      # reproduce app.py:388 KeyError -> 500 text/plain
    KUBECTL_BIN: str = "kubectl"         # executable looked up on PATH (app.py:216)
    API_FAST_PATH: bool = True           # pure-ASGI fast path for valid POSTs (api/app.py)

    # --- LLM backend selection ---
    LLM_BACKEND: str = "stub"            # stub | engine | openai
    MODEL: str = "llama3-8b"             # llama3-8b | llama3-70b | mixtral-8x7b | tiny-llama | tiny-mixtral
    WEIGHTS: str = "random:0"            # safetensors dir/file or random:<seed>
    TP: int = 1
    DP: int = 1
    ENGINE_PROCESS: bool = True          # run the engine (a TP group) in its own process(es): the API keeps its GIL
    EP: int = 1
    MAX_BATCH: int = 256
    MAX_NEW_TOKENS: int = 24
    KV_BLOCK_SIZE: int = 16
    GPU_MEM_FRACTION: float = 0.90
    HIPGRAPH_BUCKETS: str = "1,2,4,8,16,32,48,64,96,128,192,256"
    SAFE_DECODE: bool = True
    IGNORE_EOS: bool = False
    PREFIX_CACHING: bool = True
    MAX_NUM_BATCHED_TOKENS: int = 0     # 0: per model (ModelConfig.default_step_tokens)
    FAULT_LLM_DELAY_MS: int = 0
    FAULT_LLM_ERROR: str = ""
    # --- multi-worker HTTP tier (serve.py) ---
    WORKERS: int = 1                     # API worker processes sharing the port (SO_REUSEPORT)
    SHARED_STATE: str = ""               # shared-memory segment name for the cache + limiter ("" = process-local)
    ENGINE_DEVICES: str = ""             # DP replica devices, e.g. "cuda:0,cuda:1" or "cpu,cpu" ("" = cuda:0..DP-1)

    @property
    def log_level(self) -> str:
        return self.LOG_LEVEL.upper()

    @classmethod
    def from_env(cls, environ: Optional[Mapping[str, str]] = None, dotenv: bool = True,
                 dotenv_path: Optional[str] = None) -> "Settings":
        """Build settings from the environment (after `load_dotenv`, as app.py:24-36 does).

        Integers go through plain `int()` like the reference, so a malformed value raises at
        start-up exactly where the reference would crash at import.
        """
        if environ is None:
            if dotenv:
                load_dotenv(dotenv_path)
            environ = os.environ
        kw = {}
        for f in dataclasses.fields(cls):
            if f.name not in environ:
                continue
            raw = environ[f.name]
            if f.type in ("int", int):
                kw[f.name] = int(raw)
            elif f.type in ("float", float):
                kw[f.name] = float(raw)
            elif f.type in ("bool", bool):
                kw[f.name] = raw.strip().lower() in ("1", "true", "yes", "on")
            else:
                kw[f.name] = raw
        s = cls(**kw)
        # app.py:27 — an empty API_AUTH_KEY is falsy and disables auth, same as unset.
        if not s.API_AUTH_KEY:
            s.API_AUTH_KEY = None
        s.LOG_LEVEL = s.LOG_LEVEL.upper()
        return s

    def graph_buckets(self):
        return sorted({int(x) for x in self.HIPGRAPH_BUCKETS.split(",") if x.strip()})
