"""ctypes binding to the in-tree HIP kernel library (`ops/lib/libkagent_hip.so`).

The library is built by `ai_agent_kubectl_amd.build.build_hip()` (hipcc --offload-arch=gfx950) from
`csrc/*.hip`.  Every kernel entry point is a plain `extern "C"` launcher that takes raw device
pointers and the HIP stream, so calls made while torch is capturing a hipGraph
(`torch.cuda.CUDAGraph`) are recorded into the graph like any torch kernel.

There is deliberately no fallback: on a GPU the engine refuses to run without this library
(`require()` raises), so a silent eager-PyTorch path can never masquerade as the HIP path.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
DEFAULT_LIB = os.path.join(LIB_DIR, "libkagent_hip.so")


def _lib_path() -> str:
    """The in-tree library, always, unless a diagnostic run asks for another build of it: KA_HIP_LIB is
    honoured only together with KA_HIP_LIB_DIAG=1 (A/B kernel experiments, scripts/), so no stray
    environment variable can route the engine, the tests or the bench to an experimental build."""
    alt = os.environ.get("KA_HIP_LIB")
    if alt and os.environ.get("KA_HIP_LIB_DIAG") == "1":
        return alt
    if alt:
        raise RuntimeError("KA_HIP_LIB is set without KA_HIP_LIB_DIAG=1: refusing to load a non-default "
                           f"kernel library ({alt}); unset it, or set KA_HIP_LIB_DIAG=1 for a diagnostic run")
    return DEFAULT_LIB


LIB_PATH = _lib_path()

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None
_err: Optional[str] = None

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float

_RESTYPES = {"ka_gemm_big_ws_bytes": ctypes.c_size_t, "ka_decode_persistent_ws": ctypes.c_size_t,
             "ka_decode_persistent_xbytes": ctypes.c_size_t, "ka_decode_persistent_xflag_offset": ctypes.c_size_t,
             "ka_decode_cascade_ws": ctypes.c_size_t}

_SIGS = {
    "ka_rmsnorm": [P, P, P, P, I, I, F, P],
    "ka_rope_kv": [P, P, P, P, P, P, P, I, I, I, I, I, P],
    "ka_silu_mul": [P, P, I, I, P],
    "ka_embedding": [P, P, P, I, I, I, I, P],
    "ka_masked_argmax": [P, P, P, P, P, I, I, I, I, P, I, P],
    "ka_argmax_slices": [I, I],
    "ka_moe_topk": [P, P, P, I, I, I, P],
    "ka_paged_decode": [P, P, P, P, P, I, P, I, I, I, I, I, F, P],
    "ka_paged_decode_rope": [P, P, P, I, I, P, P, P, P, P, P, I, P, I, I, I, I, I, F, P],
    "ka_paged_decode_rope_cascade": [P, P, P, I, I, P, P, P, P, P, P, I, P, I, I, I, I, I, F, P, P, P],
    "ka_decode_cascade_ws": [I, I],
    "ka_paged_prefill": [P, P, P, P, P, I, P, P, I, I, I, I, I, I, F, P],
    "ka_gemm_skinny": [P, P, P, P, I, I, I, I, P],
    "ka_gemv_swiglu": [P, P, P, P, I, I, I, I, P],
    "ka_rmsnorm_splitk": [P, P, P, I, I, P, I, I, F, P],
    "ka_rope_kv_splitk": [P, P, P, P, I, P, P, P, I, I, I, I, I, P],
    "ka_silu_mul_splitk": [P, P, I, I, I, P],
    "ka_kv_block_copy": [P, P, P, P, I, I, ctypes.c_long, ctypes.c_long, P],
    "ka_prefetch": [P, ctypes.c_long, I, P, P],
    "ka_gemm_mfma": [P, P, P, P, I, I, I, I, I, I, I, I, I, P],
    "ka_gemv_rows": [P, P, P, P, I, I, I, I, I, I, P],
    "ka_gemm_mfma_swiglu": [P, P, P, I, I, I, I, I, I, P],
    "ka_gemm_mfma_grouped": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P],
    "ka_gemm_big": [P, P, P, P, I, I, I, I, I, I, I, P, ctypes.c_size_t, P],
    "ka_gemm_big_ws_bytes": [],
    "ka_gemm_big_plan": [I, I, I, I, ctypes.c_size_t, P, P],
    "ka_gemm_big_tn": [I, I, I],
    "ka_gemm_big_grouped": [P, P, P, P, I, P, I, I, I, I, I, I, I, P],
    "ka_gemm_big_err": [P, P],
    "ka_gemm_big_argmax": [P, P, P, P, I, I, I, I, P, P, I, I, P, P],
    "ka_argmax_finish": [P, P, P, P, I, I, I, P],
    "ka_argmax_combine": [P, P, P, I, I, P],
    "ka_decode_persistent": [P, P, P, I, I, I, I, I, F, F, P, P, ctypes.c_long, P, P, P, P, P, P, P, I, I, P],
    "ka_decode_persistent_tp": [P, P, P, I, I, I, I, I, F, F, P, P, ctypes.c_long, P, P, P, P, P, P, P, I, I, I, I,
                                P, P, P, P],
    "ka_decode_persistent_xbytes": [],
    "ka_decode_persistent_xflag_offset": [],
    "ka_decode_persistent_max_b": [I, I, I],
    "ka_decode_persistent_max_b2": [I, I, I, I],
    "ka_decode_persistent_ws": [I, I, I, I],
    "ka_decode_persistent_err": [P, P],
    "ka_decode_persistent_err_offset": [],
    "ka_gm_bn": [I],
    "ka_gm_bm": [I],
    "ka_moe_align": [P, P, P, I, I, I, P],
    "ka_moe_gemm": [P, P, P, P, P, I, I, I, I, I, I, I, P, P],
    "ka_moe_combine": [P, P, P, I, P, P, I, I, I, I, I, P],
    "ka_moe_sort": [P, P, P, P, P, P, I, I, I, I, I, P],
    "ka_allreduce_oneshot": [P, P, P, P, P, P, P, I, I, I, I, I, P],
    "ka_allgather_oneshot": [P, P, P, P, P, P, P, I, I, I, I, I, P],
    "ka_allreduce_rmsnorm": [P, P, P, P, F, P, P, P, P, P, I, I, I, I, I, I, I, I, P],
    "ka_ar_alloc": [P, ctypes.c_size_t],
    "ka_ar_free": [P],
    "ka_ar_get_handle": [P, P],
    "ka_ar_open_handle": [P, P],
    "ka_ar_close_handle": [P],
}


def load(path: str = LIB_PATH) -> Optional[ctypes.CDLL]:
    """Load the library once; returns None (and remembers why) if it is missing."""
    global _lib, _err
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            _err = f"HIP kernel library not built: {path} (run python -c 'import __graft_entry__ as g; g.build()')"
            return None
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            _err = f"failed to load {path}: {e}"
            return None
        for name, argtypes in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = lib
        return _lib


def require() -> ctypes.CDLL:
    lib = load()
    if lib is None:
        raise RuntimeError(_err or "HIP kernel library unavailable")
    return lib


def available() -> bool:
    return load() is not None


def check(code: int, what: str) -> None:
    if code != 0:
        raise RuntimeError(f"{what} failed with hipError {code}")
