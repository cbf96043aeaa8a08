"""GEMM plan autotuning for the decode path.

For every projection shape (N, K) of the loaded model and every decode batch bucket M, time the
hand-written weight-streaming kernel at a few split-K factors against hipBLASLt (`F.linear`) on the
model's *own* weights, rotating over layers so each call streams from HBM as in a real step, and
record the winner in `ops.GEMM_PLAN`.  Done once at engine start (before hipGraph capture), so the
captured graphs contain the fastest kernel per shape.
"""
from __future__ import annotations

import logging
from typing import Dict, List, Sequence, Tuple

import torch

from . import GEMM_PLAN, linear, skinny_split

logger = logging.getLogger("app.engine")


import os as _os

# TunableOp results for the decode GEMM shapes on MI355X (ROCm 7.x); loaded at start, extended
# (and re-written) if new shapes appear.  Set KA_TUNABLEOP=0 to use hipBLASLt's heuristics only.
DEFAULT_TUNABLEOP_FILE = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "tuned",
                                       "tunableop_mi355x.csv")


def _time(fn, weights: List[torch.Tensor], reps: int = 12) -> float:
    for i in range(3):
        fn(weights[i % len(weights)])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(weights[i % len(weights)])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def _tunableop_begin() -> bool:
    """KA_TUNABLEOP=1: let torch TunableOp search hipBLASLt/rocBLAS solutions for the decode shapes
    while we time them (results cached in KA_TUNABLEOP_FILE); tuning is switched off afterwards so
    prefill's ragged shapes never trigger online tuning during serving."""
    import os
    if os.environ.get("KA_TUNABLEOP", "1") != "1":
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    fname = os.environ.get("KA_TUNABLEOP_FILE", DEFAULT_TUNABLEOP_FILE)
    if fname:
        tun.set_filename(fname)
        if os.path.exists(fname):
            tun.read_file(fname)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(int(os.environ.get("KA_TUNABLEOP_MS", "60")))
    return True


def _tunableop_end() -> None:
    tun = torch.cuda.tunable
    tun.tuning_enable(False)
    try:
        tun.write_file()
    except Exception:  # pragma: no cover
        pass


@torch.inference_mode()
def tune_linear(groups: Dict[Tuple[int, int], List[torch.Tensor]], Ms: Sequence[int]) -> Dict:
    """groups: (N, K) -> list of weight tensors of that shape (one per layer)."""
    tunable = _tunableop_begin()
    try:
        return _tune(groups, Ms)
    finally:
        if tunable:
            _tunableop_end()


def _tune(groups, Ms) -> Dict:
    report = {}
    for (N, K), ws in groups.items():
        ws = ws[: max(2, min(len(ws), 16))]
        for M in sorted(set(int(m) for m in Ms if m <= 256)):
            x = torch.randn(M, K, device=ws[0].device, dtype=ws[0].dtype)
            GEMM_PLAN.pop((M, N, K), None)
            t_blas = _time(lambda w: torch.nn.functional.linear(x, w), ws)
            best = ("blas", 0, t_blas)
            if K % 64 == 0 and N % 4 == 0:
                cands = sorted({skinny_split(M, N, K, t) for t in (256, 512, 1024, 2048)})
                for sp in cands:
                    t = _time(lambda w: linear(x, w, split=sp), ws)
                    if t < best[2]:
                        best = ("skinny", sp, t)
            GEMM_PLAN[(M, N, K)] = (best[0], best[1])
            report[(M, N, K)] = {"choice": best[0], "split": best[1], "us": round(best[2], 1),
                                 "blas_us": round(t_blas, 1)}
    logger.info("gemm plan: %s", report)
    return report
