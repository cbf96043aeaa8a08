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


@torch.inference_mode()
def tune_linear(groups: Dict[Tuple[int, int], List[torch.Tensor]], Ms: Sequence[int]) -> Dict:
    """groups: (N, K) -> list of weight tensors of that shape (one per layer)."""
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
