"""Decode-GEMM microbenchmark: hand-written weight-streaming kernel vs hipBLASLt (F.linear).

Weights rotate over several copies (> 512 MB total) so every call streams from HBM as in a real
decode step (consecutive layers never share weights).  Prints effective HBM GB/s of W.
"""
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, ws, reps=40):
    torch.cuda.synchronize()
    for i in range(4):
        fn(ws[i % len(ws)])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(ws[i % len(ws)])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    Ms = [int(m) for m in os.environ.get("MS", "1,16,64,128,256").split(",")]
    out = []
    for name, (N, K) in SHAPES.items():
        ncopy = max(2, (768 << 20) // (N * K * 2) + 1)
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(ncopy)]
        for M in Ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            t_blas = timeit(lambda w: torch.nn.functional.linear(x, w), ws)
            best = None
            for wgs in (256, 512, 1024, 2048):
                sp = ops.skinny_split(M, N, K, wgs)
                t = timeit(lambda w: ops.linear(x, w, split=sp), ws)
                if best is None or t < best[0]:
                    best = (t, sp, wgs)
            gb = N * K * 2 / 1e9
            row = {"gemm": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t_blas, 1),
                   "skinny_us": round(best[0], 1), "split": best[1], "target_wgs": best[2],
                   "hipblaslt_TBps": round(gb / t_blas * 1e3, 2), "skinny_TBps": round(gb / best[0] * 1e3, 2)}
            print(json.dumps(row), flush=True)
            out.append(row)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
