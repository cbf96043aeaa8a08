"""Batch-1 decode GEMVs: weights streamed from HBM (rotating copies larger than the 256 MB Infinity
Cache) vs from the MALL (one copy, or a prefetch_kernel pass just before), timed as hipGraph replays
of 20 launches (inter-kernel gaps included, as in the decode graph).

  python scripts/bench_gemv_mall.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

dev, BF = "cuda", torch.bfloat16
REPS = 20


def graph_time(fn, n=REPS, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(n):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(iters):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


for name, N, K in [("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)]:
    nbytes = N * K * 2
    copies = max(2, (640 << 20) // nbytes + 1)
    Ws = [torch.randn(N, K, device=dev, dtype=BF) for _ in range(copies)]
    x = torch.randn(1, K, device=dev, dtype=BF)
    ops.linear(x, Ws[0])
    cold = graph_time(lambda i: ops.linear(x, Ws[i % copies]))
    warm = graph_time(lambda i: ops.linear(x, Ws[0]))
    pf = graph_time(lambda i: ops.prefetch(Ws[i % copies]))
    both = graph_time(lambda i: (ops.prefetch(Ws[i % copies]), ops.linear(x, Ws[i % copies])))
    print(f"{name:8s} {nbytes / 1e6:6.1f} MB  cold {cold:7.2f} us ({nbytes / cold / 1e6:5.2f} TB/s)  "
          f"mall-warm {warm:7.2f} us ({nbytes / warm / 1e6:5.2f} TB/s)  prefetch {pf:7.2f} us  "
          f"prefetch+gemv {both:7.2f} us -> gemv after prefetch ~{both - pf:6.2f} us", flush=True)
    del Ws
    torch.cuda.empty_cache()
