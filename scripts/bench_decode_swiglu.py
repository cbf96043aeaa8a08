"""Decode-size gate_up: the GEMM plan's kernel + SiLU·mul (what the model runs) against the ring
kernel with the SwiGLU epilogue over the [gate; up] weight (ops.linear_gm_swiglu), weights rotated
past the Infinity Cache, timed as hipGraph replays of 20 launches; numerics vs fp32."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.ops import autotune  # noqa: E402

dev, BF = "cuda", torch.bfloat16
I, K = 14336, 4096
copies = 4
Ws = [(torch.randn(2 * I, K, device=dev) / K ** 0.5).to(BF) for _ in range(copies)]


def graph_time(fn, n=20, iters=8):
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


import json  # noqa: E402
plans = json.load(open(autotune.DEFAULT_PLAN_FILE))["plans"]
for M in (64, 128, 160, 192, 256, 320, 384, 512):
    x = torch.randn(M, K, device=dev, dtype=BF)
    e = plans.get(f"{M},{2 * I},{K},plain")
    if e:
        ops.GEMM_PLAN[(M, 2 * I, K)] = tuple(e[:3])
    base = graph_time(lambda i: ops.silu_mul(ops.linear(x, Ws[i % copies], defer_reduce=True)))
    ref = torch.nn.functional.silu(x.float() @ Ws[0][:I].float().t()) * (x.float() @ Ws[0][I:].float().t())
    res = []
    for cfg in (2, 3, 4, 5, 12):
        try:
            y = ops.linear_gm_swiglu(x, Ws[0], cfg)
        except RuntimeError as err:
            res.append(f"cfg{cfg}: {err}")
            continue
        torch.cuda.synchronize()
        errv = (y.float() - ref).abs().max().item()
        t = graph_time(lambda i: ops.linear_gm_swiglu(x, Ws[i % copies], cfg))
        res.append(f"cfg{cfg} {t:6.1f} us (err {errv:.3f})")
    print(f"M={M:4d} plan {e[:3] if e else None} + silu: {base:6.1f} us | " + " | ".join(res), flush=True)
