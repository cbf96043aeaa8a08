"""Batch-1 GEMV: the current kernel (gemv_ring_kernel through ops.linear / ka_gemv_swiglu at the
plan's split) against the row-streaming kernel (ka_gemv_rows) over rows-per-wave x split-K, on the
Llama-3-8B projection shapes; weights rotated past the Infinity Cache, hipGraph replays of 20
launches; numerics vs fp32."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.ops import _p, _stream  # noqa: E402

dev, BF = "cuda", torch.bfloat16
M = int(os.environ.get("M", "1"))
lib = ops.require()


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


shapes = [("qkv", 6144, 4096, 2, False), ("o", 4096, 4096, 4, False), ("gate_up", 28672, 4096, 1, False),
          ("down_swiglu", 4096, 14336, 4, True), ("lm_head", 128256, 4096, 1, False)]
for name, N, K, plan_split, swiglu in shapes:
    copies = max(3, (768 << 20) // (N * K * 2))
    Ws = [(torch.randn(N, K, device=dev) / K ** 0.5).to(BF) for _ in range(copies)]
    Kx = 2 * K if swiglu else K
    x = torch.randn(M, Kx, device=dev, dtype=BF)
    xs = ops.silu_mul(x) if swiglu else x
    ref = xs.float() @ Ws[0].float().t()
    ws = torch.empty(16 * M * N, device=dev, dtype=torch.float32)
    y = torch.empty(M, N, device=dev, dtype=BF)
    defer = plan_split > 1

    def base(i):
        if swiglu:
            ops.check(lib.ka_gemv_swiglu(None if defer else _p(y), _p(x), _p(Ws[i % copies]), _p(ws), M, N, K,
                                         plan_split, _stream()), "gemv_swiglu")
        else:
            ops.check(lib.ka_gemm_skinny(None if defer else _p(y), _p(x), _p(Ws[i % copies]), _p(ws), M, N, K,
                                         plan_split, _stream()), "skinny")
    tb = graph_time(base)
    gb = N * K * 2 / 1e3
    print(f"{name:12s} N={N} K={K}  current (split {plan_split}): {tb:6.1f} us {gb / tb:6.0f} GB/s", flush=True)
    res = []
    for split, var in [(sp, v) for sp in (1, 2, 4, 8) for v in (0, 1, 2, 3)]:
        if K % (512 * split) or M * (K // split) * 2 * (4 if M > 2 else M) > 65536 * M:
            continue
        for rw in (1, 2, 4, 8):
            d = split > 1 and defer

            def fn(i, split=split, rw=rw, d=d, var=var):
                ops.check(lib.ka_gemv_rows(None if d else _p(y), _p(x), _p(Ws[i % copies]), _p(ws), M, N, K, split,
                                           rw, int(swiglu) | (var << 1), _stream()), "gemv_rows")
            try:
                fn(0)
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            if d:
                got = ws[: split * M * N].view(split, M, N).sum(0)
            else:
                got = y.float()
            err = (got - ref).abs().max().item()
            t = graph_time(fn)
            res.append((t, split, rw, var, err, d))
    res.sort()
    for t, split, rw, var, err, d in res[:8]:
        print(f"    rows split {split} rw {rw:2d} ring {16 if var & 1 else 8} {'nt' if var & 2 else 'rt'}"
              f"{' (partials)' if d else ''}: {t:6.1f} us {gb / t:6.0f} GB/s err {err:.4f}", flush=True)
    del Ws
    torch.cuda.empty_cache()
