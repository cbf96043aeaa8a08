"""Mixtral-8x7B expert block microbenchmark (ops.moe_experts: align + grouped w13 GEMM + SiLU.mul +
grouped w2 GEMM + combine) at decode token counts, split-K (default plan) vs a forced split of 1.
Weights rotate over 4 layer copies (11 GB) so every call streams from HBM.  Prints the effective
HBM rate of the weights the routed experts actually read."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

E, H, I, k = 8, 4096, 14336, 2
NL = 4
w13 = [(torch.randn(E, 2 * I, H, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(NL)]
w2 = [(torch.randn(E, H, I, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(NL)]


def timeit(fn, reps=24):
    for i in range(4):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


orig = ops.moe_split
for T in (1, 2, 4, 8, 16, 32, 64, 128, 256):
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    tw, tid = ops.moe_topk(torch.randn(T, E, device="cuda", dtype=torch.bfloat16), k)
    active = len(set(tid.flatten().tolist()))
    gb = active * 3 * H * I * 2 / 1e9
    res = {}
    variants = [("split", orig), ("nosplit", lambda *a, **kw: 1)]
    if os.environ.get("MOE_TARGETS"):
        import functools
        variants += [(f"t{t}", functools.partial(orig, target_wgs=int(t))) for t in os.environ["MOE_TARGETS"].split(",")]
    for name, fn in variants:
        ops.moe_split = fn
        res[name] = timeit(lambda i: ops.moe_experts(x, w13[i % NL], w2[i % NL], tw, tid, 0))
    ops.moe_split = orig
    print(f"T={T:4d} active experts={active} plan split w13={orig(T * k, E, 2 * I, H)} w2={orig(T * k, E, H, I)}  "
          f"split {res['split']:7.1f} us ({gb / res['split'] * 1e3:4.2f} TB/s)  "
          f"nosplit {res['nosplit']:7.1f} us ({gb / res['nosplit'] * 1e3:4.2f} TB/s)"
          + "".join(f"  {n} {v:7.1f}" for n, v in res.items() if n.startswith("t")), flush=True)
