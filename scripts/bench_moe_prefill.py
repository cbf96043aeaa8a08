"""Mixtral-8x7B MoE block at prefill token counts: the device-routed grouped paths
(ops.moe_experts_grouped: expert-sorted rows on gemm_big's grouped mode, and the grouped ring kernel
per configuration) against the host-synced sorted path
(models/moe.py moe_sorted: one host read of the expert counts per layer + hipBLASLt per expert).
Prints ms per block and the expert GEMMs' TFLOP/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.models.config import get_config  # noqa: E402
from ai_agent_kubectl_amd.models.moe import moe_sorted  # noqa: E402

cfg = get_config("mixtral-8x7b")
E, H, I, k = cfg.num_experts, cfg.hidden, cfg.intermediate, cfg.top_k
L = {"w13": (torch.randn(E, 2 * I, H, device="cuda") * 0.02).to(torch.bfloat16),
     "w2": (torch.randn(E, H, I, device="cuda") * 0.02).to(torch.bfloat16),
     "router": (torch.randn(E, H, device="cuda") * 0.02).to(torch.bfloat16)}


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for T in (1024, 4096, 8192):
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    tw, tid = ops.moe_topk(ops.linear(x, L["router"]), k)
    flop = 2 * T * k * 3 * H * I
    want = moe_sorted(x, L, cfg, 0, 1).float()
    line = [f"T={T:5d}"]
    ms = timeit(lambda: moe_sorted(x, L, cfg, 0, 1))
    line.append(f"sorted+hipBLASLt {ms:7.2f} ms ({flop / ms / 1e9:6.1f} TF/s)")
    for mode, c in (("big", None), ("gm", 2), ("gm", 19)):
        saved = ops.MOE_GROUPED_CFG, ops.MOE_PREFILL
        ops.MOE_PREFILL = mode
        ops.MOE_GROUPED_CFG = c if c is not None else saved[0]
        try:
            err = (ops.moe_experts_grouped(x, L["w13"], L["w2"], tw, tid, 0).float() - want).abs().max().item()
            ms = timeit(lambda: ops.moe_experts_grouped(x, L["w13"], L["w2"], tw, tid, 0))
        finally:
            ops.MOE_GROUPED_CFG, ops.MOE_PREFILL = saved
        name = "grouped gemm_big" if mode == "big" else f"grouped gm cfg {c}"
        line.append(f"{name} {ms:7.2f} ms ({flop / ms / 1e9:6.1f} TF/s, maxdiff {err:.3f})")
    print(" | ".join(line), flush=True)
