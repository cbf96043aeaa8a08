"""Print the decode GEMM plan the engine's autotune picks for the Llama-3-8B projection shapes.

Usage (GPU): python scripts/autotune_report.py [M ...]   (default: 128 256)
O / down are tuned as the model runs them at TP = 1: together with the fused reduce + RMSNorm.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ai_agent_kubectl_amd.ops.autotune import tune_linear  # noqa: E402

Ms = [int(a) for a in sys.argv[1:]] or [128, 256]
shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
groups = {s: [(torch.randn(*s, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(16)] for s in shapes}
for fed in ((), ((4096, 4096), (4096, 14336))):
    rep = tune_linear(groups, Ms, norm_fed=fed, bf16_partials=True)
    print("norm-fed O/down" if fed else "plain (reduce kernel charged)")
    for k, v in sorted(rep.items()):
        print(" ", k, v)
