"""gemm_big split-tail diagnosis: which 256 x 256 tiles / 128 x 128 quadrants of Y = X W^T are wrong,
and whether a wrong quadrant equals one K slice's contribution (a lost / stale slice)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

torch.manual_seed(0)
dev, BF = "cuda", torch.bfloat16
for (M, N, K) in [(4096, 6144, 4096), (2944, 6144, 4096), (777, 6144, 4096)]:
    x = torch.randn(M, K, device=dev, dtype=BF)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(BF)
    ref = x.float() @ w.float().t()
    half0 = x[:, :K // 2].float() @ w[:, :K // 2].float().t()
    for rep in range(3):
        y = ops.linear_big(x, w).float()
        torch.cuda.synchronize()
        bad = ((y - ref).abs() > 0.05 + 0.02 * ref.abs())
        tm, tn = (M + 255) // 256, (N + 255) // 256
        wrong = []
        for i in range(tm):
            for j in range(tn):
                for qm in range(2):
                    for qn in range(2):
                        r0, c0 = i * 256 + qm * 128, j * 256 + qn * 128
                        b = bad[r0:r0 + 128, c0:c0 + 128]
                        if b.numel() and b.any():
                            d = (y - ref)[r0:r0 + 128, c0:c0 + 128]
                            h0 = half0[r0:r0 + 128, c0:c0 + 128]
                            h1 = (ref - half0)[r0:r0 + 128, c0:c0 + 128]
                            yy = y[r0:r0 + 128, c0:c0 + 128]
                            kind = ("=slice0" if (yy - h0).abs().max() < 0.05 else
                                    "=slice1" if (yy - h1).abs().max() < 0.05 else
                                    "=2x?" if (yy - 2 * ref[r0:r0 + 128, c0:c0 + 128]).abs().max() < 0.1 else "other")
                            wrong.append((i, j, qm * 2 + qn, int(b.sum()), kind))
        print(f"M={M} N={N} rep{rep}: bad {int(bad.sum())} in {len(wrong)} quadrants, err {ops.gemm_big_err(torch.device(dev))}")
        for wq in wrong[:24]:
            print("   tile", wq)
