"""gemm_mfma (the decode ring kernels) under the launch pattern that exposed gemm_big's unordered
LDS-DMA completion: every launch alternates with an unrelated GEMM, and each result is checked
against fp32 of the same bf16 operands (GPU diagnostics; profiles/r5/gemm_big_clamp/README.md).

Shapes: the 8B decode projections at the planned configuration of each bucket, plus row counts that
are not a multiple of the tile (rows past M re-read other rows)."""
import math
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..', '..')))
import torch  # noqa: E402

from ai_agent_kubectl_amd import ops  # noqa: E402

dev, BF = "cuda", torch.bfloat16
torch.manual_seed(0)
REPS = int(os.environ.get("DIAG_REPS", "100"))
CFGS = [int(c) for c in os.environ.get("DIAG_CFGS", "2,3,4,5,12,19").split(",")]
SHAPES = [(256, 6144, 4096), (256, 4096, 14336), (200, 4096, 4096), (64, 28672, 4096), (100, 6144, 4096),
          (8, 4096, 14336), (16, 6144, 4096)]
other = torch.randn(4096, 4096, device=dev, dtype=BF)
wo = (torch.randn(4096, 4096, device=dev) / 64).to(BF)
total_bad = 0
for (M, N, K) in SHAPES:
    x = torch.randn(M, K, device=dev, dtype=BF)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(BF)
    ref = x.float() @ w.float().t()
    for cfg in CFGS:
        bad_reps = 0
        worst = 0.0
        try:
            ops.linear_gm(x, w, cfg, 1)
        except (ValueError, RuntimeError) as e:   # a configuration that does not take this shape
            print(f"M={M} N={N} K={K} cfg={cfg}: skipped ({str(e)[:60]})", flush=True)
            continue
        for rep in range(REPS):
            torch.nn.functional.linear(other, wo)
            y = ops.linear_gm(x, w, cfg, 1).float()
            err = (y - ref).abs()
            bad = err > 0.03 + 0.02 * ref.abs()
            if bool(bad.any()):
                bad_reps += 1
                r, c = bad.nonzero(as_tuple=True)
                if bad_reps <= 3:
                    print(f"  M={M} N={N} cfg={cfg} rep {rep}: {int(bad.sum())} bad, rows "
                          f"{sorted(set(r.tolist()))[:12]} cols {int(c.min())}..{int(c.max())}", flush=True)
            worst = max(worst, float(err.max()))
        total_bad += bad_reps
        print(f"M={M} N={N} K={K} cfg={cfg}: {bad_reps} wrong of {REPS} launches (max err {worst:.4f})", flush=True)
print(f"TOTAL wrong launches: {total_bad}", flush=True)
