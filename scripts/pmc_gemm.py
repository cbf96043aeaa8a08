"""Driver for PMC counter passes over the M = 256 gate_up GEMM variants (one process, each variant
run 16 times on rotating weights): hipBLASLt, tile cfg 2 (128x128 register-staged), tile cfg 15
(256x256 register-staged, split 2), stream cfg 13 (256x256 LDS-DMA, split 2), stream cfg 14
(128x256 LDS-DMA)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from ai_agent_kubectl_amd import ops  # noqa: E402

M, N, K = 256, 28672, 4096
ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(6)]
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
variants = [("blas", lambda w: torch.nn.functional.linear(x, w))]
for cfg, sp in ((2, 1), (15, 2), (13, 2), (14, 1)):
    variants.append((f"cfg{cfg}", lambda w, c=cfg, s=sp: ops.linear_tile(x, w, c, s, defer_reduce=True)))
for name, fn in variants:
    for i in range(16):
        fn(ws[i % len(ws)])
    torch.cuda.synchronize()
print("done")
