"""gemm_big split tail: error structure inside the first tail quadrant (rows / columns / k ranges)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

torch.manual_seed(0)
dev, BF = "cuda", torch.bfloat16
M, N, K = 4096, 6144, 4096
x = torch.randn(M, K, device=dev, dtype=BF)
w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(BF)
ref = x.float() @ w.float().t()
y = ops.linear_big(x, w).float()
torch.cuda.synchronize()
r0, c0 = 8 * 256, 8 * 256      # tile (8, 8): a tail tile
d = (y - ref)[r0:r0 + 256, c0:c0 + 256]
bad = d.abs() > 0.05 + 0.02 * ref[r0:r0 + 256, c0:c0 + 256].abs()
print("tile bad", int(bad.sum()), "max", float(d.abs().max()))
print("bad per row (first 64 rows):", bad.sum(1)[:64].tolist())
print("bad per col (first 64 cols):", bad.sum(0)[:64].tolist())
print("rows with bad:", int((bad.sum(1) > 0).sum()), "cols with bad:", int((bad.sum(0) > 0).sum()))
idx = bad.nonzero()[:20].tolist()
for (i, j) in idx[:12]:
    gi, gj = r0 + i, c0 + j
    parts = [float(x[gi, k0:k0 + 128].float() @ w[gj, k0:k0 + 128].float()) for k0 in range(0, K, 128)]
    print(f"  ({i},{j}) y={float(y[gi, gj]):.4f} ref={float(ref[gi, gj]):.4f} diff={float(y[gi, gj] - ref[gi, gj]):.4f}",
          "| 2-ktile parts near diff:", [k for k, p in enumerate(parts) if abs(p - float(y[gi, gj] - ref[gi, gj])) < 0.02][:4])
# whole-tensor: are non-tail tiles clean?
full_bad = ((y - ref).abs() > 0.05 + 0.02 * ref.abs())
print("bad in rows < 2048:", int(full_bad[:2048].sum()), " bad in tile cols < 2048 of rows >= 2048:", int(full_bad[2048:, :2048].sum()))
# does a bad value equal the reference somewhere else in its row / column neighbourhood?
for (i, j) in idx[:10]:
    gi, gj = r0 + i, c0 + j
    v = float(y[gi, gj])
    row = ref[gi, c0:c0 + 256]
    col = ref[r0:r0 + 256, gj]
    hits_r = (row - v).abs().lt(0.01).nonzero().flatten().tolist()
    hits_c = (col - v).abs().lt(0.01).nonzero().flatten().tolist()
    print(f"  ({i},{j}) y={v:.4f}: same-row ref matches at cols {hits_r[:6]}, same-col ref matches at rows {hits_c[:6]}")
# the same product through the no-tail path of the same kernel
os.environ["KA_GEMM_BIG_TAIL"] = "0"
ops.GEMM_BIG_TAIL = False
y0 = ops.linear_big(x, w).float()
print("no-tail launch: bad", int(((y0 - ref).abs() > 0.05 + 0.02 * ref.abs()).sum()))
