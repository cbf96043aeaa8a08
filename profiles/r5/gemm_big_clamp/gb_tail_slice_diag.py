"""gemm_big split tail, TN 6, partial last m-tile (2944 x 6144 x 4096, 2 K-slices per tail tile): on a
wrong launch, which rows / columns are wrong and what the wrong values are made of (the full sum, one
slice only, a slice twice, another row's values) (GPU diagnostics)."""
import math
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..', '..')))
import torch  # noqa: E402

from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.ops import _hip  # noqa: E402

lib = _hip.require()
dev, BF = "cuda", torch.bfloat16
torch.manual_seed(0)
M, N, K = 2944, 6144, 4096
x = torch.randn(M, K, device=dev, dtype=BF)
w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(BF)
x2 = torch.randn(4096, K, device=dev, dtype=BF)
ref = x.float() @ w.float().t()
s0 = x[:, :K // 2].float() @ w[:, :K // 2].float().t()
s1 = ref - s0
found = 0
for rep in range(60):
    ops.linear_big(x2, w)            # another shape in between (the failures follow a shape change)
    y = ops.linear_big(x, w).float()
    err = (y - ref).abs()
    bad = err > 0.03 + 0.02 * ref.abs()
    nb = int(bad.sum())
    if not nb:
        continue
    found += 1
    r, c = bad.nonzero(as_tuple=True)
    rows = sorted(set(r.tolist()))
    tiles = sorted(set(zip((r // 256).tolist(), (c // 192).tolist())))
    print(f"rep {rep}: bad {nb}, rows {rows[:40]} ({len(rows)}), tiles {tiles[:20]} ({len(tiles)})", flush=True)
    g, rr, s0b, s1b = y[bad], ref[bad], s0[bad], s1[bad]
    for name, cand in (("slice 0 only", s0b), ("slice 1 only", s1b), ("slice 0 twice", 2 * s0b + s1b),
                       ("slice 1 twice", s0b + 2 * s1b), ("zero", torch.zeros_like(g))):
        print(f"   |got - {name}| max {float((g - cand).abs().max()):.4f}  mean {float((g - cand).abs().mean()):.4f}",
              flush=True)
    # per (tile row 0..255 within the m-tile, column within the 192-wide tile): counts
    tr = (r % 256)
    tc = (c % 192)
    print(f"   tile rows {sorted(set(tr.tolist()))[:40]}", flush=True)
    print(f"   tile cols min {int(tc.min())} max {int(tc.max())}, wave-n halves {sorted(set((tc // 96).tolist()))}",
          flush=True)
    # does a wrong row hold another row's reference (a row mix-up)?
    rw = rows[0]
    cols = bad[rw].nonzero().flatten()
    d = (y[:, cols] - y[rw, cols]).abs().sum(1)
    dd = (ref[:, cols] - y[rw, cols]).abs().sum(1)
    print(f"   row {rw}: closest reference row {int(dd.argmin())} (dist {float(dd.min()):.3f}, own {float(dd[rw]):.3f})",
          flush=True)
    if found >= 4:
        break
print(f"{found} wrong launches; tail error word {ops.gemm_big_err(torch.device(dev))}", flush=True)
