"""gemm_big intermittent wrong rows: for each shape, launches alternating with another shape until a
few wrong results; prints the wrong rows / tiles (in tile-local coordinates) (GPU diagnostics)."""
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
other = torch.randn(4096, 4096, device=dev, dtype=BF)
SHAPES = [(2944, 6144, 4096), (4096, 1152, 4096), (2944, 4096, 4096), (4096, 4096, 4096)]
if os.environ.get("DIAG_SHAPES"):   # e.g. "2944x6144x4096,4096x1152x4096"
    SHAPES = [tuple(int(v) for v in t.split("x")) for t in os.environ["DIAG_SHAPES"].split(",")]
REPS = int(os.environ.get("DIAG_REPS", "40"))
for (M, N, K) in SHAPES:
    x = torch.randn(M, K, device=dev, dtype=BF)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(BF)
    wo = (torch.randn(6144, K, device=dev) / math.sqrt(K)).to(BF)
    ref = x.float() @ w.float().t()
    tn = int(lib.ka_gemm_big_tn(M, N, 0))
    BN = 32 * tn
    found = 0
    for rep in range(REPS):
        ops.linear_big(other, wo)
        y = ops.linear_big(x, w).float()
        bad = (y - ref).abs() > 0.03 + 0.02 * ref.abs()
        nb = int(bad.sum())
        if not nb:
            continue
        found += 1
        r, c = bad.nonzero(as_tuple=True)
        tiles = sorted(set(zip((r // 256).tolist(), (c // BN).tolist())))
        print(f"M={M} N={N} tn={tn} rep {rep}: bad {nb} tiles {tiles[:12]} ({len(tiles)}) tile rows "
              f"{sorted(set((r % 256).tolist()))[:24]} tile cols {int((c % BN).min())}..{int((c % BN).max())}",
              flush=True)
        if found >= 6:
            break
    print(f"M={M} N={N} tn={tn}: {found} wrong of {rep + 1} launches", flush=True)
    del x, w, wo, ref
