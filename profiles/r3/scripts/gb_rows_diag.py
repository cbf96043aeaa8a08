"""gemm_big full-matrix error map for the shapes with a partial last m-tile (M % 256 != 0), split tail
on and off: which rows / tiles are wrong (GPU)."""
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


def run(x, w, tail, epi=0):
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N // 2 if epi == 3 else N, device=dev, dtype=BF)
    ws = ops.gemm_big_ws(x.device) if tail else None
    _hip.check(lib.ka_gemm_big(y.data_ptr(), None, x.data_ptr(), w.data_ptr(), M, N, K, K, y.shape[1], epi, 0,
                               ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
                               ops._stream()), "gemm_big")
    return y


for (M, N, K) in [(2944, 6144, 4096), (2944, 4096, 4096), (2900, 4096, 14336), (4000, 6144, 4096), (777, 6144, 4096)]:
    x = torch.randn(M, K, device=dev, dtype=BF)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(BF)
    ref = x.float() @ w.float().t()
    tn = lib.ka_gemm_big_tn(M, N, 0)
    for tail in (True, False):
        for rep in range(2):
            y = run(x, w, tail).float()
            err = (y - ref).abs()
            bad = err > 0.03 + 0.02 * ref.abs()
            nb = int(bad.sum())
            msg = f"M={M} N={N} K={K} tn={tn} tail={int(tail)} rep{rep}: max err {float(err.max()):.4f} bad {nb}"
            if nb:
                r, c = bad.nonzero(as_tuple=True)
                rows = sorted(set(r.tolist()))
                tiles = sorted(set(zip((r // 256).tolist(), (c // (32 * tn)).tolist())))
                msg += f"\n   rows {rows[:24]}{' ...' if len(rows) > 24 else ''} ({len(rows)})\n   tiles {tiles[:24]} ({len(tiles)})"
                # are the wrong rows' values equal to another row's reference (a row mix-up)?
                rr = rows[0]
                cols = bad[rr].nonzero().flatten()[:4].tolist()
                msg += f"\n   row {rr} cols {cols}: got {[round(float(y[rr, c]), 3) for c in cols]} want " \
                       f"{[round(float(ref[rr, c]), 3) for c in cols]}"
            print(msg, flush=True)
    print(f"tail error word {ops.gemm_big_err(torch.device(dev))}", flush=True)
    del x, w, ref
