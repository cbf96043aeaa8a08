"""gemm_big numerics diagnostic (GPU): full-matrix error maps of the bf16 and SwiGLU epilogues and
repeated fused-LM-head runs against fp32, for the library named by KA_HIP_LIB (default: in-tree)."""
import math
import os

sys_path_root = os.path.abspath(os.path.join(os.path.dirname(__file__), '..', '..', '..'))
import sys

sys.path.insert(0, sys_path_root)

import torch

from ai_agent_kubectl_amd import ops
from ai_agent_kubectl_amd.ops import _hip

lib = _hip.require()
print("lib", _hip.LIB_PATH)
torch.manual_seed(0)
dev, BF = "cuda", torch.bfloat16


def gb(x, w, epi=0):
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N // 2 if epi == 3 else N, device=dev, dtype=BF)
    ws = ops.gemm_big_ws(x.device)
    _hip.check(lib.ka_gemm_big(y.data_ptr(), None, x.data_ptr(), w.data_ptr(), M, N, K, K, y.shape[1], epi, 0,
                               ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
                               ops._stream()), "gemm_big")
    return y


for (M, N, K) in [(300, 64128, 4096), (4096, 4096, 4096), (777, 6144, 4096), (2944, 28672, 4096)]:
    x = torch.randn(M, K, device=dev, dtype=BF)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(BF)
    ref = x.float() @ w.float().t()
    for rep in range(3):
        y = gb(x, w).float()
        err = (y - ref).abs()
        bad = err > 0.02 + 0.01 * ref.abs()
        nb = int(bad.sum())
        msg = f"bf16 M={M} N={N} rep{rep}: max err {float(err.max()):.4f} bad {nb}"
        if nb:
            r, c = bad.nonzero(as_tuple=True)
            msg += f" rows {sorted(set((r // 16 * 16).tolist()))[:12]} cols/256 {sorted(set((c // 256).tolist()))[:12]}" \
                   f" first {list(zip(r[:6].tolist(), c[:6].tolist()))}"
        print(msg, flush=True)
    if N % 256 == 0 and N <= 28672:
        I = N // 2
        y = gb(x, w, 3).float()
        r3 = torch.nn.functional.silu(ref[:, :I]) * ref[:, I:]
        err = (y - r3).abs()
        print(f"swiglu M={M} I={I}: max err {float(err.max()):.4f} bad {int((err > 0.02 + 0.01 * r3.abs()).sum())}",
              flush=True)
    del x, w, ref

M, V, K = 300, 64128, 4096
x = torch.randn(M, K, device=dev, dtype=BF)
w = (torch.randn(V, K, device=dev) * 0.02).to(BF)
ref = (x.float() @ w.float().t())
for rep in range(5):
    idx, val = ops.lm_head_argmax(x, w, None, None)
    chosen = ref.gather(1, idx.long()[:, None]).squeeze(1)
    best = ref.max(1).values
    d = (val - chosen).abs()
    print(f"lm_head rep{rep}: |val-ref[idx]| max {float(d.max()):.4f} rows>0.05 {(d > 0.05).nonzero().flatten().tolist()[:10]}"
          f" best-chosen max {float((best - chosen).max()):.4f}", flush=True)
sys.exit(0)
