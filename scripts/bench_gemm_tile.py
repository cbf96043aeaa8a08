import torch, time, sys
sys.path.insert(0, "/root/repo")
from ai_agent_kubectl_amd import ops
from ai_agent_kubectl_amd.ops.autotune import _time, tile_candidates
shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
for M in (128, 256, 384, 512):
    tot_b = tot_t = 0
    for N, K in shapes:
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(8)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        tb = _time(lambda w: torch.nn.functional.linear(x, w), ws, reps=24)
        res = []
        for cfg, sp in tile_candidates(M, N, K):
            t = _time(lambda w: ops.linear_tile(x, w, cfg, sp), ws, reps=24)
            res.append((t, cfg, sp))
        res.sort()
        best = res[0] if res else (float("inf"), -1, -1)
        tot_b += tb; tot_t += min(tb, best[0])
        fl = 2 * M * N * K
        print(f"M={M:4d} N={N:6d} K={K:6d} blas {tb:7.1f}us ({fl/tb/1e6:6.0f} TF)  tile best {best[0]:7.1f}us cfg={best[1]} split={best[2]} ({fl/best[0]/1e6:6.0f} TF)  top3={[(round(a,1),b,c) for a,b,c in res[:3]]}", flush=True)
        del ws
    print(f"M={M} per-layer blas {tot_b:.1f} us  best-of {tot_t:.1f} us", flush=True)
