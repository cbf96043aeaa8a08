"""Time the gemm_mfma ring configurations x split-K at the decode projection shapes (partials left
for the fused consumer, as the plan runs them).  GPU only.

    python scripts/bench_gm_cfgs.py [M ...]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ai_agent_kubectl_amd import ops  # noqa: E402

BF = torch.bfloat16
Ms = [int(m) for m in sys.argv[1:]] or [128, 256]
SHAPES = {"QKV": (6144, 4096), "O": (4096, 4096), "down": (4096, 14336), "lm_head": (128256, 4096)}
CFGS = (2, 4, 5, 12, 6, 8, 19)


def timeit(fn, reps=30):
    # weights rotated through 4 copies so each launch streams them from HBM as in a decode step
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % 4)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000


for M in Ms:
    x = torch.randn(M, 4096 if M else 0, device="cuda", dtype=BF)
    for name, (N, K) in SHAPES.items():
        xs = torch.randn(M, K, device="cuda", dtype=BF)
        ws = [(torch.randn(N, K, device="cuda") / math.sqrt(K)).to(BF) for _ in range(4)]
        res = []
        for cfg in CFGS:
            bn, bm = ops.gm_shape(cfg)
            if bm > 2 * M and bm > 64:
                continue
            for sp in (1, 2, 4, 8):
                if K % (64 * sp) or K // sp < 256:
                    continue
                try:
                    ops.linear_gm(xs, ws[0], cfg, sp, defer_reduce=True, bf16_partials=True)
                except (ValueError, RuntimeError):
                    continue
                t = timeit(lambda i: ops.linear_gm(xs, ws[i], cfg, sp, defer_reduce=True, bf16_partials=True))
                tiles = ((N + bn - 1) // bn) * ((M + bm - 1) // bm) * sp
                res.append((t, cfg, sp, tiles))
        res.sort()
        print(f"M={M} {name} {N}x{K}: " + "  ".join(f"cfg{c}/s{s} ({w} wg) {t:.1f}" for t, c, s, w in res[:6]),
              flush=True)
        del ws
