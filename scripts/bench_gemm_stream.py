"""Decode-GEMM microbenchmark: the deep-prefetch LDS-DMA stream kernels (gemm_tile cfg 10-14,
csrc/gemm_stream.hip) against the register-staged tile kernels (cfg 0-4, 9) and hipBLASLt on the
Llama-3-8B projection shapes, weights rotated over 8 copies (> the 256 MB MALL for the large
shapes) so every call streams its weights from HBM as in a decode step.

Times are per call; "defer" = split-K partials left for the fused consumer (what the model runs),
"full" includes the split-K reduce kernel.  Also checks every stream cfg against fp32.
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.ops.autotune import _time, tile_candidates  # noqa: E402

SHAPES = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")]
Ms = [int(a) for a in sys.argv[1:]] or [256, 128]


def main():
    torch.manual_seed(0)
    for M in Ms:
        tot = {"blas": 0.0, "old": 0.0, "new": 0.0}
        for N, K, name in SHAPES:
            ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(8)]
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            want = x.float() @ ws[0].float().t()
            tb = _time(lambda w: torch.nn.functional.linear(x, w), ws, reps=24)
            old, new = [], []
            for cfg, sp in tile_candidates(M, N, K, cfgs=(0, 1, 2, 3, 4, 9, 14, 15, 17, 18, 19, 20)):
                if cfg >= 17 and sp == 1:
                    err = (ops.linear_tile(x, ws[0], cfg, sp).float() - want).abs().max().item()
                    assert err < 0.1, (cfg, err)
                t = _time(lambda w: ops.linear_tile(x, w, cfg, sp, defer_reduce=True), ws, reps=24)
                (new if cfg >= 17 else old).append((round(t, 1), cfg, sp))
            old.sort()
            new.sort()
            fl = 2 * M * N * K
            gb = N * K * 2 / 1e9
            bo, bn = old[0][0], new[0][0]
            tot["blas"] += tb
            tot["old"] += min(tb, bo)
            tot["new"] += min(tb, bo, bn)
            print(f"M={M:4d} {name:8s} N={N:6d} K={K:6d}  blas {tb:6.1f}us ({gb / tb * 1e3:5.2f} TB/s)  "
                  f"tile {bo:6.1f}us  pf2 {bn:6.1f}us ({gb / bn * 1e3:5.2f} TB/s, {fl / bn / 1e6:5.0f} TF)  "
                  f"pf2 top4={new[:4]}  tile top2={old[:2]}", flush=True)
            del ws
        print(f"M={M} per-layer: blas {tot['blas']:.1f} us, best-of(blas,tile) {tot['old']:.1f} us, "
              f"best-of(all) {tot['new']:.1f} us", flush=True)


if __name__ == "__main__":
    main()
