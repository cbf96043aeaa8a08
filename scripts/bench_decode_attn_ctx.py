"""Fused RoPE + KV append + decode attention at B = 256 (Llama-3-8B heads) against the context length:
does the kernel's time follow the number of 32-token chunks each wave walks in sequence (a latency
chain) or the bytes it reads?  The QKV input is the decode path's split-K 4 bf16 partials.

    python scripts/bench_decode_attn_ctx.py [--ctx 33,65,97,121,129,131,161] [--shared 4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

HQ, HKV, D, BS = 32, 8, 128, 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", default="33,65,97,121,129,131,161")
    ap.add_argument("--shared", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=64)
    args = ap.parse_args()
    B = args.batch
    NB = 12000
    kc = torch.randn(8, NB, HKV, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(8, NB, HKV, D, BS, device="cuda", dtype=torch.bfloat16)
    cos_sin = ops.rope_cos_sin(4096, D, 500000.0, device="cuda")
    N = (HQ + 2 * HKV) * D
    srcs = [ops.SplitK((torch.randn(4, B, N, device="cuda") * 0.5).to(torch.bfloat16), 4) for _ in range(4)]
    for ctx in (int(c) for c in args.ctx.split(",")):
        mb = (ctx + BS - 1) // BS
        sh = min(args.shared, mb - 1)
        bt = torch.zeros(B, mb, dtype=torch.int32)
        nxt = sh
        for b in range(B):
            for j in range(mb):
                if j < sh:
                    bt[b, j] = j
                else:
                    bt[b, j] = nxt
                    nxt += 1
        bt = bt.cuda()
        cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        pos = torch.full((B,), ctx - 1, dtype=torch.int32, device="cuda")
        slots = (bt[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS).to(torch.int32).contiguous()

        def run(i):
            return ops.decode_attention_rope(srcs[i % 4], pos, cos_sin, slots, kc[i % 8], vc[i % 8], bt, cl,
                                             HQ, HKV, D, D ** -0.5)

        for i in range(8):
            run(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(args.reps):
            run(i)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / args.reps * 1e3
        chunks = (ctx - 1 + 31) // 32
        print(f"nw2_min={os.environ.get('KA_DECODE_NW2_MIN_WGS', 'default')} B={B} ctx={ctx:4d} "
              f"chunks={chunks} shared_blocks={sh}: {us:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
