"""Decode attention microbenchmark (B=256, Llama-3-8B heads): shared-prefix vs unique blocks, and
context length, for the kernel selected by KA_DECODE_WAVE_MIN (run twice to compare kernels)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

B, HQ, HKV, D, BS = 256, 32, 8, 128, 16
NB = 40000
kc = torch.randn(32, NB, HKV, BS, D, device="cuda", dtype=torch.bfloat16)   # 32 layers: cold caches
vc = torch.randn(32, NB, HKV, D, BS, device="cuda", dtype=torch.bfloat16)
q = torch.randn(B, HQ, D, device="cuda", dtype=torch.bfloat16)


def tables(ctx, shared):
    mb = (ctx + BS - 1) // BS
    bt = torch.zeros(B, mb, dtype=torch.int32)
    nxt = shared
    for b in range(B):
        for j in range(mb):
            if j < shared:
                bt[b, j] = j
            else:
                bt[b, j] = nxt
                nxt += 1
    return bt.cuda()


for ctx, shared in ((120, 4), (120, 0), (256, 4), (512, 4), (1024, 4)):
    bt = tables(ctx, shared)
    cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
    for i in range(3):
        ops.attention_decode(q, kc[i], vc[i], bt, cl, D ** -0.5)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(32):
        ops.attention_decode(q, kc[i], vc[i], bt, cl, D ** -0.5)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 32 * 1e3
    uniq = B * (((ctx + BS - 1) // BS) - shared) * HKV * BS * D * 2 * 2
    print(f"wave_min={os.environ.get('KA_DECODE_WAVE_MIN', '512')} ctx={ctx:5d} shared_blocks={shared} "
          f"{us:7.1f} us  unique KV {uniq / 1e6:6.1f} MB -> {uniq / us / 1e6:5.2f} TB/s", flush=True)

# ---- fused RoPE + KV append + decode attention (the model's decode path), ctx 120 + new token ----
cos_sin = ops.rope_cos_sin(4096, D, 500000.0, device="cuda")
for bsz in (256, 16, 1):
    for split in (1, 4):
        ctx = 121
        bt = tables(ctx, 4)[:bsz].contiguous()
        cl = torch.full((bsz,), ctx, dtype=torch.int32, device="cuda")
        pos = torch.full((bsz,), ctx - 1, dtype=torch.int32, device="cuda")
        slots = (bt[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS).to(torch.int32).contiguous()
        N = (HQ + 2 * HKV) * D
        if split == 1:
            srcs = [torch.randn(bsz, N, device="cuda", dtype=torch.bfloat16) for _ in range(4)]
        else:
            srcs = [ops.SplitK(torch.randn(split, bsz, N, device="cuda") * 0.5, split) for _ in range(4)]
        run = lambda i: ops.decode_attention_rope(srcs[i % 4], pos, cos_sin, slots, kc[i], vc[i], bt, cl,
                                                  HQ, HKV, D, D ** -0.5)
        for i in range(3):
            run(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(32):
            run(i)
        e1.record()
        torch.cuda.synchronize()
        print(f"fused rope+append+attn B={bsz:3d} ctx={ctx} qkv={'bf16' if split == 1 else f'splitK{split}'} "
              f"{e0.elapsed_time(e1) / 32 * 1e3:7.1f} us", flush=True)
