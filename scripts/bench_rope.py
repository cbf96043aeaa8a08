"""Prefill RoPE + paged-KV append (the 16-token window kernel) at a bench-sized step: T tokens of
Llama-3-8B heads, slots in runs of consecutive blocks (sub-block-reuse offsets), bf16 QKV and fp32
split-K partials.  Library from KA_HIP_LIB (A/B against another build)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

HQ, HKV, D, BS = 32, 8, 128, 16
for T in (8035, 4077, 2944):
    NB = T // BS + 600
    kc = torch.zeros(NB, HKV, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros(NB, HKV, D, BS, device="cuda", dtype=torch.bfloat16)
    qkv = torch.randn(T, (HQ + 2 * HKV) * D, device="cuda", dtype=torch.bfloat16)
    cs = ops.rope_cos_sin(8192, D, 5e5, device="cuda")
    pos = (torch.arange(T, device="cuda", dtype=torch.int32) % 40) + 60
    slots = (torch.arange(T, device="cuda", dtype=torch.int32) + 7 * (torch.arange(T, device="cuda") // 34)).int()
    for name, src in (("bf16", qkv), ("splitK2", ops.SplitK(torch.randn(2, T, qkv.shape[1], device="cuda"), 2))):
        for _ in range(3):
            ops.rope_kv_write(src, pos, cs, slots, kc, vc, HQ, HKV, D)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.rope_kv_write(src, pos, cs, slots, kc, vc, HQ, HKV, D)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        byts = T * ((HQ + 2 * HKV) * D * (2 if name == "bf16" else 8) + (HQ + 2 * HKV) * D * 2)
        print(f"{os.path.basename(os.environ.get('KA_HIP_LIB', 'in-tree'))} T={T} {name}: {us:7.1f} us "
              f"({byts / us / 1e6:4.2f} TB/s)", flush=True)
