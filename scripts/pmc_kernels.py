"""Workload for profiles/scripts_archive/gpu_pmc_kernels.sh: a few dispatches of each hand-written hot kernel at its
serving shape — prefill attention (256 seqs x 32 new tokens, ctx 104), fused RoPE + KV append +
decode attention (B = 256, ctx 121, QKV split-K partials), the batch-1 GEMV (gate_up, M = 1) and
the B = 256 tile GEMM (down projection, split-K 8) — for rocprofv3 --pmc."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

torch.manual_seed(0)
HQ, HKV, D, BS = 32, 8, 128, 16
NB = 6000
kc = torch.randn(NB, HKV, BS, D, device="cuda", dtype=torch.bfloat16)
vc = torch.randn(NB, HKV, D, BS, device="cuda", dtype=torch.bfloat16)

# prefill attention
S, QL, CTX = 256, 32, 104
q = torch.randn(S * QL, HQ, D, device="cuda", dtype=torch.bfloat16)
mb = (CTX + BS - 1) // BS
bt = torch.tensor([[j if j < 4 else 4 + s * (mb - 4) + (j - 4) for j in range(mb)] for s in range(S)],
                  dtype=torch.int32, device="cuda")
starts = torch.arange(0, S * QL + 1, QL, dtype=torch.int32, device="cuda")
ctx = torch.full((S,), CTX, dtype=torch.int32, device="cuda")
for _ in range(8):
    ops.attention_prefill(q, kc, vc, bt, starts, ctx, QL, D ** -0.5)

# fused decode attention, B = 256
B, C2 = 256, 121
mb2 = (C2 + BS - 1) // BS
bt2 = torch.tensor([[j if j < 4 else 4 + b * (mb2 - 4) + (j - 4) for j in range(mb2)] for b in range(B)],
                   dtype=torch.int32, device="cuda")
cl = torch.full((B,), C2, dtype=torch.int32, device="cuda")
pos = torch.full((B,), C2 - 1, dtype=torch.int32, device="cuda")
slots = (bt2[:, (C2 - 1) // BS] * BS + (C2 - 1) % BS).to(torch.int32).contiguous()
cos_sin = ops.rope_cos_sin(4096, D, 500000.0, device="cuda")
P = ops.SplitK(torch.randn(4, B, (HQ + 2 * HKV) * D, device="cuda") * 0.5, 4)
for _ in range(8):
    ops.decode_attention_rope(P, pos, cos_sin, slots, kc, vc, bt2, cl, HQ, HKV, D, D ** -0.5)

# batch-1 GEMV (gate_up) and B = 256 tile GEMM (down, split-K 8)
ws = [(torch.randn(28672, 4096, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(3)]
x1 = torch.randn(1, 4096, device="cuda", dtype=torch.bfloat16)
for i in range(8):
    ops.linear(x1, ws[i % 3], split=1)
wd = [(torch.randn(4096, 14336, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(3)]
x256 = torch.randn(256, 14336, device="cuda", dtype=torch.bfloat16)
for i in range(8):
    ops.linear_gm(x256, wd[i % 3], 4, 8, defer_reduce=True)
torch.cuda.synchronize()
print("done", flush=True)
