"""Prefill attention microbenchmark: 256 sequences x 32 new tokens over a 104-token context with a
shared 64-token prefix (the bench's prefill step), Llama-3-8B heads, 32 layers of cold caches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402

S, QL, CTX, HQ, HKV, D, BS = 256, 32, 104, 32, 8, 128, 16
NB = 6000
kc = torch.randn(32, NB, HKV, BS, D, device="cuda", dtype=torch.bfloat16)
vc = torch.randn(32, NB, HKV, D, BS, device="cuda", dtype=torch.bfloat16)
q = torch.randn(S * QL, HQ, D, device="cuda", dtype=torch.bfloat16)
mb = (CTX + BS - 1) // BS
bt = torch.zeros(S, mb, dtype=torch.int32)
nxt = 4
for s in range(S):
    for j in range(mb):
        bt[s, j] = j if j < 4 else nxt
        nxt += j >= 4
bt = bt.cuda()
starts = torch.arange(0, S * QL + 1, QL, dtype=torch.int32, device="cuda")
ctx = torch.full((S,), CTX, dtype=torch.int32, device="cuda")
for i in range(3):
    ops.attention_prefill(q, kc[i], vc[i], bt, starts, ctx, QL, D ** -0.5)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(32):
    ops.attention_prefill(q, kc[i], vc[i], bt, starts, ctx, QL, D ** -0.5)
e1.record()
torch.cuda.synchronize()
print(f"prefill attention S={S} qlen={QL} ctx={CTX}: {e0.elapsed_time(e1) / 32 * 1e3:.1f} us/layer", flush=True)
