import sys, torch
sys.path.insert(0, "/root/repo")
from ai_agent_kubectl_amd.ops.autotune import tune_linear
from ai_agent_kubectl_amd.ops.autotune import _time
from ai_agent_kubectl_amd import ops
shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
groups = {s: [(torch.randn(*s, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(16)] for s in shapes}
rep = tune_linear(groups, [1, 2, 8])
for k, v in sorted(rep.items()):
    print(k, v)
# detail for O at M=1
x = torch.randn(1, 4096, device="cuda", dtype=torch.bfloat16)
ws = groups[(4096, 4096)]
for sp in (1, 2, 4, 8, 16):
    print("skinny O split", sp, round(_time(lambda w: ops.linear(x, w, split=sp), ws), 1))
print("blas O", round(_time(lambda w: torch.nn.functional.linear(x, w), ws), 1))
