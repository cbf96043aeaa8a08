"""CPU contracts of the op layer's dispatch helpers (the GPU kernels are in test_kernels_gpu.py)."""
import torch

from ai_agent_kubectl_amd import ops
from ai_agent_kubectl_amd.ops import reference as ref


def test_linear_swiglu_cpu_is_reference():
    torch.manual_seed(0)
    x = torch.randn(9, 256, dtype=torch.bfloat16)
    w13 = (torch.randn(2 * 128, 256) / 16).to(torch.bfloat16)
    y = ops.linear_swiglu(x, w13)
    torch.testing.assert_close(y.float(), ref.silu_mul(ref.linear(x, w13)).float())
    assert not ops.use_prefill_swiglu(x, w13)   # CPU tensors never take the HIP path


def test_swiglu_gemm_shape_rules():
    x = torch.zeros(2048, 4096, dtype=torch.bfloat16)
    assert ops.swiglu_gemm_ok(x, torch.zeros(2 * 14336, 4096, dtype=torch.bfloat16))
    assert not ops.swiglu_gemm_ok(x, torch.zeros(2 * 14336 + 128, 4096, dtype=torch.bfloat16))
    assert not ops.swiglu_gemm_ok(x[:, :4000], torch.zeros(256, 4000, dtype=torch.bfloat16))
