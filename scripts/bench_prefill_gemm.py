"""Prefill GEMM microbenchmark: hipBLASLt heuristic vs TunableOp (cold, rotating weights) at ragged
and 256-padded token counts, for the Llama-3-8B projection shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.ops.autotune import _time  # noqa: E402

SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]


def run(Ms, label):
    for M in Ms:
        tot, fl = 0.0, 0
        row = []
        for N, K in SHAPES:
            ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(4)]
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            t = _time(lambda w: torch.nn.functional.linear(x, w), ws, reps=8)
            tot += t
            fl += 2 * M * N * K
            row.append(f"{N}x{K}:{t:.0f}us")
            del ws
        print(f"{label} M={M:5d} layer {tot:8.1f} us  {fl / tot / 1e6:6.0f} TF  " + " ".join(row), flush=True)


run([4000, 4096, 8035, 8192], "heuristic")
tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(200)
tun.set_rotating_buffer_size(1024)
tun.set_filename("/tmp/tunableop_prefill.csv")
run([4096, 8192], "tuning  ")
tun.tuning_enable(False)
run([4096, 8192], "tuned   ")
