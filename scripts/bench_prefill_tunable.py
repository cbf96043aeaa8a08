"""Prefill GEMM: hipBLASLt default heuristic vs TunableOp's best solution (rotating buffer) for the
Llama-3-8B projection shapes at prefill M (whole 256-row tiles).  Prints us and PFLOP/s."""
import os
import sys

import torch

SHAPES = [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")]
Ms = [int(a) for a in sys.argv[1:]] or [4096, 8192]


def t_us(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    torch.manual_seed(0)
    res = {}
    for M in Ms:
        for N, K, name in SHAPES:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
            res[(M, name)] = [t_us(lambda: torch.nn.functional.linear(x, w))]
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(os.path.join(os.environ.get("OUT", "gpurun_out"), "tunable_prefill.csv"))
    tun.set_max_tuning_duration(200)
    tun.set_rotating_buffer_size(512)
    for M in Ms:
        for N, K, name in SHAPES:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
            torch.nn.functional.linear(x, w)   # tunes
            tun.tuning_enable(False)
            res[(M, name)].append(t_us(lambda: torch.nn.functional.linear(x, w)))
            tun.tuning_enable(True)
            fl = 2 * M * N * K
            a, b = res[(M, name)]
            print(f"M={M:5d} {name:8s} default {a:8.1f} us ({fl / a / 1e9:5.2f} PF)  tuned {b:8.1f} us "
                  f"({fl / b / 1e9:5.2f} PF)  {a / b:5.3f}x", flush=True)
    tun.write_file()


if __name__ == "__main__":
    main()
