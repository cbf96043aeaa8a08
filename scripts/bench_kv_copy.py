"""Paged-KV block copy (sub-block prefix reuse, csrc/elementwise.hip kv_block_copy_kernel): `pairs`
(src, dst) block pairs over the 32 layers of Llama-3-8B's cache, time per call.  Library from
KA_HIP_LIB (A/B against another build).

    python scripts/bench_kv_copy.py [--pairs 16,64,256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", default="16,64,256")
    args = ap.parse_args()
    L, NB, HKV, BS, D = 32, 1200, 8, 16, 128
    kc = torch.randn(L, NB, HKV, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(L, NB, HKV, D, BS, device="cuda", dtype=torch.bfloat16)
    for n in (int(p) for p in args.pairs.split(",")):
        perm = torch.randperm(NB)[:2 * n].to(torch.int32)
        src, dst = perm[:n].cuda(), perm[n:].cuda()
        for _ in range(3):
            ops.kv_block_copy(kc, vc, src, dst)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.kv_block_copy(kc, vc, src, dst)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        byts = 2 * 2 * n * L * HKV * BS * D * 2   # read + write, K and V
        print(f"{os.path.basename(os.path.dirname(os.environ.get('KA_HIP_LIB', 'in-tree/x')))} pairs={n}: "
              f"{us:7.1f} us ({byts / us / 1e6:4.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
