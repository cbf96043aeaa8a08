"""Every ring-kernel (csrc/gemm_mfma.hip) launch the persisted decode plan dispatches for Llama-3-8B,
under the launch pattern that exposed unordered LDS-DMA completion (each launch right after an
unrelated GEMM, every output checked against fp32), with and without the duplicate-address
amplifier (ldx = 0).  VERDICT r5 next #1; results: profiles/r6/lds_dma_safety/.

    python scripts/gm_plan_stress.py [--launches 500] [--buckets 128,...,512]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.ops import stress  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=500)
    ap.add_argument("--buckets", default="128,160,192,256,320,384,448,512")
    ap.add_argument("--amplifier", default="1,0")
    args = ap.parse_args()
    combos = stress.dispatched_combos(tuple(int(b) for b in args.buckets.split(",")))
    print(f"{len(combos)} dispatched (M, N, K, cfg, split, epi) combinations", flush=True)
    total = 0
    t0 = time.time()
    for amp in (int(a) for a in args.amplifier.split(",")):
        res = stress.stress(combos, args.launches, bool(amp), log=lambda s: print(s, flush=True))
        wrong = sum(res.values())
        total += wrong
        print(f"amplifier={amp}: {wrong} wrong launches in {len(combos) * args.launches} ({time.time() - t0:.0f} s)",
              flush=True)
    print(f"TOTAL wrong launches: {total}", flush=True)
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
