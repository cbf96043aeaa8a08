"""Summarise a rocprofv3 `*_kernel_stats.csv` (--stats) into markdown: the top kernels and the share
of each kernel family (hand-written HIP by source file, hipBLASLt / rocBLAS `Cijk_*`, torch).

    python scripts/summarize_kernel_stats.py gpurun_out/<tag>/prof/run_kernel_stats.csv [--top 25]
"""
import argparse
import csv

FAMILIES = [
    ("decode_persistent.hip (batch-1 all-layers kernel)", ("pd::", "decode_layers_kernel", "zero_sync_kernel")),
    ("gemm_big.hip (prefill gate_up + SwiGLU, fused LM head)", ("gb::",)),
    ("gemm_mfma.hip (decode ring GEMMs)", ("gm::",)),
    ("gemm_skinny.hip (row GEMV / skinny)", ("gemv_rows", "gemm_skinny", "gemv_ring", "splitk_reduce")),
    ("attention.hip (paged decode / prefill attention)", ("paged_decode", "paged_prefill", "cascade_prefix",
                                                          "attention")),
    ("elementwise.hip (norms, RoPE + KV append, SiLU, embedding)", ("rmsnorm", "rope", "silu", "embedding",
                                                                    "kv_window")),
    ("sampling.hip (argmax / router)", ("argmax", "moe_topk")),
    ("moe.hip", ("moe_",)),
    ("allreduce.hip (one-shot collectives)", ("oneshot", "allreduce", "allgather")),
    ("hipBLASLt / rocBLAS (Cijk_*)", ("Cijk_",)),
    ("torch / runtime (weight init, copies, fills)", ("at::native", "__amd_rocclr", "elementwise_kernel")),
]


def family(name):
    for fam, keys in FAMILIES:
        if any(k in name for k in keys):
            return fam
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = {}
    for r in rows:
        f = family(r["Name"])
        fam[f] = fam.get(f, 0.0) + float(r["TotalDurationNs"])
    print(f"Total kernel time {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches.\n")
    print("| family | ms | share |\n|---|---|---|")
    for f, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"| {f} | {v / 1e6:.1f} | {100 * v / tot:.1f} % |")
    print(f"\n| kernel | calls | avg µs | total ms | share |\n|---|---|---|---|---|")
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:args.top]:
        name = r["Name"].replace("|", "/")
        name = name if len(name) <= 90 else name[:87] + "..."
        print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{float(r['TotalDurationNs']) / 1e6:.2f} | {100 * float(r['TotalDurationNs']) / tot:.1f} % |")


if __name__ == "__main__":
    main()
