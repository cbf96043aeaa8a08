"""Summarise the two PMC passes of scripts/gpu_pmc_gemm.sh (gpurun_out/pmc/*counter_collection.csv) as a
markdown table (profiles/pmc_gemm_m256_gate_up.md)."""
import collections
import csv
import sys

NAMES = {"Cijk": ("hipBLASLt MT128x256x64", 66.2),
         "gemm_tile_kernel<2, 2, 4, 4": ("tile cfg 2 (128x128, reg-staged, split 1)", 81.6),
         "gemm_tile_kernel<4, 2, 4, 8": ("tile cfg 15 (256x256, reg-staged, split 2)", 80.8),
         "gemm_stream_kernel<4, 2, 4, 8, 4, 2>": ("stream cfg 13 (256x256, LDS-DMA S=4, W nt, split 2)", 109.3),
         "gemm_stream_kernel<2, 4, 4, 4, 6, 0>": ("stream cfg 14 (128x256, LDS-DMA S=6, split 1)", 87.6)}


def main(d="gpurun_out/pmc"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in (f"{d}/p1_counter_collection.csv", f"{d}/p2_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            for k in NAMES:
                if k in r["Kernel_Name"]:
                    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("# PMC counters: M=256 gate_up GEMM (N=28672, K=4096) variants on one MI355X\n")
    print("`scripts/gpu_pmc_gemm.sh`: two `rocprofv3 --pmc` passes over `scripts/pmc_gemm.py` (16 dispatches per variant")
    print("on rotating weights; values averaged per dispatch).  Wall times: `profiles/gemm_stream_vs_tile_m256_m128.txt`.\n")
    print("| variant | wall us | GRBM_GUI_ACTIVE | SQ_WAVE_CYCLES | SQ_WAIT_INST_ANY / WAVE_CYCLES | TA_BUSY_avr | "
          "TCC_EA0_RDREQ | TCC_HIT | TD_TC_STALL | MFMA_BUSY |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for k, (label, us) in NAMES.items():
        v = {c: sum(x) / len(x) for c, x in agg[k].items()}
        print(f"| {label} | {us} | {v['GRBM_GUI_ACTIVE']:.3g} | {v['SQ_WAVE_CYCLES']:.3g} | "
              f"{100 * v['SQ_WAIT_INST_ANY'] / v['SQ_WAVE_CYCLES']:.0f} % | {v['TA_BUSY_avr']:.3g} | "
              f"{v['TCC_EA0_RDREQ_sum']:.3g} | {v['TCC_HIT_sum']:.3g} | {v['TD_TC_STALL_sum']:.3g} | "
              f"{v['SQ_VALU_MFMA_BUSY_CYCLES']:.3g} |")
    print("""
Reading: every variant issues the same MFMA work (SQ_VALU_MFMA_BUSY_CYCLES identical).  The memory-side request
count (TCC_EA0_RDREQ) shows hipBLASLt, cfg 14 and cfg 15 fetch the weights once, cfg 2 (two 128-row M tiles) ~1.6x,
and the non-temporal LDS-DMA loads of cfg 13 issue ~1.7x the requests for the same bytes — why `nt` lost in the
wall-time sweep (cfg 10 vs cfg 14).  The hand-written variants spend 42-54 % of wave time waiting on memory against
hipBLASLt's 33 %, with the texture address unit busier for the LDS-DMA kernels: at M = 256 the kernels are bound by
the per-CU load path (W from HBM plus the X panel re-read from L2 by every column tile plus split-K partials), not by
MFMA issue or prefetch depth; six LDS-DMA stages in flight did not move the wall time.  Decision: decode keeps the
per-shape autotuned choice (hipBLASLt for gate_up, the register-staged tile kernel for QKV / O / down).""")


if __name__ == "__main__":
    main(*sys.argv[1:])
