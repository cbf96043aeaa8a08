"""Idle time between consecutive kernels in a rocprofv3 `--kernel-trace` CSV: how much of a decode step's
wall time is kernel boundaries rather than kernels.  Takes the last `--last` dispatches (the tail of a
graph-replay loop), sorts them by start time and reports busy time, total gap and the gap before each
kernel family.

    python scripts/trace_gaps.py <run_kernel_trace.csv> [--last 2000]
"""
import argparse
import csv
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=2000)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            try:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
            except (KeyError, ValueError):
                continue
    rows.sort()
    rows = rows[-args.last:]
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    gaps = defaultdict(list)
    total_gap = 0
    for (s0, e0, _), (s1, e1, n1) in zip(rows, rows[1:]):
        g = max(0, s1 - e0)
        total_gap += g
        gaps[n1.split("(")[0][:70]].append(g)
    print(f"{len(rows)} kernels over {span / 1e3:.1f} us: busy {busy / 1e3:.1f} us ({100 * busy / span:.1f} %), "
          f"gaps {total_gap / 1e3:.1f} us, mean gap {total_gap / max(1, len(rows) - 1) / 1e3:.2f} us")
    print("gap before each kernel family (us): count, median, mean, total")
    for n, g in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {len(g):6d} {statistics.median(g) / 1e3:7.2f} {statistics.mean(g) / 1e3:7.2f} {sum(g) / 1e3:9.1f}  {n}")


if __name__ == "__main__":
    main()
