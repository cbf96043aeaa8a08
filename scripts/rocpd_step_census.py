"""Per-step kernel census of the last N decode-graph replays in a rocprofv3 rocpd database.

    python scripts/rocpd_step_census.py run_results.db [--steps 40] [--delim argmax_finish_kernel]

Steps are delimited by the step's last kernel (default: the argmax finish); prints, per kernel name and
grid, the mean count and microseconds per step, and the step's total busy time.
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--delim", default="argmax_finish_kernel")
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    rows = list(con.execute("select name, start, end, grid_x, workgroup_x from kernels order by start"))
    ends = [i for i, r in enumerate(rows) if r[0].startswith(args.delim)]
    ends = ends[-(args.steps + 1):]
    sel = rows[ends[0] + 1: ends[-1] + 1]
    n = len(ends) - 1
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e, gx, wx in sel:
        key = (name.split("(")[0][:90], gx // max(wx, 1))
        agg[key][0] += 1
        agg[key][1] += (e - s) / 1e3
    busy = sum(v[1] for v in agg.values()) / n
    wall = (sel[-1][2] - sel[0][1]) / 1e3 / n
    print(f"{n} steps: busy {busy:.1f} us/step, wall {wall:.1f} us/step")
    for (name, wg), (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{us / n:9.1f} us  {c / n:6.1f}x  wg {wg:6d}  {us / c:8.2f} us each  {name}")


if __name__ == "__main__":
    main()
