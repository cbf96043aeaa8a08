"""GPU busy/idle analysis of a rocprofv3 kernel trace (run on the GPU box next to the trace).

Unions the kernel intervals over the last `--window` seconds of the trace (the timed region of a
bench run) and prints the busy fraction, the idle time split by gap size, and the largest gaps with
the kernels on either side — i.e. where the device waits on the host.

  python scripts/trace_busy.py /tmp/ka_prof [--window 2.0] > gpurun_out/trace_busy.txt
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--window", type=float, default=2.0)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {a.root}")
    ev = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    ev.sort()
    t_end = max(e[1] for e in ev)
    t0 = t_end - int(a.window * 1e9)
    ev = [e for e in ev if e[1] > t0]
    busy = 0
    gaps = []
    cur_s, cur_e, prev_name = ev[0][0], ev[0][1], ev[0][2]
    for s, e, name in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = name if e >= cur_e else prev_name
    busy += cur_e - cur_s
    span = t_end - max(t0, ev[0][0])
    print(f"window {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f}%)  "
          f"idle {(span - busy) / 1e6:.1f} ms in {len(gaps)} gaps  kernels {len(ev)}")
    for lo, hi in ((0, 5e3), (5e3, 20e3), (20e3, 100e3), (100e3, 1e6), (1e6, 1e12)):
        g = [x for x in gaps if lo <= x[0] < hi]
        print(f"  gaps {lo / 1e3:7.0f}-{hi / 1e3:7.0f} us: n={len(g):6d}  total {sum(x[0] for x in g) / 1e6:8.2f} ms")
    print("largest gaps:")
    for d, before, after in sorted(gaps, reverse=True)[:25]:
        print(f"  {d / 1e3:9.1f} us  after {before!r:72}  before {after!r}")


if __name__ == "__main__":
    main()
