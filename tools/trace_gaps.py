"""Per-kernel busy time and the idle gaps between consecutive dispatches of a rocprofv3 kernel trace.

usage: python tools/trace_gaps.py <kernel_trace.csv> [--match SUBSTR] [--after SUBSTR]

Reads the trace rocprofv3 --kernel-trace writes (Kernel_Name, Start_Timestamp, End_Timestamp), keeps
the dispatches from the first one whose name contains --after (default: all), and prints per kernel
name: launches, average duration, and the average idle gap before it (end of the previous dispatch
to its start).  The gap is what a kernel boundary costs on the critical path.
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--after", default=None, help="start at the first dispatch whose name contains this")
    ap.add_argument("--until", default=None, help="stop before the first later dispatch containing this")
    ap.add_argument("--skip-short", type=float, default=0.0, help="drop dispatches shorter than this (us)")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if a.after:
        i = next(i for i, r in enumerate(rows) if a.after in r[2])
        rows = rows[i:]
    if a.until:
        j = next((j for j, r in enumerate(rows) if j > 0 and a.until in r[2]), len(rows))
        rows = rows[:j]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for s, e, name in rows:
        short = name.split("(")[0][:60]
        if (e - s) / 1e3 < a.skip_short:
            continue
        dur[short].append((e - s) / 1e3)
        if prev_end is not None:
            gap[short].append((s - prev_end) / 1e3)
        prev_end = e
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(sum(v) for v in dur.values())
    print(f"span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us, dispatches {len(rows)}")
    print(f"{'kernel':60s} {'n':>6s} {'avg us':>9s} {'sum us':>10s} {'gap avg':>8s} {'gap sum':>9s}")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        g = gap.get(k, [])
        print(f"{k:60s} {len(dur[k]):6d} {sum(dur[k]) / len(dur[k]):9.2f} {sum(dur[k]):10.1f} "
              f"{(sum(g) / len(g) if g else 0):8.2f} {sum(g):9.1f}")


if __name__ == "__main__":
    main()
