#!/usr/bin/env python3
"""The kernel timeline of ONE single-pair forward from a rocprofv3 kernel trace
of tools/single_pair_run.py: the last forward's launches (it starts at the last
compat launch) with start offset, duration and the gap before each, plus totals
per kernel.  Usage: python tools/single_pair_timeline.py <kernel_trace.csv> [title]"""
import csv
import subprocess
import sys


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    names = sorted({r[2] for r in rows})
    try:
        dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
        dmap = dict(zip(names, dem))
    except OSError:
        dmap = {n: n for n in names}
    starts = [i for i, r in enumerate(rows) if "compat" in dmap[r[2]]]
    fwd = rows[starts[-1]:]
    t0 = fwd[0][0]
    print(f"# {title}: one forward, {len(fwd)} launches, span {(fwd[-1][1] - t0) / 1e3:.1f} us\n")
    print("| # | kernel | start us | dur us | gap us |")
    print("|---|---|---|---|---|")
    prev = t0
    busy, gaps, per = 0.0, 0.0, {}
    for i, (a, b, n) in enumerate(fwd):
        nm = dmap[n].split("(")[0]
        nm = nm if len(nm) < 70 else nm[:67] + "..."
        gap = (a - prev) / 1e3 if i else 0.0
        print(f"| {i} | `{nm}` | {(a - t0) / 1e3:.1f} | {(b - a) / 1e3:.2f} | {gap:.2f} |")
        busy += (b - a) / 1e3
        gaps += gap
        per.setdefault(nm, [0, 0.0])
        per[nm][0] += 1
        per[nm][1] += (b - a) / 1e3
        prev = b
    print(f"\nkernel time {busy:.1f} us, gaps {gaps:.1f} us\n")
    print("| kernel | launches | total us | avg us |")
    print("|---|---|---|---|")
    for nm, (c, tot) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{nm}` | {c} | {tot:.1f} | {tot / c:.2f} |")


if __name__ == "__main__":
    main()
