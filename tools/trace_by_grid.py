"""Per-kernel average durations from a rocprofv3 kernel_trace.csv, split by grid
shape (a bench run mixes batched and single-pair launches of the same kernel).
Usage: python tools/trace_by_grid.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    agg = collections.defaultdict(list)
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g = f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
        agg[(r["Kernel_Name"][:60], g)].append(d)
    for (k, g), v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:top]:
        print(f"{k:60s} grid {g:>16s} n={len(v):4d} avg {sum(v) / len(v):9.2f} us  total {sum(v) / 1e3:8.3f} ms")


if __name__ == "__main__":
    main()
