#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_summary.md (+ copies of
the rocprofv3 kernel_stats.csv).  FETCH_SIZE / WRITE_SIZE are rocprofv3's KB
per dispatch; per MI355X_MICROARCH.md §HBM, FETCH_SIZE under-reports wide
coalesced streaming reads by 2x on gfx950, so `hbm_read_corrected` = 2 x
FETCH_SIZE is an upper-bound correction (exact only for 16-B/lane streams).

Usage: python tools/summarize_profile.py <tag> [gpurun_out/prof_<tag>]
"""
import csv
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0]
    return n.replace("pdsc::", "")


def main(tag, src=None):
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    pmc = defaultdict(lambda: defaultdict(list))
    import glob
    for p in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    extra = sorted({c for k in pmc.values() for c in k} - {"FETCH_SIZE", "WRITE_SIZE"})
    lines = [f"# rocprofv3 summary `{tag}`", "",
             "Kernel-trace stats (`rocprofv3 --kernel-trace --stats`) and per-dispatch HBM counters "
             "from separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of the same command "
             "(see tools/profile.sh).  KB = rocprofv3 units (1024 B).", "",
             "| kernel | calls | avg us | total ms | % | FETCH_SIZE KB/dispatch | 2x FETCH (corr.) MB | WRITE_SIZE KB/dispatch |",
             "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        k = short(r["Name"])
        f = pmc[k]["FETCH_SIZE"]
        w = pmc[k]["WRITE_SIZE"]
        fa = sum(f) / len(f) if f else float("nan")
        wa = sum(w) / len(w) if w else float("nan")
        lines.append(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} | "
                     f"{fa:.0f} | {2 * fa * 1024 / 1e6:.1f} | {wa:.0f} |")
    if extra:
        lines += ["", "Other counters (mean per dispatch):", "",
                  "| kernel | " + " | ".join(extra) + " |", "|---|" + "---|" * len(extra)]
        for r in rows:
            k = short(r["Name"])
            vals = [sum(pmc[k][c]) / len(pmc[k][c]) if pmc[k][c] else float("nan") for c in extra]
            lines.append(f"| {k} | " + " | ".join(f"{v:.4g}" for v in vals) + " |")
    out = os.path.join(dst, f"{tag}_summary.md")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
