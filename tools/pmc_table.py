#!/usr/bin/env python3
"""Per-kernel averages of a tools/prof_bin.sh run (diagnostics): duration from the
kernel trace, every collected counter per dispatch, and the derived effective
clock (SQ_BUSY_CYCLES / 32 SEs / duration), MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES /
(1024 SIMDs x clock x duration)) and wait fractions of SQ_WAVE_CYCLES.
Usage: python tools/pmc_table.py gpurun_out/pb_<tag> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
dur = defaultdict(list)
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
    if flt in r["Kernel_Name"]:
        dur[(r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "")))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
ctr = defaultdict(lambda: defaultdict(list))
for p in glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        if flt in r["Kernel_Name"]:
            key = (r["Kernel_Name"], r.get("Grid_Size", ""))
            ctr[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key in sorted(dur):
    name = key[0].split("(")[0][-60:]
    d = sorted(dur[key])[len(dur[key]) // 2]
    c = {k: sum(v) / len(v) for k, v in ctr.get(key, {}).items()}
    print(f"{name}  grid {key[1]}  {d:.1f} us (median of {len(dur[key])})")
    for k, v in sorted(c.items()):
        print(f"    {k:28s} {v:.4g}")
    if "SQ_BUSY_CYCLES" in c:
        clk = c["SQ_BUSY_CYCLES"] / 32 / (d * 1e-6)
        print(f"    effective clock              {clk / 1e9:.2f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            print(f"    MFMA busy                    {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * clk * d * 1e-6):.3f}")
    if "GRBM_GUI_ACTIVE" in c:
        print(f"    GRBM clock                   {c['GRBM_GUI_ACTIVE'] / 8 / (d * 1e-6) / 1e9:.2f} GHz")
    if "SQ_WAVE_CYCLES" in c:
        for w in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if w in c:
                print(f"    {w + ' frac':28s} {c[w] / c['SQ_WAVE_CYCLES']:.3f}")
