#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_summary.md, the raw
rocprofv3 kernel_stats.csv, and profiles/<tag>_traffic.json.

A bench run launches the same kernel at several shapes (the batched headline
forward, the N=5000 path forward, single-pair forwards), so every row is keyed
by (kernel, grid size): the per-grid average is what bench.py's HIP-event
launch time must agree with.

HBM counters (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KB
(1024 B) per dispatch from separate --pmc passes.  On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so `hbm_bytes` =
2 x FETCH_SIZE + WRITE_SIZE (the read correction is exact for 16-B/lane
streams and an upper bound for narrower reads).

Usage: python tools/summarize_profile.py <tag> [gpurun_out/prof_<tag>]
"""
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def demangle(names):
    names = sorted(set(names))
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                             check=True).stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        out = names
    res = {}
    for n, d in zip(names, out):
        if d.startswith("_Z"):  # binutils' c++filt predates _Float16 (DF16_) mangling
            m = re.match(r"_ZN4pdsc(\d+)", d)
            if m:
                ln = int(m.group(1))
                base = d[m.end():m.end() + ln]
                targs = re.match(r"IL[ib](\d+)E", d[m.end() + ln:])
                d = base + (f"<{targs.group(1)}>" if targs else "")
        res[n] = d.split("(")[0].replace("pdsc::", "").replace("void ", "")
    return res


def main(tag, src=None):
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    trace = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    pmc_rows = []
    for p in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
        pmc_rows += list(csv.DictReader(open(p)))
    dm = demangle([r["Kernel_Name"] for r in trace] + [r["Kernel_Name"] for r in pmc_rows])

    dur = defaultdict(list)
    for r in trace:
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        dur[(dm[r["Kernel_Name"]], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = defaultdict(lambda: defaultdict(list))
    for r in pmc_rows:
        pmc[(dm[r["Kernel_Name"]], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    extra = sorted({c for k in pmc.values() for c in k} - {"FETCH_SIZE", "WRITE_SIZE"})

    def mean(v):
        return sum(v) / len(v) if v else float("nan")

    keys = sorted(dur, key=lambda k: -sum(dur[k]))
    lines = [f"# rocprofv3 summary `{tag}`", "",
             "`rocprofv3 --kernel-trace --stats` of `bench.py` (tools/profile.sh) plus separate `--pmc` "
             "passes of the same command.  Rows are (kernel, grid threads): one bench run launches each "
             "kernel at the headline shape and at the N=5000 path / single-pair shapes.  FETCH/WRITE in "
             "KB (1024 B) per dispatch; `HBM MB` = (2 x FETCH + WRITE) x 1024 B (gfx950 FETCH_SIZE "
             "under-counts wide reads by 2x, MI355X_MICROARCH.md §HBM).", "",
             "| kernel | grid threads | calls | avg us | total ms | FETCH KB | WRITE KB | HBM MB/dispatch |",
             "|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for k in keys:
        name, g = k
        f, w = mean(pmc[k]["FETCH_SIZE"]), mean(pmc[k]["WRITE_SIZE"])
        hbm = (2 * f + w) * 1024
        lines.append(f"| {name} | {g} | {len(dur[k])} | {mean(dur[k]):.2f} | {sum(dur[k]) / 1e3:.3f} | "
                     f"{f:.0f} | {w:.0f} | {hbm / 1e6:.1f} |")
        traffic.setdefault(name, {})[str(g)] = {
            "calls": len(dur[k]), "avg_us": round(mean(dur[k]), 3),
            "fetch_kb": None if f != f else round(f, 1), "write_kb": None if w != w else round(w, 1),
            "hbm_bytes": None if hbm != hbm else round(hbm)}
    if extra:
        lines += ["", "Other counters (mean per dispatch):", "",
                  "| kernel | grid | " + " | ".join(extra) + " |", "|---|---|" + "---|" * len(extra)]
        for k in keys:
            vals = [mean(pmc[k][c]) for c in extra]
            lines.append(f"| {k[0]} | {k[1]} | " + " | ".join(f"{v:.4g}" for v in vals) + " |")
            for c, v in zip(extra, vals):
                if v == v:
                    traffic[k[0]][str(k[1])][c] = v
    need = {"SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES",
            "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"}
    if need <= set(extra):
        # Derived (MI355X_MICROARCH.md constants table): SQ_BUSY_CYCLES summed over the
        # 32 shader engines gives the effective clock over the dispatch; MFMA-busy
        # cycles over (1024 SIMDs x those cycles) = the matrix pipes' busy fraction;
        # SQ_WAIT_* and SQ_WAVE_CYCLES are both quad-cycle counts (their ratio is exact).
        lines += ["", "Derived per dispatch (kernels >= 20 us): effective clock = SQ_BUSY_CYCLES / 32 SEs / "
                  "duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock x duration); "
                  "waits as fractions of SQ_WAVE_CYCLES.", "",
                  "| kernel | grid | avg us | clock GHz | MFMA busy | VALU/MFMA instr | WAIT_ANY | WAIT_INST_ANY |",
                  "|---|---|---|---|---|---|---|---|"]
        for k in keys:
            d = mean(dur[k])
            if not d >= 20.0:
                continue
            m = {c: mean(pmc[k][c]) for c in need}
            if any(v != v for v in m.values()):
                continue
            cyc = m["SQ_BUSY_CYCLES"] / 32.0
            clk = cyc / (d * 1e3)
            busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc) if cyc > 0 else float("nan")
            ratio = m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"] if m["SQ_INSTS_MFMA"] > 0 else float("nan")
            wc = m["SQ_WAVE_CYCLES"]
            lines.append(f"| {k[0]} | {k[1]} | {d:.1f} | {clk:.2f} | {busy:.3f} | {ratio:.2f} | "
                         f"{m['SQ_WAIT_ANY'] / wc:.2f} | {m['SQ_WAIT_INST_ANY'] / wc:.2f} |")
    open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump({"tag": tag, "kernels": traffic}, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
