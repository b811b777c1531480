"""Single-pair forward timeline (diagnostic): run under rocprofv3 --kernel-trace,
then `python tools/single_pair_trace.py --summarize <run_kernel_trace.csv>`
prints per-kernel durations of one forward, the sum, the span and the gaps."""
import csv
import os
import sys

import numpy as np


def run(reps=30):
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from pointdsc_amd import kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    d = synthetic_batch(1, 1000, seed=7)
    c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    plan = kernels.ForwardPlan(m.pdsc_config(), m.packed_weights(), 1, 1000, dev)
    for _ in range(reps):
        plan.run(c, s, t)
    torch.cuda.synchronize(dev)


def summarize(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last forward: from the last pw_first launch on
    idx = [i for i, r in enumerate(rows) if "pw_first" in r["Kernel_Name"] or "pw2_first" in r["Kernel_Name"]]
    start = idx[-1] - 1  # the compat launch before it
    seg = rows[start:]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    tot = 0
    by = {}
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pdsc::", "")[:50]
        by.setdefault(name, []).append(d)
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:52s} x{len(v):3d} {np.mean(v):7.2f} us  {sum(v):7.1f} us")
    print(f"kernels {len(seg)}, sum {tot:.1f} us, span {(t1 - t0) / 1e3:.1f} us, gaps {(t1 - t0) / 1e3 - tot:.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
