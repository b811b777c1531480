#!/usr/bin/env python3
"""Where the fused tail's last launch (best_refine_kernel: select_best + the
post-refinement of models/PointDSC.py:403-438) spends its time for one pair:
s_memrealtime stamps (10 ns) of pair 0's workgroup from the diagnostic build
(make -C pointdsc_amd/csrc variant V=stamps VFLAGS=-DATT_STAMPS), per
iteration: the count pass (residuals + weights + block sums), the H pass (its
second residual pass + block sums) and the fp64 solve on one thread.
Usage: PDSC_LIB_VARIANT=stamps python tools/refine_stamps.py [N ...]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ST_PER_WAVE, ST_WGS = 256, 64


def one(N):
    from pointdsc_amd import _lib, kernels
    from pointdsc_amd.PointDSC import PointDSC
    from pointdsc_amd.synthetic import BENCH_CLS, PRESETS, synthetic_batch, trained_state_dict
    dev = torch.device("cuda:0")
    p = PRESETS["3dmatch"]
    m = PointDSC(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, ratio=0.1,
                 inlier_threshold=p["inlier_threshold"], sigma_d=p["sigma_d"], k=40, nms_radius=p["nms_radius"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in trained_state_dict("3dmatch", 12, *BENCH_CLS).items()})
    m = m.to(dev).eval()
    d = synthetic_batch(1, N, seed=7000)
    c, s, t = (torch.from_numpy(d[k]).to(dev) for k in ("corr_pos", "src_keypts", "tgt_keypts"))
    plan = kernels.ForwardPlan(m.pdsc_config(), m.packed_weights(), 1, N, dev)
    L = _lib.load()
    for _ in range(3):
        plan.run(c, s, t)
    torch.cuda.synchronize()
    reps = []
    for _ in range(5):
        assert L.pdsc_diag_nsm_stamps_clear() == 0
        plan.run(c, s, t)
        torch.cuda.synchronize()
        buf = np.zeros(ST_WGS * 4 * ST_PER_WAVE, np.uint64)
        assert L.pdsc_diag_nsm_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
        st = buf.reshape(ST_WGS * 4, ST_PER_WAVE)[-1].astype(np.int64)
        its = int(st[98])
        us = lambda a, b: float(st[b] - st[a]) / 100.0
        row = {"iterations": its, "total_us": us(0, 99), "select_us": us(0, 1), "count_pass_us": [], "h_pass_us": [],
               "solve_us": []}
        prev = 1
        for it in range(its):
            row["count_pass_us"].append(us(prev, 2 + 3 * it))
            if it + 1 < its or st[3 + 3 * it] > 0 and st[4 + 3 * it] > st[2 + 3 * it]:
                row["h_pass_us"].append(us(2 + 3 * it, 3 + 3 * it))
                row["solve_us"].append(us(3 + 3 * it, 4 + 3 * it))
                prev = 4 + 3 * it
        reps.append(row)
    return {"N": N, "runs": reps}


def main():
    Ns = [int(x) for x in sys.argv[1:]] or [1000, 5000]
    for N in Ns:
        print(json.dumps(one(N)), flush=True)


if __name__ == "__main__":
    main()
